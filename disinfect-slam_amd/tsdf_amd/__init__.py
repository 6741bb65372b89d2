"""tsdf_amd -- Python host mirror of the reference TSDF interface over the MI355X C ABI.

Reference interface mirrored (yuzhou42/disinfect-slam):
  * TSDFGrid            utils/tsdf/voxel_tsdf.cuh:32-124  (Integrate / RayCast / GatherValid /
                        GatherVoxels) -- here `TSDFGrid`, same argument meaning and order;
  * CameraIntrinsics    utils/cuda/camera.cuh:12-51, CameraParams :53-68
  * SE3                 utils/cuda/lie_group.cuh:6-45
  * BoundingCube        utils/tsdf/voxel_tsdf.cuh:12-27
  * VoxelSpatialTSDF    utils/tsdf/voxel_types.cuh:48-57 (numpy structured dtype VOXEL_DTYPE)
The C++17 facade (TSDFSystem / TSDFGrid / DISINFSystem TSDF methods) lives in ../host/.
Frames may be numpy arrays (host, copied by the engine) or torch CUDA tensors (device, no copy).
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from . import _lib
from ._lib import (SHARD_RECORD_BYTES, STATUS_DDA_OVERFLOW, STATUS_NEWKEY_OVERFLOW,
                   STATUS_PIPELINE_TIMEOUT, STATUS_POOL_EXHAUSTED, STATUS_SHARD_ABORTED, STATUS_SHARD_OVERFLOW, TSDF_MEM_DEVICE,
                   TSDF_MEM_HOST, TSDFError)

NUM_ENTRY = 1 << 22
NUM_BUCKET = 1 << 21
BLOCK_LEN = 8
BLOCK_VOLUME = 512
BLOCK_RECORD_BYTES = 16 + 12 * BLOCK_VOLUME  # TSDF_BLOCK_RECORD_BYTES: key header + block
VOXEL_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("tsdf", "<f4")])

__all__ = [
    "CameraIntrinsics", "CameraParams", "SE3", "BoundingCube", "TSDFGrid", "Engine", "ShardGroup",
    "VOXEL_DTYPE", "TSDFError", "hash_block", "block_owner", "load_library", "FOREIGN_IDX",
    "STATUS_SHARD_ABORTED",
    "STATUS_PIPELINE_TIMEOUT",
]
FOREIGN_IDX = 0x7FFFFFFF  # a shard's index entry of a block another shard holds (kForeignIdx)


def load_library():
    return _lib.load()


def hash_block(x: int, y: int, z: int) -> int:
    """voxel_hash.cu:31-35 Hash."""
    return int(_lib.load().tsdf_hash_block(x, y, z))


def block_owner(x: int, y: int, z: int, shard_count: int) -> int:
    return int(_lib.load().tsdf_block_owner(x, y, z, shard_count))


@dataclasses.dataclass(frozen=True)
class CameraIntrinsics:
    """camera.cuh:12-51 CameraIntrinsics<float>."""
    fx: float
    fy: float
    cx: float
    cy: float

    def Inverse(self) -> "CameraIntrinsics":
        f32 = np.float32
        fx_inv = f32(1) / f32(self.fx)
        fy_inv = f32(1) / f32(self.fy)
        return CameraIntrinsics(float(fx_inv), float(fy_inv), float(-f32(self.cx) * fx_inv),
                                float(-f32(self.cy) * fy_inv))

    def _c(self) -> _lib.Intrinsics:
        c = self.__dict__.get("_cc")
        if c is None:  # frozen dataclass: cache the ctypes struct once
            c = _lib.Intrinsics(self.fx, self.fy, self.cx, self.cy)
            object.__setattr__(self, "_cc", c)
        return c


@dataclasses.dataclass(frozen=True)
class CameraParams:
    """camera.cuh:53-68 CameraParams(intrinsics, img_h, img_w)."""
    intrinsics: CameraIntrinsics
    img_h: int
    img_w: int


def _qmul_sse(a, b):
    """Eigen quat_product<SSE, float> (host Eigen, Geometry/arch/Geometry_SSE.h)."""
    f32 = np.float32
    a0, a1, a2, a3 = (f32(v) for v in a)
    b0, b1, b2, b3 = (f32(v) for v in b)
    x = (a0 * b3 - a2 * b1) + (a1 * b2 + a3 * b0)
    y = (a1 * b3 - a0 * b2) + (a2 * b0 + a3 * b1)
    z = (a2 * b3 - a1 * b0) + (a0 * b1 + a3 * b2)
    w = (a3 * b3 - a0 * b0) - (a2 * b2 + a1 * b1)
    return np.array([x, y, z, w], np.float32)


def _qrot(q, v):
    """Eigen QuaternionBase::_transformVector."""
    f32 = np.float32
    qx, qy, qz, qw = (f32(c) for c in q)
    vx, vy, vz = (f32(c) for c in v)
    ux = qy * vz - qz * vy
    uy = qz * vx - qx * vz
    uz = qx * vy - qy * vx
    ux, uy, uz = ux + ux, uy + uy, uz + uz
    cx = qy * uz - qz * uy
    cy = qz * ux - qx * uz
    cz = qx * uy - qy * ux
    return np.array([(vx + qw * ux) + cx, (vy + qw * uy) + cy, (vz + qw * uz) + cz], np.float32)


class SE3:
    """lie_group.cuh:6-45 SE3<float>: rotation quaternion (x, y, z, w) + translation."""

    def __init__(self, q_xyzw=(0.0, 0.0, 0.0, 1.0), t=(0.0, 0.0, 0.0)):
        self.q = np.asarray(q_xyzw, dtype=np.float32).reshape(4).copy()
        self.t = np.asarray(t, dtype=np.float32).reshape(3).copy()

    @staticmethod
    def Identity() -> "SE3":
        return SE3()

    def GetR(self):
        return self.q.copy()

    def GetT(self):
        return self.t.copy()

    def Inverse(self) -> "SE3":
        f32 = np.float32
        x, y, z, w = (f32(c) for c in self.q)
        n2 = (x * x + z * z) + (y * y + w * w)
        qi = np.array([-x / n2, -y / n2, -z / n2, w / n2], np.float32) if n2 > 0 else np.zeros(4, np.float32)
        return SE3(qi, _qrot(qi, -self.t))

    def Apply(self, v):
        return (_qrot(self.q, v) + self.t).astype(np.float32)

    def __mul__(self, other: "SE3") -> "SE3":
        return SE3(_qmul_sse(self.q, other.q), _qrot(self.q, other.t) + self.t)

    def _c(self) -> _lib.Pose:
        c = self.__dict__.get("_cc")
        if c is None:  # SE3 is treated as immutable: cache the ctypes struct once
            c = _lib.Pose(*[float(v) for v in self.q], *[float(v) for v in self.t])
            self._cc = c
        return c


@dataclasses.dataclass(frozen=True)
class BoundingCube:
    """voxel_tsdf.cuh:12-27 BoundingCube<float>."""
    xmin: float
    xmax: float
    ymin: float
    ymax: float
    zmin: float
    zmax: float

    def as_array(self):
        return np.array([self.xmin, self.xmax, self.ymin, self.ymax, self.zmin, self.zmax], np.float32)


def _is_torch_cuda(x) -> bool:
    return hasattr(x, "data_ptr") and hasattr(x, "is_cuda") and bool(x.is_cuda)


_raw_stream = None


def _current_raw_stream(device: int) -> int:
    """torch's current stream on `device` as a raw hipStream_t (the cheap accessor when this torch has
    it: torch.cuda.current_stream() builds a Stream object per call)."""
    global _raw_stream
    if _raw_stream is None:
        import torch
        f = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        _raw_stream = f if f is not None else (lambda d: torch.cuda.current_stream(d).cuda_stream)
    return int(_raw_stream(device) or 0)


def _ptr(x):
    if x is None:
        return None
    if _is_torch_cuda(x):
        return C.c_void_p(x.data_ptr())
    return x.ctypes.data_as(C.c_void_p)


def _np(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)



class FrameGraph:
    """One instantiated per-frame hipGraph of an Engine (tsdf_graph_create). frame() takes device
    tensors only; rgba / normal are device tensors (render_height, render_width, 4) u8 or None."""

    def __init__(self, eng, width, height, render_width=0, render_height=0, deferred=False, batch=1):
        self._eng = eng
        self.width, self.height = width, height
        self.render_width, self.render_height = render_width, render_height
        h = C.c_void_p()
        if batch > 1:  # tsdf_graph_create_batch: `batch` frames per graph launch
            _lib.check(_lib.load().tsdf_graph_create_batch(eng._h, width, height, render_width, render_height,
                                                           int(deferred), batch, C.byref(h)), "tsdf_graph_create_batch")
        else:
            fn = "tsdf_graph_create_deferred" if deferred else "tsdf_graph_create"
            _lib.check(getattr(_lib.load(), fn)(eng._h, width, height, render_width, render_height, C.byref(h)), fn)
        self.batch = batch
        self._g = h
        self.deferred = deferred

    def frame(self, rgb, depth, ht, lt, K, cam_T_world, max_depth, render_K=None,
              render_cam_T_world=None, rgba=None, normal=None):
        for a in (rgb, depth, ht, lt, rgba, normal):
            if a is not None and (not _is_torch_cuda(a) or not a.is_contiguous()):
                raise ValueError("graph frames take contiguous device tensors")
        H, W = int(depth.shape[0]), int(depth.shape[1])
        fr = _lib.Frame(W, H, _ptr(rgb), _ptr(depth), _ptr(ht), _ptr(lt), TSDF_MEM_DEVICE)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        Rk = None
        if render_K is not None:
            Rk = render_K._c() if isinstance(render_K, CameraIntrinsics) else \
                _lib.Intrinsics(*[float(v) for v in render_K])
        self._eng._wait_torch(depth)
        prev = self._eng._pending
        _lib.check(_lib.load().tsdf_graph_frame(
            self._g, C.byref(fr), C.byref(Kc), C.byref(cam_T_world._c()), max_depth,
            C.byref(Rk) if Rk is not None else None,
            C.byref(render_cam_T_world._c()) if render_cam_T_world is not None else None,
            _ptr(rgba), _ptr(normal)), "tsdf_graph_frame")
        self._eng._signal_torch(depth)
        if self.batch > 1:
            # a batched graph writes a frame's images when its batch launches (full, or at the engine's
            # next other call): every image of the unlaunched frames stays referenced until such a call
            if rgba is not None or normal is not None:
                self._eng._pending = (prev or ()) + (rgba, normal)
            return
        self._eng._after_call(prev)
        if self.deferred and (rgba is not None or normal is not None):
            self._eng._pending = (rgba, normal)  # written by the next launch (or engine call)

    def close(self):
        if getattr(self, "_g", None):
            _lib.load().tsdf_graph_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

class ShardFrameGraph:
    """A shard engine's graph-captured sharded frame (tsdf_graph_create_shard): begin / update / end
    as three graph launches around the caller's two exchanges. Device frames and device slots."""

    def __init__(self, eng, width, height, slice_index=0, slice_count=1):
        self._eng = eng
        self.width, self.height = width, height
        self.split = slice_count > 1
        h = C.c_void_p()
        _lib.check(_lib.load().tsdf_graph_create_shard(eng._h, width, height, slice_index, slice_count,
                                                       C.byref(h)), "tsdf_graph_create_shard")
        self._g = h

    def begin(self, rgb, depth, ht, lt, K, cam_T_world, max_depth, keys_out, keys_in, key_cap, cands_out,
              cands_in, cand_cap):
        for a in (rgb, depth, ht, lt, keys_out, keys_in, cands_out, cands_in):
            if a is not None and (not _is_torch_cuda(a) or not a.is_contiguous()):
                raise ValueError("shard graph frames take contiguous device tensors")
        H, W = int(depth.shape[0]), int(depth.shape[1])
        fr = _lib.Frame(W, H, _ptr(rgb), _ptr(depth), _ptr(ht), _ptr(lt), TSDF_MEM_DEVICE)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        self._eng._wait_torch(depth, keys_out, cands_out)
        _lib.check(_lib.load().tsdf_graph_shard_begin(
            self._g, C.byref(fr), C.byref(Kc), C.byref(cam_T_world._c()), max_depth, _ptr(keys_out),
            _ptr(keys_in), key_cap, _ptr(cands_out), _ptr(cands_in), cand_cap), "tsdf_graph_shard_begin")
        self._eng._signal_torch(keys_out)
        self._frame = (rgb, depth, ht, lt)  # read again by the update segment (see Engine.integrate_shard_begin)

    def update(self, keys_in=None, cands_out=None):
        self._eng._wait_torch(keys_in)
        _lib.check(_lib.load().tsdf_graph_shard_update(self._g), "tsdf_graph_shard_update")
        keep, self._frame = getattr(self, "_frame", None) or (), None
        self._eng._signal_torch(cands_out, *keep)

    def end(self, cands_in=None):
        self._eng._wait_torch(cands_in)
        _lib.check(_lib.load().tsdf_graph_shard_end(self._g), "tsdf_graph_shard_end")
        self._eng._signal_torch(cands_in)

    def close(self):
        if getattr(self, "_g", None):
            _lib.load().tsdf_graph_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One MI355X TSDF volume (one GPU shard). Thin owner of a tsdf_engine* handle."""

    def __init__(self, voxel_size=0.005, truncation=0.03, max_width=1920, max_height=1080,
                 num_block_bits=18, device=0, shard_index=0, shard_count=1, stream=None):
        L = _lib.load()
        cfg = _lib.Config()
        L.tsdf_config_default(C.byref(cfg))
        cfg.voxel_size = voxel_size
        cfg.truncation = truncation
        cfg.max_width = max_width
        cfg.max_height = max_height
        cfg.num_block_bits = num_block_bits
        cfg.shard_index = shard_index
        cfg.shard_count = shard_count
        if stream is not None:  # a torch.cuda.Stream or a raw hipStream_t (0 = the legacy default stream)
            cfg.stream = C.c_void_p(int(getattr(stream, "cuda_stream", getattr(stream, "value", stream)) or 0))
            cfg.use_stream = 1
        h = C.c_void_p()
        _lib.check(L.tsdf_create(C.byref(cfg), device, C.byref(h)), "tsdf_create")
        self._h = h
        # the engine orders its stream after / before torch's current stream around every call that
        # reads / writes a torch device tensor (tsdf_stream_wait / _signal) whenever the two differ
        # (an engine-owned stream, or a caller's stream other than torch's current one)
        es = C.c_void_p()
        _lib.check(L.tsdf_get_stream(h, C.byref(es)), "tsdf_get_stream")
        self._stream = int(es.value or 0)
        self.voxel_size = voxel_size
        self.truncation = truncation
        self.num_blocks = int(L.tsdf_num_blocks(h))
        self.device = device
        self.shard_index = shard_index
        self.shard_count = shard_count
        # device images of a deferred raycast (raycast(deferred=True), deferred graph frames) that the
        # engine's NEXT call writes: referenced until then (torch's allocator must not reuse them), and
        # torch's current stream is ordered after that call -- see _after_call
        self._pending = None

    def _after_call(self, prev):
        """Engine call wrapper epilogue: the call launched the deferred raycast `prev` was waiting for
        (every engine entry point does, tsdf_raycast_deferred included), so torch's current stream now
        waits for the engine's queued work -- the images may be read there -- and the reference goes."""
        if prev is None:
            return
        if self._pending is prev:
            self._pending = None
        self._signal_torch(*(t for t in prev if t is not None))

    def close(self):
        self._pending = None
        if getattr(self, "_h", None):
            _lib.load().tsdf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- hot path ----
    def _frame(self, rgb, depth, ht, lt):
        dev = _is_torch_cuda(depth)
        if dev:
            H, W = int(depth.shape[0]), int(depth.shape[1])
            for a in (rgb, depth, ht, lt):
                if a is not None and not a.is_contiguous():
                    raise ValueError("device frames must be contiguous")
        else:
            rgb = _np(rgb, np.uint8)
            depth = _np(depth, np.float32)
            ht = _np(ht, np.float32)
            lt = _np(lt, np.float32)
            H, W = depth.shape
        if tuple(rgb.shape[:2]) != (H, W):
            raise ValueError("rgb / depth size mismatch (voxel_tsdf.cu:352-353)")
        # the arrays stay referenced by the caller for the duration of the call
        return _lib.Frame(W, H, _ptr(rgb), _ptr(depth), _ptr(ht), _ptr(lt),
                          TSDF_MEM_DEVICE if dev else TSDF_MEM_HOST), (rgb, depth, ht, lt)

    def _rgbd_inputs(self, rgb, depth_u16, mask):
        dev = _is_torch_cuda(depth_u16)
        if dev:
            for a in (rgb, depth_u16, mask):
                if a is not None and not a.is_contiguous():
                    raise ValueError("device frames must be contiguous")
        else:
            rgb = _np(rgb, np.uint8)
            depth_u16 = _np(depth_u16, np.uint16)
            mask = _np(mask, np.uint8)
        H, W = int(depth_u16.shape[0]), int(depth_u16.shape[1])
        if tuple(rgb.shape[:2]) != (H, W) or (mask is not None and tuple(mask.shape[:2]) != (H, W)):
            raise ValueError("rgb / depth / mask size mismatch")
        return dev, rgb, depth_u16, mask, W, H

    def rgbd_half(self, rgb, depth_u16, mask, depth_factor: float):
        """DISINFSystem::feed_rgbd_frame preprocessing alone (x0.5 resize, depth scale, mask):
        returns (rgb (H/2, W/2, 3) u8, depth (H/2, W/2) f32), host arrays or device tensors."""
        dev, rgb, depth_u16, mask, W, H = self._rgbd_inputs(rgb, depth_u16, mask)
        if dev:
            import torch
            ro = torch.empty((H // 2, W // 2, 3), dtype=torch.uint8, device=depth_u16.device)
            do = torch.empty((H // 2, W // 2), dtype=torch.float32, device=depth_u16.device)
        else:
            ro = np.zeros((H // 2, W // 2, 3), np.uint8)
            do = np.zeros((H // 2, W // 2), np.float32)
        self._wait_torch(depth_u16, ro)
        _lib.check(_lib.load().tsdf_rgbd_half(self._h, _ptr(rgb), _ptr(depth_u16), _ptr(mask), W, H,
                                              depth_factor, _ptr(ro), _ptr(do),
                                              TSDF_MEM_DEVICE if dev else TSDF_MEM_HOST), "tsdf_rgbd_half")
        self._signal_torch(depth_u16, ro)
        return ro, do

    def feed_rgbd_frame(self, rgb, depth_u16, mask, depth_factor: float, K, cam_T_world: SE3,
                        max_depth: float):
        """DISINFSystem::feed_rgbd_frame after its pose lookup: preprocessing + Integrate on the GPU
        (K = intrinsics of the half-size image)."""
        dev, rgb, depth_u16, mask, W, H = self._rgbd_inputs(rgb, depth_u16, mask)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        self._wait_torch(depth_u16)
        _lib.check(_lib.load().tsdf_feed_rgbd_frame(self._h, _ptr(rgb), _ptr(depth_u16), _ptr(mask), W, H,
                                                    depth_factor, C.byref(Kc), C.byref(cam_T_world._c()),
                                                    max_depth, TSDF_MEM_DEVICE if dev else TSDF_MEM_HOST),
                   "tsdf_feed_rgbd_frame")
        self._signal_torch(depth_u16)

    def frame_graph(self, width: int, height: int, render_width: int = 0, render_height: int = 0,
                    deferred: bool = False, batch: int = 1):
        """Graph-captured frame loop (tsdf_graph_*, BASELINE config C5): integrate (+ raycast of
        a render camera) as one hipGraph launch per frame. deferred=True (tsdf_graph_create_deferred):
        each frame's images are written by the next frame's launch (or the engine's next other call)."""
        return FrameGraph(self, width, height, render_width, render_height, deferred, batch)

    def shard_frame_graph(self, width: int, height: int, slice_index: int = 0, slice_count: int = 1):
        """A shard's graph-captured sharded frame (tsdf_graph_create_shard)."""
        return ShardFrameGraph(self, width, height, slice_index, slice_count)

    # ---- stream ordering with torch (device tensors on torch's current stream) ----
    def _torch_stream(self, tensors):
        """torch's current stream when it differs from the engine stream and a device tensor is
        involved, else None (same stream: already ordered)."""
        if not any(_is_torch_cuda(t) for t in tensors if t is not None):
            return None
        import torch
        cur = _current_raw_stream(torch.cuda.current_device())
        return None if cur == self._stream else cur

    def _wait_torch(self, *tensors):
        """Engine stream waits for torch's current stream when a device tensor goes in."""
        cur = self._torch_stream(tensors)
        if cur is not None:
            _lib.check(_lib.load().tsdf_stream_wait(self._h, C.c_void_p(cur)), "tsdf_stream_wait")

    def _signal_torch(self, *tensors):
        """Torch's current stream waits for the engine when a device tensor it wrote / reads is
        handed back (or may be freed by the caller)."""
        cur = self._torch_stream(tensors)
        if cur is not None:
            _lib.check(_lib.load().tsdf_stream_signal(self._h, C.c_void_p(cur)), "tsdf_stream_signal")

    # ---- sharded frames (tsdf_integrate_shard_*) ----
    @staticmethod
    def shard_slot_bytes(cap: int) -> int:
        """Bytes of one exchange slot: cap records + the count header (tsdf_shard_slot_bytes)."""
        return int(_lib.load().tsdf_shard_slot_bytes(cap))

    def _check_slot(self, buf, cap, slots, what):
        if not _is_torch_cuda(buf) or not buf.is_contiguous() or \
                buf.numel() * buf.element_size() < slots * self.shard_slot_bytes(cap):
            raise ValueError(f"{what} must be a contiguous device tensor of {slots} x shard_slot_bytes({cap})")

    def integrate_shard_begin(self, rgb, depth, ht, lt, K, cam_T_world: SE3, max_depth: float,
                              slice_index: int = 0, slice_count: int = 1, keys_out=None, key_cap: int = 0):
        """Sharded frame, phase 1: pixel records, visibility of this shard's blocks, and the DDA over
        slice `slice_index` of `slice_count` (tile-row bands); the keys it finds go to keys_out (one
        slot), or stay here when slice_count == 1 and keys_out is None (every shard runs the whole
        DDA)."""
        if keys_out is not None:
            self._check_slot(keys_out, key_cap, 1, "keys_out")
        fr, keep = self._frame(rgb, depth, ht, lt)
        self._wait_torch(depth, keys_out)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        _lib.check(_lib.load().tsdf_integrate_shard_begin(self._h, C.byref(fr), C.byref(Kc),
                                                          C.byref(cam_T_world._c()), max_depth,
                                                          slice_index, slice_count, _ptr(keys_out),
                                                          key_cap), "tsdf_integrate_shard_begin")
        self._signal_torch(keys_out)
        # the update (_update) gathers the raw device frame again: the tensors stay referenced here
        # (a temporary such as depth.float() is not freed and reused by torch's allocator) and torch's
        # stream is ordered after the engine for them only once _update is enqueued
        self._shard_frame = keep if _is_torch_cuda(depth) else None

    def integrate_shard_update(self, keys_in, key_cap: int, cands_out, cand_cap: int):
        """Sharded frame, phase 2: merge the all-gathered key slots (None after a whole-frame DDA),
        allocate, update this shard's blocks, write its carve candidates to cands_out (one slot)."""
        if keys_in is not None:
            self._check_slot(keys_in, key_cap, self.shard_count, "keys_in")
        self._check_slot(cands_out, cand_cap, 1, "cands_out")
        self._wait_torch(keys_in, cands_out)
        _lib.check(_lib.load().tsdf_integrate_shard_update(self._h, _ptr(keys_in), key_cap, _ptr(cands_out),
                                                           cand_cap), "tsdf_integrate_shard_update")
        self._release_shard_frame(keys_in, cands_out)

    def _release_shard_frame(self, *tensors):
        """The engine no longer reads the sharded frame's raw tensors once its update is enqueued:
        torch's stream waits for the engine, then the references go."""
        keep = getattr(self, "_shard_frame", None) or ()
        self._signal_torch(*tensors, *keep)
        self._shard_frame = None

    def integrate_shard_end(self, cands_in, cand_cap: int):
        """Sharded frame, phase 3: delete the all-gathered carve candidates (every shard's)."""
        self._check_slot(cands_in, cand_cap, self.shard_count, "cands_in")
        self._wait_torch(cands_in)
        _lib.check(_lib.load().tsdf_integrate_shard_end(self._h, _ptr(cands_in), cand_cap),
                   "tsdf_integrate_shard_end")
        self._signal_torch(cands_in)

    def integrate_shard_pipe(self, rgb, depth, ht, lt, K, cam_T_world, max_depth: float, cands_in, cands_out,
                             cand_cap: int) -> bool:
        """Pipelined sharded frame, one exchange per frame (tsdf_integrate_shard_pipe): this frame's
        ingest (the whole frame's DDA on every shard), the previous frame's allocation and update (this
        shard's carve candidates into cands_out, one slot), the frame before's carving of every shard's
        candidates (cands_in: the all-gathered slots of the previous call). depth None: one step of
        completing the pending frames. Returns True while more such steps (each after an exchange)
        are needed."""
        self._check_slot(cands_out, cand_cap, 1, "cands_out")
        self._check_slot(cands_in, cand_cap, self.shard_count, "cands_in")
        pend = C.c_int32(0)
        if depth is None:
            self._wait_torch(cands_in, cands_out)
            _lib.check(_lib.load().tsdf_integrate_shard_pipe(self._h, None, None, None, max_depth, _ptr(cands_in),
                                                             _ptr(cands_out), cand_cap, C.byref(pend)),
                       "tsdf_integrate_shard_pipe")
            self._signal_torch(cands_in, cands_out)
            return bool(pend.value)
        fr, keep = self._frame(rgb, depth, ht, lt)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        self._wait_torch(depth, cands_in, cands_out)
        _lib.check(_lib.load().tsdf_integrate_shard_pipe(self._h, C.byref(fr), C.byref(Kc), C.byref(cam_T_world._c()),
                                                         max_depth, _ptr(cands_in), _ptr(cands_out), cand_cap,
                                                         C.byref(pend)), "tsdf_integrate_shard_pipe")
        self._signal_torch(depth, cands_in, cands_out)  # (the frame is read by this call only)
        del keep
        return bool(pend.value)

    def integrate_shard_abort(self):
        """Abort a pending sharded frame (tsdf_integrate_shard_abort): the engine is between frames
        again; STATUS_SHARD_ABORTED is set because shards may have diverged (restore snapshots)."""
        try:
            _lib.check(_lib.load().tsdf_integrate_shard_abort(self._h), "tsdf_integrate_shard_abort")
        finally:
            self._release_shard_frame()

    def integrate(self, rgb, depth, ht, lt, K, cam_T_world: SE3, max_depth: float):
        dev = getattr(depth, "is_cuda", False) is True and hasattr(depth, "data_ptr")
        if dev:  # (the hot path: torch's stream is looked up once, no extra ordering calls when the
            # engine runs on it; ctypes passes the structs by reference itself)
            H, W = depth.shape[0], depth.shape[1]
            if not (rgb.is_contiguous() and depth.is_contiguous() and (ht is None or ht.is_contiguous())
                    and (lt is None or lt.is_contiguous())):
                raise ValueError("device frames must be contiguous")
            if rgb.shape[0] != H or rgb.shape[1] != W:
                raise ValueError("rgb / depth size mismatch (voxel_tsdf.cu:352-353)")
            fr = _lib.Frame(W, H, rgb.data_ptr(), depth.data_ptr(), ht.data_ptr() if ht is not None else None,
                            lt.data_ptr() if lt is not None else None, TSDF_MEM_DEVICE)
            Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
            cur = _current_raw_stream(depth.get_device())
            L = _lib.load()
            if cur != self._stream:
                _lib.check(L.tsdf_stream_wait(self._h, C.c_void_p(cur)), "tsdf_stream_wait")
            rc = L.tsdf_integrate(self._h, fr, Kc, cam_T_world._c(), max_depth)
            if rc:
                _lib.check(rc, "tsdf_integrate")
            if cur != self._stream:
                _lib.check(L.tsdf_stream_signal(self._h, C.c_void_p(cur)), "tsdf_stream_signal")
            return
        else:
            rgb = _np(rgb, np.uint8)
            depth = _np(depth, np.float32)
            ht = _np(ht, np.float32)
            lt = _np(lt, np.float32)
            H, W = depth.shape
        if tuple(rgb.shape[:2]) != (H, W):
            raise ValueError("rgb / depth size mismatch (voxel_tsdf.cu:352-353)")
        fr = _lib.Frame(W, H, _ptr(rgb), _ptr(depth), _ptr(ht), _ptr(lt),
                        TSDF_MEM_DEVICE if dev else TSDF_MEM_HOST)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        self._wait_torch(depth)
        _lib.check(_lib.load().tsdf_integrate(self._h, C.byref(fr), C.byref(Kc),
                                              C.byref(cam_T_world._c()), max_depth),
                   "tsdf_integrate")
        self._signal_torch(depth)  # the caller may overwrite / free the frame after this

    def synchronize(self):
        _lib.check(_lib.load().tsdf_synchronize(self._h), "tsdf_synchronize")

    def flush(self):
        """Enqueue the deferred update of the last integrated frame (pipelined frames) on the engine
        stream without waiting: a device synchronisation (torch.cuda.synchronize) afterwards covers
        every frame integrated so far."""
        _lib.check(_lib.load().tsdf_flush(self._h), "tsdf_flush")

    # ---- extraction ----
    def raycast(self, K, width, height, cam_T_world: SE3, max_depth: float, rgba=None, normal=None,
                deferred=False):
        """tsdf_raycast; deferred=True (device tensors only): tsdf_raycast_deferred -- the images are
        written by the engine's next call (fused with the next frame's ingest when that is integrate;
        flush() otherwise); after that call they may be read on torch's current stream (the engine keeps
        them referenced until then and orders torch's stream after the call)."""
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        if deferred:
            if rgba is None or not _is_torch_cuda(rgba) or (normal is not None and not _is_torch_cuda(normal)):
                raise ValueError("a deferred raycast writes device tensors")
            self._wait_torch(rgba, normal)
            _lib.check(_lib.load().tsdf_raycast_deferred(self._h, C.byref(Kc), width, height,
                                                         C.byref(cam_T_world._c()), max_depth, _ptr(rgba),
                                                         _ptr(normal)), "tsdf_raycast_deferred")
            self._pending = (rgba, normal)
            return rgba, normal
        if rgba is not None and _is_torch_cuda(rgba):
            self._wait_torch(rgba, normal)
            _lib.check(_lib.load().tsdf_raycast(self._h, C.byref(Kc), width, height,
                                                C.byref(cam_T_world._c()), max_depth, _ptr(rgba),
                                                _ptr(normal), TSDF_MEM_DEVICE), "tsdf_raycast")
            self._signal_torch(rgba, normal)
            return rgba, normal
        rgba = np.zeros((height, width, 4), np.uint8)
        normal = np.zeros((height, width, 4), np.uint8)
        _lib.check(_lib.load().tsdf_raycast(self._h, C.byref(Kc), width, height,
                                            C.byref(cam_T_world._c()), max_depth, _ptr(rgba),
                                            _ptr(normal), TSDF_MEM_HOST), "tsdf_raycast")
        return rgba, normal

    def raycast_rows(self, K, width, height, cam_T_world: SE3, max_depth: float, row0: int, nrows: int,
                     rgba=None, normal=None):
        """Rows [row0, row0 + nrows) of raycast(K, width, height, ...) (tsdf_raycast_rows): numpy
        (nrows, width, 4) u8 images, or into the given device tensors."""
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        if rgba is not None and _is_torch_cuda(rgba):
            self._wait_torch(rgba, normal)
            _lib.check(_lib.load().tsdf_raycast_rows(self._h, C.byref(Kc), width, height,
                                                     C.byref(cam_T_world._c()), max_depth, row0, nrows,
                                                     _ptr(rgba), _ptr(normal), TSDF_MEM_DEVICE), "tsdf_raycast_rows")
            self._signal_torch(rgba, normal)
            return rgba, normal
        rgba = np.zeros((nrows, width, 4), np.uint8)
        normal = np.zeros((nrows, width, 4), np.uint8)
        _lib.check(_lib.load().tsdf_raycast_rows(self._h, C.byref(Kc), width, height, C.byref(cam_T_world._c()),
                                                 max_depth, row0, nrows, _ptr(rgba), _ptr(normal), TSDF_MEM_HOST),
                   "tsdf_raycast_rows")
        return rgba, normal

    def _grouped(self, fn, args, ngroups, device):
        """Two-call grouped records (tsdf_render_bands / tsdf_pack_halo) -> (counts, records)."""
        counts = np.zeros(ngroups, np.int64)
        _lib.check(fn(*args, None, 0, _ptr(counts), TSDF_MEM_HOST), fn.__name__)
        n = int(counts.sum())
        if device:
            import torch
            out = torch.empty((n, BLOCK_RECORD_BYTES), dtype=torch.uint8, device=f"cuda:{self.device}")
        else:
            out = np.empty((n, BLOCK_RECORD_BYTES), np.uint8)
        if n:
            self._wait_torch(out)
            _lib.check(fn(*args, _ptr(out), n, _ptr(counts), TSDF_MEM_DEVICE if device else TSDF_MEM_HOST),
                       fn.__name__)
            self._signal_torch(out)
        return counts, out

    def render_bands(self, K, width, height, cam_T_world: SE3, max_depth: float, rows, device=False):
        """(counts per band, records grouped by band) of this shard's blocks the rays of rows
        [rows[b], rows[b + 1]) can read (tsdf_render_bands)."""
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        r = np.ascontiguousarray(rows, dtype=np.int32)
        self._rows_keep = r
        L = _lib.load()
        return self._grouped(L.tsdf_render_bands, (self._h, C.byref(Kc), width, height, C.byref(cam_T_world._c()),
                                                   max_depth, r.shape[0] - 1, _ptr(r)), r.shape[0] - 1, device)

    def pack_halo(self, device=False):
        """(counts per destination shard, records grouped by destination) of this shard's blocks that
        other shards' marching cubes read (tsdf_pack_halo)."""
        return self._grouped(_lib.load().tsdf_pack_halo, (self._h,), self.shard_count, device)

    def render_blocks(self, K, width, height, cam_T_world: SE3, max_depth: float, device=False):
        """Records (n, TSDF_BLOCK_RECORD_BYTES) uint8 of the blocks a raycast of this camera can read
        (tsdf_render_blocks): a numpy array, or a torch tensor on this engine's GPU when device."""
        L = _lib.load()
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        pc = cam_T_world._c()
        n = C.c_int64()
        _lib.check(L.tsdf_render_blocks(self._h, C.byref(Kc), width, height, C.byref(pc), max_depth,
                                        None, 0, C.byref(n), TSDF_MEM_HOST), "tsdf_render_blocks")
        if device:
            import torch
            out = torch.empty((n.value, BLOCK_RECORD_BYTES), dtype=torch.uint8,
                              device=f"cuda:{self.device}")
            kind = TSDF_MEM_DEVICE
        else:
            out = np.empty((n.value, BLOCK_RECORD_BYTES), np.uint8)
            kind = TSDF_MEM_HOST
        if n.value:
            self._wait_torch(out)
            _lib.check(L.tsdf_render_blocks(self._h, C.byref(Kc), width, height, C.byref(pc),
                                            max_depth, _ptr(out), n.value, C.byref(n), kind),
                       "tsdf_render_blocks")
            self._signal_torch(out)
        return out

    def pack_blocks(self, bounds=None, device=False):
        """Records (n, TSDF_BLOCK_RECORD_BYTES) of the Query block selection (tsdf_pack_blocks;
        bounds None = every live block): numpy, or a torch tensor on this engine's GPU."""
        L = _lib.load()
        b = None if bounds is None else np.ascontiguousarray(
            bounds.as_array() if isinstance(bounds, BoundingCube) else bounds, dtype=np.float32)
        n = C.c_int64()
        _lib.check(L.tsdf_pack_blocks(self._h, _ptr(b), None, 0, C.byref(n), TSDF_MEM_HOST),
                   "tsdf_pack_blocks")
        if device:
            import torch
            out = torch.empty((n.value, BLOCK_RECORD_BYTES), dtype=torch.uint8,
                              device=f"cuda:{self.device}")
        else:
            out = np.empty((n.value, BLOCK_RECORD_BYTES), np.uint8)
        if n.value:
            self._wait_torch(out)
            _lib.check(L.tsdf_pack_blocks(self._h, _ptr(b), _ptr(out), n.value, C.byref(n),
                                          TSDF_MEM_DEVICE if device else TSDF_MEM_HOST),
                       "tsdf_pack_blocks")
            self._signal_torch(out)
        return out

    def import_blocks(self, records, replace=False):
        """Allocate and fill the blocks of render records (tsdf_import_blocks); numpy or GPU tensor.
        replace: empty the volume first, so it holds exactly these blocks."""
        n = int(records.shape[0]) if records.ndim == 2 else int(records.size) // BLOCK_RECORD_BYTES
        kind = TSDF_MEM_DEVICE if _is_torch_cuda(records) else TSDF_MEM_HOST
        if kind == TSDF_MEM_HOST:
            records = np.ascontiguousarray(records, dtype=np.uint8)
        self._wait_torch(records)  # e.g. an all-gather / torch.cat still queued on torch's stream
        _lib.check(_lib.load().tsdf_import_blocks(self._h, _ptr(records), n, kind, int(replace)),
                   "tsdf_import_blocks")
        self._signal_torch(records)

    def reset(self):
        """Empty the volume (tsdf_reset)."""
        _lib.check(_lib.load().tsdf_reset(self._h), "tsdf_reset")

    def extract_mesh(self, bounds=None, missing_tsdf: float = 0.99, min_weight: int = 0,
                     out=None, owner=None) -> np.ndarray:
        """Marching-cubes triangles (n, 3, 3) float32 of the selected blocks (tsdf_extract_mesh).
        out: optional device tensor of >= 9 n floats to receive them on the GPU instead.
        owner: (shard_index, shard_count) -- only the blocks of that shard emit
        (tsdf_extract_mesh_owned; the others are read as neighbours)."""
        L = _lib.load()
        b = None if bounds is None else np.ascontiguousarray(
            bounds.as_array() if isinstance(bounds, BoundingCube) else bounds, dtype=np.float32)
        oi, oc = owner if owner is not None else (0, 1)
        fn = lambda ptr, cap, n, kind: L.tsdf_extract_mesh_owned(self._h, _ptr(b), missing_tsdf, min_weight,
                                                                 oi, oc, ptr, cap, C.byref(n), kind)
        n = C.c_int64()
        if out is not None:  # one call: count, scan and emission enqueued together, one host read
            if not (_is_torch_cuda(out) and out.is_contiguous() and str(out.dtype) == "torch.float32"):
                raise ValueError("out must be a contiguous float32 device tensor")
            self._wait_torch(out)
            _lib.check(fn(_ptr(out), out.numel() // 9, n, TSDF_MEM_DEVICE), "tsdf_extract_mesh")
            self._signal_torch(out)
            return out[:9 * n.value].view(-1, 3, 3)
        _lib.check(fn(None, 0, n, TSDF_MEM_HOST), "tsdf_extract_mesh")
        tris = np.zeros((n.value, 3, 3), np.float32)
        if n.value:
            _lib.check(fn(_ptr(tris), n.value, n, TSDF_MEM_HOST), "tsdf_extract_mesh")
        return tris

    def query(self, bounds=None) -> np.ndarray:
        L = _lib.load()
        b = None if bounds is None else np.ascontiguousarray(
            bounds.as_array() if isinstance(bounds, BoundingCube) else bounds, dtype=np.float32)
        n = C.c_int64()
        _lib.check(L.tsdf_query(self._h, _ptr(b), None, 0, C.byref(n)), "tsdf_query")
        out = np.zeros(n.value, VOXEL_DTYPE)
        if n.value:
            _lib.check(L.tsdf_query(self._h, _ptr(b), out.ctypes.data_as(C.c_void_p), n.value,
                                    C.byref(n)), "tsdf_query")
        return out

    def snapshot(self) -> np.ndarray:
        """The whole volume between frames as bytes (tsdf_snapshot_save): restore() on an engine
        of the same voxel size, truncation and pool size continues the stream bit for bit."""
        L = _lib.load()
        n = C.c_int64()
        _lib.check(L.tsdf_snapshot_bytes(self._h, C.byref(n)), "tsdf_snapshot_bytes")
        buf = np.empty(n.value, np.uint8)
        _lib.check(L.tsdf_snapshot_save(self._h, _ptr(buf), n.value), "tsdf_snapshot_save")
        return buf

    def restore(self, snapshot):
        buf = np.ascontiguousarray(snapshot, dtype=np.uint8)
        _lib.check(_lib.load().tsdf_snapshot_load(self._h, _ptr(buf), buf.size), "tsdf_snapshot_load")

    def stats(self, clear_status=False) -> dict:
        s = _lib.Stats()
        _lib.check(_lib.load().tsdf_get_stats(self._h, C.byref(s), int(clear_status)), "tsdf_get_stats")
        return {k: getattr(s, k) for k, _ in _lib.Stats._fields_}

    def profile_begin(self, integrate_only: bool = False, every: int = 1, kernel_events: bool = False):
        """HIP-event timing of every `every`-th following integrate call: all phases (marker
        events between them), only k_integrate (marker events around it), or -- kernel_events --
        k_integrate's own dispatch timestamps (start/stop events bound to the launch)."""
        mode = 2 if kernel_events else (1 if integrate_only else 0)
        _lib.check(_lib.load().tsdf_profile_begin(self._h, mode, every), "tsdf_profile_begin")

    def profile_end(self) -> dict:
        p = _lib.Profile()
        _lib.check(_lib.load().tsdf_profile_end(self._h, C.byref(p)), "tsdf_profile_end")
        return {k: getattr(p, k) for k, _ in _lib.Profile._fields_}

    def dump(self, pool: bool = True) -> dict:
        pos = np.zeros((NUM_ENTRY, 4), np.int16)
        idx = np.zeros(NUM_ENTRY, np.int32)
        heap = np.zeros(self.num_blocks, np.int32)
        free = np.zeros(1, np.int32)
        out = dict(entry_pos=pos, entry_idx=idx, heap=heap)
        tsdf = prob = rgbw = None
        if pool:
            nv = self.num_blocks * BLOCK_VOLUME
            tsdf = np.zeros(nv, np.float32)
            prob = np.zeros(nv, np.float32)
            rgbw = np.zeros((nv, 4), np.uint8)
            out.update(tsdf=tsdf, prob=prob, rgbw=rgbw)
        _lib.check(_lib.load().tsdf_debug_dump(self._h, _ptr(pos), _ptr(idx), _ptr(heap), _ptr(free),
                                               _ptr(tsdf), _ptr(prob), _ptr(rgbw)), "tsdf_debug_dump")
        out["free"] = int(free[0])
        return out

    # ---- VoxelHashTable / VoxelMemPool level ----
    def hash_allocate(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.int16).reshape(-1, 3)
        _lib.check(_lib.load().tsdf_hash_allocate(self._h, _ptr(k), k.shape[0]), "tsdf_hash_allocate")

    def hash_delete(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.int16).reshape(-1, 3)
        _lib.check(_lib.load().tsdf_hash_delete(self._h, _ptr(k), k.shape[0]), "tsdf_hash_delete")

    def hash_retrieve(self, points) -> dict:
        p = np.ascontiguousarray(points, dtype=np.int16).reshape(-1, 3)
        n = p.shape[0]
        rgbw = np.zeros((n, 4), np.uint8)
        tsdf = np.zeros(n, np.float32)
        prob = np.zeros(n, np.float32)
        bpo = np.zeros((n, 4), np.int16)
        bidx = np.zeros(n, np.int32)
        _lib.check(_lib.load().tsdf_hash_retrieve(self._h, _ptr(p), n, _ptr(rgbw), _ptr(tsdf),
                                                  _ptr(prob), _ptr(bpo), _ptr(bidx)), "tsdf_hash_retrieve")
        return dict(rgbw=rgbw, tsdf=tsdf, prob=prob, block_pos_off=bpo, block_idx=bidx)

    def hash_assign(self, points, rgbw) -> int:
        p = np.ascontiguousarray(points, dtype=np.int16).reshape(-1, 3)
        v = np.ascontiguousarray(rgbw, dtype=np.uint8).reshape(-1, 4)
        missing = C.c_int()
        _lib.check(_lib.load().tsdf_hash_assign(self._h, _ptr(p), p.shape[0], _ptr(v),
                                                C.byref(missing)), "tsdf_hash_assign")
        return missing.value

    def num_active_blocks(self) -> int:
        n = C.c_int32()
        _lib.check(_lib.load().tsdf_num_active_blocks(self._h, C.byref(n)), "tsdf_num_active_blocks")
        return n.value

    def pool_acquire(self, n: int) -> np.ndarray:
        out = np.zeros(n, np.int32)
        _lib.check(_lib.load().tsdf_pool_acquire(self._h, n, _ptr(out)), "tsdf_pool_acquire")
        return out

    def pool_release(self, idx):
        i = np.ascontiguousarray(idx, dtype=np.int32)
        _lib.check(_lib.load().tsdf_pool_release(self._h, _ptr(i), i.shape[0]), "tsdf_pool_release")

    def pool_set_weight(self, block: int, w: int):
        _lib.check(_lib.load().tsdf_pool_set_weight(self._h, int(block), int(w)), "tsdf_pool_set_weight")

    def pool_get_weights(self, block: int) -> np.ndarray:
        out = np.zeros(BLOCK_VOLUME, np.uint8)
        _lib.check(_lib.load().tsdf_pool_get_weights(self._h, int(block), _ptr(out)), "tsdf_pool_get_weights")
        return out


def _engine_call(fn):
    """Every public Engine method that enters the library settles a pending deferred raycast after
    its call (Engine._after_call)."""
    def wrapper(self, *a, **k):
        prev = self._pending
        r = fn(self, *a, **k)
        self._after_call(prev)
        return r
    wrapper.__name__, wrapper.__doc__, wrapper.__wrapped__ = fn.__name__, fn.__doc__, fn
    return wrapper


for _name, _fn in list(vars(Engine).items()):
    if callable(_fn) and not _name.startswith("_") and _name not in ("close", "frame_graph", "shard_frame_graph") \
            and not isinstance(_fn, (staticmethod, classmethod)):
        setattr(Engine, _name, _engine_call(_fn))
del _name, _fn


class Group:
    """One volume spatially sharded over `devices` (one shard per entry; a device may repeat) with the
    exchange inside the library (tsdf_group_*, csrc/tsdf_group.hip): each shard's update kernel
    writes its carve candidates into every shard's inbox, so a frame is one launch per shard and no
    collective. Same results as one volume (the union of the shards)."""

    def __init__(self, devices, voxel_size=0.005, truncation=0.03, max_width=1920, max_height=1080,
                 num_block_bits=18):
        L = _lib.load()
        cfg = _lib.Config()
        L.tsdf_config_default(C.byref(cfg))
        cfg.voxel_size, cfg.truncation = voxel_size, truncation
        cfg.max_width, cfg.max_height, cfg.num_block_bits = max_width, max_height, num_block_bits
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        _lib.check(L.tsdf_group_create(C.byref(cfg), devs, len(devices), C.byref(h)), "tsdf_group_create")
        self._g = h
        self.n = len(devices)
        self.devices = list(devices)
        self.num_blocks = 1 << num_block_bits
        self.voxel_size, self.truncation = voxel_size, truncation

    def integrate(self, rgb, depth, ht, lt, K, cam_T_world: SE3, max_depth: float):
        """Host arrays, or device tensors on devices[0] (contiguous; torch's stream is synchronised
        first: the group runs on its own streams, and torch's current stream is ordered after the
        group's work afterwards -- tsdf_group_stream_signal -- so the frame's tensors may be reused or
        freed on it)."""
        dev = _is_torch_cuda(depth)
        if dev:
            import torch
            torch.cuda.current_stream().synchronize()
            for a in (rgb, depth, ht, lt):
                if a is not None and not a.is_contiguous():
                    raise ValueError("device frames must be contiguous")
            H, W = int(depth.shape[0]), int(depth.shape[1])
        else:
            rgb, depth = _np(rgb, np.uint8), _np(depth, np.float32)
            ht, lt = _np(ht, np.float32), _np(lt, np.float32)
            H, W = depth.shape
        fr = _lib.Frame(W, H, _ptr(rgb), _ptr(depth), _ptr(ht), _ptr(lt), TSDF_MEM_DEVICE if dev else TSDF_MEM_HOST)
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        L = _lib.load()
        _lib.check(L.tsdf_group_integrate(self._g, C.byref(fr), C.byref(Kc), C.byref(cam_T_world._c()), max_depth),
                   "tsdf_group_integrate")
        if dev:
            _lib.check(L.tsdf_group_stream_signal(self._g, C.c_void_p(_current_raw_stream(self.devices[0]))),
                       "tsdf_group_stream_signal")

    def flush(self):
        _lib.check(_lib.load().tsdf_group_flush(self._g), "tsdf_group_flush")

    def synchronize(self):
        _lib.check(_lib.load().tsdf_group_synchronize(self._g), "tsdf_group_synchronize")

    def stats(self, clear_status=False) -> dict:
        s = _lib.Stats()
        _lib.check(_lib.load().tsdf_group_get_stats(self._g, C.byref(s), int(clear_status)), "tsdf_group_get_stats")
        return {k: getattr(s, k) for k, _ in _lib.Stats._fields_}

    def query(self, bounds=None) -> np.ndarray:
        b = None if bounds is None else np.ascontiguousarray(
            bounds.as_array() if isinstance(bounds, BoundingCube) else bounds, dtype=np.float32)
        n = C.c_int64()
        L = _lib.load()
        _lib.check(L.tsdf_group_query(self._g, _ptr(b), None, 0, C.byref(n)), "tsdf_group_query")
        out = np.zeros(n.value, VOXEL_DTYPE)
        if n.value:
            _lib.check(L.tsdf_group_query(self._g, _ptr(b), out.ctypes.data_as(C.c_void_p), n.value, C.byref(n)),
                       "tsdf_group_query")
        return out

    def raycast(self, K, width, height, cam_T_world: SE3, max_depth: float):
        Kc = K._c() if isinstance(K, CameraIntrinsics) else _lib.Intrinsics(*[float(v) for v in K])
        rgba = np.zeros((height, width, 4), np.uint8)
        normal = np.zeros((height, width, 4), np.uint8)
        _lib.check(_lib.load().tsdf_group_raycast(self._g, C.byref(Kc), width, height, C.byref(cam_T_world._c()),
                                                  max_depth, _ptr(rgba), _ptr(normal), TSDF_MEM_HOST),
                   "tsdf_group_raycast")
        return rgba, normal

    def shard(self, i: int) -> "Engine":
        """Shard i's engine (tsdf_group_shard: completes the pending frames first), a borrowed handle
        the group owns -- for dumps, statistics and profiling of one shard; do not close it."""
        h = C.c_void_p()
        _lib.check(_lib.load().tsdf_group_shard(self._g, i, C.byref(h)), "tsdf_group_shard")
        eng = Engine.__new__(Engine)
        eng._h, eng.num_blocks, eng._pending, eng._stream = h, self.num_blocks, None, -1
        eng.device, eng.shard_index, eng.shard_count = self.devices[i], i, self.n
        eng.voxel_size, eng.truncation = self.voxel_size, self.truncation
        eng.close = lambda: None  # (borrowed)
        return eng

    def shard_dump(self, i: int, pool: bool = True) -> dict:
        """tsdf_debug_dump of shard i's engine (tsdf_group_shard)."""
        return self.shard(i).dump(pool)

    def close(self):
        if getattr(self, "_g", None):
            _lib.load().tsdf_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardGroup:
    """G shard engines of one spatially sharded volume on ONE GPU, exchanging their key
    and carve-candidate slots with device copies where a multi-GPU job all-gathers them
    (tsdf_amd.dist.integrate_sharded). The engines run on torch's current stream, so the copies are
    ordered between the phases. For tests and single-GPU rehearsals of the sharded path.
    split: True -- shard i runs the DDA over tile-row band i of G and the keys are exchanged;
    False -- every shard runs the whole frame's DDA, only carve candidates are exchanged."""

    def __init__(self, shard_count: int, voxel_size=0.005, truncation=0.03, max_width=1920,
                 max_height=1080, num_block_bits=18, device=0, key_cap=16384, cand_cap=16384,
                 split=True, stream=None, graph=None, pipe=False):
        import torch
        self.G = shard_count
        # pipe: pipelined sharded frames (tsdf_integrate_shard_pipe, one exchange per frame, every shard
        # runs the whole DDA); reads of the volume need flush() first
        self.pipe = pipe
        if pipe and (split or graph is not None):
            raise ValueError("pipelined sharded frames run the whole DDA on every shard (split=False, no graph)")
        self.graph_size = graph  # (width, height): frames through each shard's captured graph
        self.split = split
        self.key_cap, self.cand_cap = key_cap, cand_cap
        # all shards on ONE stream (torch's current one unless given), so the phases and the slot
        # reads / writes between them are ordered
        stream = torch.cuda.current_stream(device) if stream is None else stream
        self.engines = [Engine(voxel_size, truncation, max_width, max_height, num_block_bits, device,
                               shard_index=i, shard_count=shard_count, stream=stream)
                        for i in range(shard_count)]
        dev = f"cuda:{device}"
        self._keys = torch.zeros((shard_count, Engine.shard_slot_bytes(key_cap)), dtype=torch.uint8, device=dev)
        self._cands = torch.zeros((shard_count, Engine.shard_slot_bytes(cand_cap)), dtype=torch.uint8, device=dev)
        self.keys_exchanged = 0   # key records that went through the exchange (all frames)
        self.cands_exchanged = 0  # carve-candidate records likewise
        self.cands_by_shard = [0] * shard_count  # ... by the shard that sent them
        # pipelined: call n writes its candidates into slot set n % 2 and reads set (n - 1) % 2 (the
        # "all-gather" of the previous call: every shard's slot)
        self._pc = torch.zeros((2, shard_count, Engine.shard_slot_bytes(cand_cap)), dtype=torch.uint8,
                               device=dev) if pipe else None
        self._ncall = 0
        self.graphs = None
        if graph is not None:
            w, h = graph
            self.graphs = [e.shard_frame_graph(w, h, i if split else 0, shard_count if split else 1)
                           for i, e in enumerate(self.engines)]

    def integrate(self, rgb, depth, ht, lt, K, cam_T_world: SE3, max_depth: float, count=False):
        try:
            self._integrate(rgb, depth, ht, lt, K, cam_T_world, max_depth, count)
        except Exception:
            self._abort_all()
            raise

    def _abort_all(self):
        # no shard stays stuck mid-frame (three-call frames and pipelined ones alike); every shard is
        # aborted even if one abort fails, and the caller sees the original error
        for e in self.engines:
            try:
                e.integrate_shard_abort()
            except Exception:
                pass

    def _pipe_step(self, rgb, depth, ht, lt, K, cam_T_world, max_depth):
        out, inb = self._pc[self._ncall & 1], self._pc[(self._ncall + 1) & 1]
        # (the call counter moves even when a shard fails part-way: the aborted shards restart from
        # "no pending frame", whose first call reads no inbox)
        self._ncall += 1
        pend = [e.integrate_shard_pipe(rgb, depth, ht, lt, K, cam_T_world, max_depth, inb, out[i], self.cand_cap)
                for i, e in enumerate(self.engines)]
        return any(pend)

    def flush(self):
        """Pipelined: complete the pending frames (steps with their exchanges); a no-op otherwise."""
        if self.pipe:
            try:
                while self._pipe_step(None, None, None, None, None, None, 4.0):
                    pass
            except Exception:
                self._abort_all()
                raise

    def _integrate(self, rgb, depth, ht, lt, K, cam_T_world, max_depth, count):
        G = self.G
        if self.pipe:
            self._pipe_step(rgb, depth, ht, lt, K, cam_T_world, max_depth)
            # this call's slots hold the candidates of the frame it updated
            self._count(count, cands=self._pc[(self._ncall - 1) & 1])
            return
        if self.graphs is not None:
            for i, g in enumerate(self.graphs):
                g.begin(rgb, depth, ht, lt, K, cam_T_world, max_depth, self._keys[i], self._keys, self.key_cap,
                        self._cands[i], self._cands, self.cand_cap)
            for g in self.graphs:
                g.update()
            for g in self.graphs:
                g.end()
            self._count(count)
            return
        for i, e in enumerate(self.engines):
            if self.split:
                e.integrate_shard_begin(rgb, depth, ht, lt, K, cam_T_world, max_depth, i, G, self._keys[i],
                                        self.key_cap)
            else:
                e.integrate_shard_begin(rgb, depth, ht, lt, K, cam_T_world, max_depth)
        keys_in = self._keys if self.split else None  # the all-gathered key slots
        for i, e in enumerate(self.engines):
            e.integrate_shard_update(keys_in, self.key_cap, self._cands[i], self.cand_cap)
        for e in self.engines:
            e.integrate_shard_end(self._cands, self.cand_cap)
        self._count(count)

    def _count(self, count, cands=None):
        if not count:
            return
        import torch
        cands = self._cands if cands is None else cands
        # per-shard candidate counts (slot headers: record 0's count word), a host sync
        per = cands[:, 8:12].contiguous().view(torch.int32).view(-1).tolist()
        self.cands_by_shard = [a + b for a, b in zip(self.cands_by_shard, per)]
        if self.split:
            self.keys_exchanged += int(self._keys[:, 8:12].contiguous().view(torch.int32).sum())
        self.cands_exchanged += sum(per)

    def synchronize(self):
        self.flush()
        for e in self.engines:
            e.synchronize()

    def stats(self):
        self.flush()
        return [e.stats() for e in self.engines]

    def close(self):
        for g in self.graphs or []:
            g.close()
        for e in self.engines:
            e.close()


class TSDFGrid:
    """voxel_tsdf.cuh:32-124 TSDFGrid(voxel_size, truncation) on the MI355X engine."""

    def __init__(self, voxel_size: float, truncation: float, **engine_kw):
        self.engine = Engine(voxel_size=voxel_size, truncation=truncation, **engine_kw)

    def Integrate(self, img_rgb, img_depth, img_ht, img_lt, max_depth: float,
                  intrinsics: CameraIntrinsics, cam_T_world: SE3):
        """voxel_tsdf.cu:347-375. img_ht / img_lt are required here as in the reference."""
        self.engine.integrate(img_rgb, img_depth, img_ht, img_lt, intrinsics, cam_T_world, max_depth)

    def RayCast(self, max_depth: float, virtual_cam: CameraParams, cam_T_world: SE3):
        """voxel_tsdf.cu:490-506; returns (rgba, normal) HxWx4 uint8 images."""
        return self.engine.raycast(virtual_cam.intrinsics, virtual_cam.img_w, virtual_cam.img_h,
                                   cam_T_world, max_depth)

    def GatherValid(self) -> np.ndarray:
        """voxel_tsdf.cu:399-425."""
        return self.engine.query(None)

    def GatherVoxels(self, volumn: BoundingCube) -> np.ndarray:
        """voxel_tsdf.cu:427-454."""
        return self.engine.query(volumn)

    def close(self):
        self.engine.close()
