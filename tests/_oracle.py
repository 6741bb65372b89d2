"""ctypes view of the CPU oracle (oracle/tsdf_oracle.c). TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the
product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle_tsdf.so")
NUM_ENTRY = 1 << 22
BLOCK_VOLUME = 512

_lib = None


class OraStats(C.Structure):
    _fields_ = [
        ("frames", C.c_int64),
        ("last_num_visible", C.c_int32),
        ("last_num_updated", C.c_int64),
        ("last_num_alloc", C.c_int32),
        ("last_num_deleted", C.c_int32),
        ("last_num_candidates", C.c_int32),
        ("active_blocks", C.c_int32),
        ("last_cross_losses", C.c_int32),
        ("pool_exhausted", C.c_int32),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.ora_create.restype = P
        L.ora_create.argtypes = [C.c_float, C.c_float, C.c_int]
        L.ora_destroy.argtypes = [P]
        L.ora_integrate.restype = C.c_int
        L.ora_integrate.argtypes = [P, P, P, P, P, C.c_int, C.c_int, P, P, P, C.c_float]
        L.ora_raycast.argtypes = [P, P, C.c_int, C.c_int, P, P, C.c_float, P, P]
        L.ora_query.restype = C.c_int64
        L.ora_query.argtypes = [P, P, P, C.c_int64]
        L.ora_get_stats.argtypes = [P, C.POINTER(OraStats)]
        L.ora_dump.argtypes = [P, P, P, P, P, P, P, P]
        L.ora_num_entries.restype = C.c_int32
        L.ora_num_blocks.restype = C.c_int32
        L.ora_num_blocks.argtypes = [P]
        L.ora_hash_allocate.argtypes = [P, P, C.c_int]
        L.ora_hash_delete.argtypes = [P, P, C.c_int]
        L.ora_hash_retrieve.argtypes = [P, P, C.c_int, P, P, P, P, P]
        L.ora_hash_assign.restype = C.c_int
        L.ora_hash_assign.argtypes = [P, P, C.c_int, P]
        L.ora_num_active_blocks.restype = C.c_int32
        L.ora_num_active_blocks.argtypes = [P]
        L.ora_pool_acquire.argtypes = [P, C.c_int, P]
        L.ora_pool_release.argtypes = [P, P, C.c_int]
        L.ora_pool_set_weight.argtypes = [P, C.c_int32, C.c_uint8]
        L.ora_pool_get_weights.argtypes = [P, C.c_int32, P]
        L.ora_set_shard.argtypes = [P, C.c_int, C.c_int]
        L.ora_shard_keys.restype = C.c_int64
        L.ora_shard_keys.argtypes = [P, P, C.c_int, C.c_int, P, P, P, C.c_float, C.c_int, C.c_int, P, P,
                                     C.c_int64]
        L.ora_shard_update.restype = C.c_int64
        L.ora_shard_update.argtypes = [P, P, P, C.c_int64, P, P, P, P, C.c_int, C.c_int, P, P, P,
                                       C.c_float, P, P, C.c_int64]
        L.ora_shard_delete.argtypes = [P, P, P, C.c_int64]
        L.ora_extract_mesh.restype = C.c_int64
        L.ora_extract_mesh.argtypes = [P, P, C.c_float, C.c_int, P, C.c_int64]
        L.ora_block_owner.restype = C.c_uint32
        L.ora_block_owner.argtypes = [C.c_int16, C.c_int16, C.c_int16, C.c_uint32]
        L.ora_hash.restype = C.c_uint32
        L.ora_hash.argtypes = [C.c_int16, C.c_int16, C.c_int16]
        L.ora_rgbd_half.argtypes = [P, P, P, C.c_int, C.c_int, C.c_float, P, P]
        L.ora_logf.restype = C.c_float
        L.ora_logf.argtypes = [C.c_float]
        L.ora_expf.restype = C.c_float
        L.ora_expf.argtypes = [C.c_float]
        L.ora_math_digest.restype = C.c_uint64
        L.ora_math_digest.argtypes = [C.c_int, C.c_uint64, C.c_uint64]
        L.ora_math_accuracy.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_double)]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def block_owner(x, y, z, shards) -> int:
    return int(lib().ora_block_owner(x, y, z, shards))


def hash_block(x, y, z) -> int:
    return int(lib().ora_hash(x, y, z))


def rgbd_half(rgb, depth_u16, mask, depth_factor):
    """DISINFSystem::feed_rgbd_frame preprocessing (disinfect_slam.cc:31-64) -> (rgb, depth f32)."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    depth_u16 = np.ascontiguousarray(depth_u16, np.uint16)
    mask = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    H, W = depth_u16.shape
    ro = np.zeros((H // 2, W // 2, 3), np.uint8)
    do = np.zeros((H // 2, W // 2), np.float32)
    lib().ora_rgbd_half(_p(rgb), _p(depth_u16), _p(mask), W, H, depth_factor, _p(ro), _p(do))
    return ro, do


class OracleGrid:
    """CPU restatement of TSDFGrid (voxel_tsdf.cuh:32-124)."""

    def __init__(self, voxel_size: float, truncation: float, num_block_bits: int = 18,
                 shard_index: int = 0, shard_count: int = 1):
        self.voxel_size = voxel_size
        self.truncation = truncation
        self.h = lib().ora_create(voxel_size, truncation, num_block_bits)
        if not self.h:
            raise MemoryError("ora_create failed")
        if shard_count > 1:
            lib().ora_set_shard(self.h, shard_index, shard_count)
        self.num_blocks = lib().ora_num_blocks(self.h)

    def close(self):
        if self.h:
            lib().ora_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def integrate(self, rgb, depth, ht, lt, max_depth, K, q, t):
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        depth = np.ascontiguousarray(depth, dtype=np.float32)
        ht = None if ht is None else np.ascontiguousarray(ht, dtype=np.float32)
        lt = None if lt is None else np.ascontiguousarray(lt, dtype=np.float32)
        H, W = depth.shape
        K = np.ascontiguousarray(K, dtype=np.float32)
        q = np.ascontiguousarray(q, dtype=np.float32)
        t = np.ascontiguousarray(t, dtype=np.float32)
        rc = lib().ora_integrate(self.h, _p(rgb), _p(depth), _p(ht), _p(lt), W, H, _p(K), _p(q),
                                 _p(t), max_depth)
        if rc != 0:
            raise RuntimeError(f"ora_integrate -> {rc}")

    # --- sharded frame (the engine's tsdf_integrate_shard_* in three phases) ---
    @staticmethod
    def _f32(*arrs):
        return [None if a is None else np.ascontiguousarray(a, dtype=np.float32) for a in arrs]

    def shard_keys(self, depth, K, q, t, max_depth, row_lo, row_hi):
        """Phase 1: DDA over rows [row_lo, row_hi) -> (keys (n, 3) int16, orders (n,) uint64)."""
        depth, K, q, t = self._f32(depth, K, q, t)
        H, W = depth.shape
        cap = max(1, W * max(0, min(row_hi, H) - max(row_lo, 0)) * 4)
        keys = np.zeros((cap, 3), np.int16)
        orders = np.zeros(cap, np.uint64)
        n = lib().ora_shard_keys(self.h, _p(depth), W, H, _p(K), _p(q), _p(t), max_depth, row_lo, row_hi,
                                 _p(keys), _p(orders), cap)
        if n > cap:
            keys = np.zeros((n, 3), np.int16)
            orders = np.zeros(n, np.uint64)
            n = lib().ora_shard_keys(self.h, _p(depth), W, H, _p(K), _p(q), _p(t), max_depth, row_lo,
                                     row_hi, _p(keys), _p(orders), n)
        return keys[:n].copy(), orders[:n].copy()

    def shard_update(self, keys, orders, rgb, depth, ht, lt, max_depth, K, q, t):
        """Phase 2: Allocate the union of the shards' keys, integrate the owned blocks ->
        (carve candidate positions (m, 3) int16, their entries (m,) int32)."""
        keys = np.ascontiguousarray(keys, dtype=np.int16).reshape(-1, 3)
        orders = np.ascontiguousarray(orders, dtype=np.uint64)
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        depth, ht, lt, K, q, t = self._f32(depth, ht, lt, K, q, t)
        H, W = depth.shape
        cap = NUM_ENTRY
        cpos = np.zeros((cap, 3), np.int16)
        cent = np.zeros(cap, np.int32)
        m = lib().ora_shard_update(self.h, _p(keys), _p(orders), keys.shape[0], _p(rgb), _p(depth), _p(ht),
                                   _p(lt), W, H, _p(K), _p(q), _p(t), max_depth, _p(cpos), _p(cent), cap)
        if m < 0:
            raise RuntimeError("ora_shard_update failed")
        return cpos[:m].copy(), cent[:m].copy()

    def shard_delete(self, cand_pos, cand_entry):
        """Phase 3: Delete the union of the shards' carve candidates (entry order)."""
        p = np.ascontiguousarray(cand_pos, dtype=np.int16).reshape(-1, 3)
        e = np.ascontiguousarray(cand_entry, dtype=np.int32)
        lib().ora_shard_delete(self.h, _p(p), _p(e), e.shape[0])

    def raycast(self, K, W, H, q, t, max_depth):
        rgba = np.zeros((H, W, 4), np.uint8)
        normal = np.zeros((H, W, 4), np.uint8)
        K = np.ascontiguousarray(K, dtype=np.float32)
        q = np.ascontiguousarray(q, dtype=np.float32)
        t = np.ascontiguousarray(t, dtype=np.float32)
        lib().ora_raycast(self.h, _p(K), W, H, _p(q), _p(t), max_depth, _p(rgba), _p(normal))
        return rgba, normal

    def query(self, bounds=None):
        b = None if bounds is None else np.ascontiguousarray(bounds, dtype=np.float32)
        n = lib().ora_query(self.h, _p(b), None, 0)
        out = np.zeros((n, 4), np.float32)
        if n:
            lib().ora_query(self.h, _p(b), _p(out), n)
        return out

    def extract_mesh(self, bounds=None, missing_tsdf=0.99, min_weight=0):
        b = None if bounds is None else np.ascontiguousarray(bounds, dtype=np.float32)
        n = lib().ora_extract_mesh(self.h, _p(b), missing_tsdf, min_weight, None, 0)
        out = np.zeros((n, 3, 3), np.float32)
        if n:
            lib().ora_extract_mesh(self.h, _p(b), missing_tsdf, min_weight, _p(out), n)
        return out

    def stats(self) -> dict:
        s = OraStats()
        lib().ora_get_stats(self.h, C.byref(s))
        return {k: getattr(s, k) for k, _ in OraStats._fields_}

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
        lib().ora_dump(self.h, _p(pos), _p(idx), _p(heap), _p(free), _p(tsdf), _p(prob), _p(rgbw))
        out["free"] = int(free[0])
        return out

    # --- hash / pool level (voxel_hash.cu / voxel_mem.cu) ---
    def hash_allocate(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.int16).reshape(-1, 3)
        lib().ora_hash_allocate(self.h, _p(k), k.shape[0])

    def hash_delete(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.int16).reshape(-1, 3)
        lib().ora_hash_delete(self.h, _p(k), k.shape[0])

    def hash_retrieve(self, points):
        p = np.ascontiguousarray(points, dtype=np.int16).reshape(-1, 3)
        n = p.shape[0]
        rgbw = np.zeros((n, 4), np.uint8)
        tsdf = np.zeros(n, np.float32)
        prob = np.zeros(n, np.float32)
        bpo = np.zeros((n, 4), np.int16)
        bidx = np.zeros(n, np.int32)
        lib().ora_hash_retrieve(self.h, _p(p), n, _p(rgbw), _p(tsdf), _p(prob), _p(bpo), _p(bidx))
        return dict(rgbw=rgbw, tsdf=tsdf, prob=prob, block_pos_off=bpo, block_idx=bidx)

    def hash_assign(self, points, rgbw):
        p = np.ascontiguousarray(points, dtype=np.int16).reshape(-1, 3)
        v = np.ascontiguousarray(rgbw, dtype=np.uint8).reshape(-1, 4)
        return lib().ora_hash_assign(self.h, _p(p), p.shape[0], _p(v))

    def num_active_blocks(self) -> int:
        return int(lib().ora_num_active_blocks(self.h))

    def pool_acquire(self, n):
        out = np.zeros(n, np.int32)
        lib().ora_pool_acquire(self.h, n, _p(out))
        return out

    def pool_release(self, idx):
        i = np.ascontiguousarray(idx, dtype=np.int32)
        lib().ora_pool_release(self.h, _p(i), i.shape[0])

    def pool_set_weight(self, block, w):
        lib().ora_pool_set_weight(self.h, int(block), int(w))

    def pool_get_weights(self, block):
        out = np.zeros(BLOCK_VOLUME, np.uint8)
        lib().ora_pool_get_weights(self.h, int(block), _p(out))
        return out
