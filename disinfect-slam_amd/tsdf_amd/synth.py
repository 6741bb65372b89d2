"""Synthetic RGB-D + high/low-touch frame source (SURVEY.md 8d / BASELINE.md 4).

The reference benchmarks nothing and ships no recorded frames, so every measurement and parity
run in this repo integrates a deterministic analytic scene:

* scene: a closed 6 x 5 x 3 m room containing 3 axis-aligned boxes and 2 spheres;
* trajectory: a smooth orbit, 1 cm of arc and 0.5 deg of yaw per frame (seed 0x5EED);
* depth: analytic ray cast, + N(0, 1 mm) noise (seeded), quantised to uint16 / 5000 (TUM factor,
  configs/TUM_RGBD_rgbd_1.yaml:44) and back to float32 metres, 2 % holes, readings beyond 3.9 m
  dropped so that depth != max_depth (the reference's 0/0 case, voxel_tsdf.cu:182-191);
* ht / lt (`touch`): "complement" (default) -- a smooth per-surface field ht in [0.02, 0.98] and
  lt = 1 - ht (no log(0), voxel_tsdf.cu:196-202); "independent" -- two independent fields over
  (0, 1] as a segmentation network's two output channels give them (examples/tsdf/online.cc:59-60,
  segmentation/inference.cc:57-65), with regions and sprinkled pixels at the extremes 1e-6,
  1 - 1e-6, the largest float below 1 and 1; "u16" -- those fields stored as uint16 PNG maps and
  read back with convertTo(CV_32FC1, 1 / 65535) (examples/tsdf/offline.cc:76-82), with exact zeros
  in the lt channel (the shelf, a strip of the walls and sprinkled pixels: p becomes exactly 1);
  "u16z" -- as "u16" with exact zeros in the ht channel too (another strip; pixels or voxels that see ht = lt = 0 fuse to NaN in
  the reference's own arithmetic, 0 / 0 -- the reference leaves that input undefined);
* rgb: a deterministic per-surface checker pattern (uint8, RGB order as TSDFGrid expects).

Frames are produced on the host with numpy (float64 geometry, one float32 rounding at the end), so
the HIP engine and the CPU oracle integrate byte-identical inputs.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

SEED = 0x5EED

# configs/TUM_RGBD_rgbd_1.yaml:11-14 (640x480)
TUM_FR1 = (517.306408, 516.469215, 318.643040, 255.313989)
# 2 x configs/zed_native_l515.yaml:27-30 (L515 full resolution 1280x720)
L515_FULL = (913.7234, 913.54254, 644.2084, 375.5897)
DEPTH_FACTOR = 5000.0
MAX_RANGE = 3.9

ROOM_MIN = np.array([0.0, 0.0, 0.0])
ROOM_MAX = np.array([6.0, 5.0, 3.0])
BOXES = [  # (min, max, surface id)
    (np.array([0.6, 0.5, 0.0]), np.array([1.6, 1.3, 0.75]), 7),   # table
    (np.array([4.3, 3.6, 0.0]), np.array([5.4, 4.6, 1.1]), 8),    # cabinet
    (np.array([2.6, 4.2, 0.0]), np.array([3.4, 4.8, 1.8]), 9),    # shelf
]
SPHERES = [  # (centre, radius, surface id)
    (np.array([4.6, 1.2, 0.9]), 0.45, 10),
    (np.array([1.4, 3.7, 1.2]), 0.35, 11),
]
NUM_SURFACES = 12


@dataclasses.dataclass
class Camera:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float

    @property
    def K(self) -> np.ndarray:
        return np.array([self.fx, self.fy, self.cx, self.cy], dtype=np.float32)


def camera(width: int = 640, height: int = 480, intrinsics=TUM_FR1) -> Camera:
    """Pinhole camera; intrinsics scaled with the image size relative to their native size."""
    native_w = 640 if intrinsics is TUM_FR1 else 1280
    s = width / native_w
    fx, fy, cx, cy = intrinsics
    return Camera(width, height, fx * s, fy * s, (cx + 0.5) * s - 0.5, (cy + 0.5) * s - 0.5)


def _rot_to_quat_xyzw(R: np.ndarray) -> np.ndarray:
    """Rotation matrix -> unit quaternion (x, y, z, w), float64 (Shoemake)."""
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        w = 0.25 * s
        x = (R[2, 1] - R[1, 2]) / s
        y = (R[0, 2] - R[2, 0]) / s
        z = (R[1, 0] - R[0, 1]) / s
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = math.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0) * 2
        q = [0.0, 0.0, 0.0]
        q[i] = 0.25 * s
        w = (R[k, j] - R[j, k]) / s
        q[j] = (R[j, i] + R[i, j]) / s
        q[k] = (R[k, i] + R[i, k]) / s
        x, y, z = q
    q = np.array([x, y, z, w])
    return q / np.linalg.norm(q)


def pose(frame: int, orbit_centre=(3.0, 2.5, 1.45), pitch_deg: float = -12.0):
    """world_T_cam of frame `frame`: camera on a circle of radius 1 cm / 0.5 deg, looking outward.

    Returns (R_wc float64 3x3, p_wc float64 3) and (q_cw xyzw float32, t_cw float32), the latter
    being the cam_T_world the engine API takes (voxel_tsdf.cuh:58-60).
    """
    dtheta = math.radians(0.5)
    radius = 0.01 / dtheta
    theta = frame * dtheta
    c = np.asarray(orbit_centre, dtype=np.float64)
    p = c + radius * np.array([math.cos(theta), math.sin(theta), 0.0])
    p[2] += 0.05 * math.sin(frame * 0.02)
    yaw = theta + math.radians(35.0)
    fwd = np.array([math.cos(yaw), math.sin(yaw), 0.0])
    pitch = math.radians(pitch_deg + 4.0 * math.sin(frame * 0.013))
    fwd = math.cos(pitch) * fwd + math.sin(pitch) * np.array([0.0, 0.0, 1.0])
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    down = np.cross(fwd, right)
    R_wc = np.stack([right, down, fwd], axis=1)  # columns: camera x (right), y (down), z (fwd)
    R_cw = R_wc.T
    t_cw = -R_cw @ p
    q = _rot_to_quat_xyzw(R_cw).astype(np.float32)
    return (R_wc, p), (q, t_cw.astype(np.float32))


def _ray_scene(o: np.ndarray, d: np.ndarray):
    """Nearest hit of rays o + s d (d: N x 3, unnormalised) with the scene. Returns (s, id, point)."""
    n = d.shape[0]
    inv = np.where(np.abs(d) > 1e-12, 1.0 / np.where(d == 0, 1.0, d), 1e12)
    # room interior: exit distance
    t_hi = np.maximum((ROOM_MIN - o) * inv, (ROOM_MAX - o) * inv)
    s_room = np.min(t_hi, axis=1)
    axis = np.argmin(t_hi, axis=1)
    positive = d[np.arange(n), axis] > 0
    sid = axis * 2 + positive.astype(np.int64)  # walls 0..5 (x-,x+,y-,y+,z- floor, z+ ceiling)
    best = s_room.copy()
    for bmin, bmax, ident in BOXES:
        t0 = (bmin - o) * inv
        t1 = (bmax - o) * inv
        tn = np.max(np.minimum(t0, t1), axis=1)
        tf = np.min(np.maximum(t0, t1), axis=1)
        hit = (tn <= tf) & (tn > 1e-6) & (tn < best)
        best = np.where(hit, tn, best)
        sid = np.where(hit, ident, sid)
    for cen, rad, ident in SPHERES:
        oc = o - cen
        a = np.einsum("ij,ij->i", d, d)
        b = 2.0 * (d @ oc)
        cc = oc @ oc - rad * rad
        disc = b * b - 4 * a * cc
        ok = disc >= 0
        sq = np.sqrt(np.where(ok, disc, 0.0))
        s0 = (-b - sq) / (2 * a)
        hit = ok & (s0 > 1e-6) & (s0 < best)
        best = np.where(hit, s0, best)
        sid = np.where(hit, ident, sid)
    pts = o + best[:, None] * d
    return best, sid, pts


_PALETTE = np.array(
    [[200, 190, 170], [190, 180, 160], [170, 180, 200], [160, 170, 190], [120, 100, 80],
     [230, 230, 230], [0, 0, 0], [150, 60, 40], [60, 120, 160], [90, 140, 70], [200, 60, 60],
     [230, 190, 40]], dtype=np.float64)
_TOUCH_BASE = np.array([0.05, 0.06, 0.04, 0.08, 0.15, 0.02, 0.0, 0.85, 0.6, 0.35, 0.9, 0.7])


TOUCH_MODES = ("complement", "independent", "u16", "u16z")
_LT_BASE = np.array([0.9, 0.3, 0.7, 0.35, 0.5, 0.95, 0.2, 0.1, 1.0, 0.6, 1e-6, 1e-6])
_U16_SCALE = np.float32(1.0 / 65535)  # cv::Mat::convertTo scale, a float in OpenCV's 16u -> 32f loop
_ONE_MINUS = np.float32(1.0 - 1e-6)
_BELOW_ONE = np.nextafter(np.float32(1.0), np.float32(0.0))


def _touch_fields(xp, pts, sid, wave, u1, u2, mode):
    """ht, lt (float32) of one frame for a non-default touch mode (module docstring). xp: numpy or torch; pts
    (N, 3) float64, sid (N,) int, wave the complement mode's field, u1 / u2 (N,) uniforms in [0, 1)."""
    def f32(a):
        return a.astype(np.float32) if xp is np else a.to(xp.float32)

    def const(v, like):
        return xp.full_like(like, float(v))

    def where(c, a, b):
        return xp.where(c, a, b)

    if mode not in TOUCH_MODES:
        raise ValueError(f"touch mode {mode!r} not in {TOUCH_MODES}")
    w2 = xp.sin(1.3 * pts[:, 0] - 2.9 * pts[:, 1] + 0.7 * pts[:, 2]) * xp.cos(3.7 * pts[:, 1] + 1.1 * pts[:, 2])
    hb = xp.asarray(_TOUCH_BASE)[sid] if xp is np else _TOUCH_BASE_T(xp, sid)
    lb = xp.asarray(_LT_BASE)[sid] if xp is np else xp.tensor(_LT_BASE, dtype=xp.float64, device=sid.device)[sid]
    ht = hb + 0.3 * wave
    lt = lb + 0.3 * w2
    ht = ht.clip(1e-6, 1.0) if xp is np else ht.clamp(1e-6, 1.0)
    lt = lt.clip(1e-6, 1.0) if xp is np else lt.clamp(1e-6, 1.0)
    ht, lt = f32(ht), f32(lt)
    # regions at the extremes (the orbit sees the cabinet, the x+ / y+ walls and, later, the shelf):
    # the cabinet ht = 1 - 1e-6, lt = 1e-6 (p -> 1 - 1e-6); the lowest 0.35 m of the walls ht = 1e-6,
    # lt = 1 (p -> 1e-6); a band of the walls 1.3-1.45 m high and sphere 11 ht = lt = 1e-6 (p stays
    # 0.5 from two tiny channels)
    z = pts[:, 2]
    wall = (sid == 1) | (sid == 3)
    low = wall & (z < 0.35)
    band = (wall & (z > 1.3) & (z < 1.45)) | (sid == 11)
    ht = where(sid == 8, const(_ONE_MINUS, ht), ht)
    lt = where(sid == 8, const(1e-6, lt), lt)
    ht = where(low | band, const(1e-6, ht), ht)
    lt = where(low, const(1.0, lt), lt)
    lt = where(band, const(1e-6, lt), lt)
    # sprinkled pixels at 1e-6, the largest float below 1 and exactly 1, per channel
    for ch, u in ((0, u1), (1, u2)):
        x = ht if ch == 0 else lt
        x = where(u < 0.004, const(1e-6, x), x)
        x = where((u >= 0.004) & (u < 0.008), const(_BELOW_ONE, x), x)
        x = where((u >= 0.008) & (u < 0.012), const(1.0, x), x)
        if ch == 0:
            ht = x
        else:
            lt = x
    if mode == "independent":
        return ht, lt

    # uint16 maps (rounded, as a PNG stores a network's probabilities), read back as f32(k) * f32(1/65535)
    def q16(x):
        k = (x.astype(np.float64) * 65535).round() if xp is np else (x.double() * 65535).round()
        return k.clip(0, 65535) if xp is np else k.clamp(0, 65535)

    kh, kl = q16(ht), q16(lt)
    kh = where(kh < 1, const(1, kh), kh)  # ht stays > 0 (zeros only where the mode asks)
    kl = where(kl < 1, const(1, kl), kl)
    # exact zeros in lt (the shelf, 12 cm strips every metre of the walls, 1 % of the pixels): p -> 1 exactly
    along = pts[:, 0] + pts[:, 1]  # along either wall (x or y is constant on it)
    strip = wall & ((along - (along // 1.0) * 1.0) < 0.12)
    kl = where((sid == 9) | strip | (u2 >= 0.990), const(0, kl), kl)
    if mode == "u16z":  # and in ht (8 cm strips between, 0.5 % of the pixels): p -> 0; where a
        # voxel sees both, ht = lt = 0 or p = 0 then lt = 0, the reference fuses 0 / 0 = NaN
        strip_h = wall & ((along + 0.5 - ((along + 0.5) // 1.0) * 1.0) < 0.08)
        kh = where(strip_h | (u1 >= 0.995), const(0, kh), kh)
    scale = float(_U16_SCALE)
    if xp is np:
        return (kh.astype(np.float32) * _U16_SCALE).astype(np.float32), (kl.astype(np.float32) * _U16_SCALE).astype(np.float32)
    return kh.to(xp.float32) * scale, kl.to(xp.float32) * scale


def _TOUCH_BASE_T(torch, sid):
    return torch.tensor(_TOUCH_BASE, dtype=torch.float64, device=sid.device)[sid]


def render(cam: Camera, frame: int, noise: bool = True, holes: float = 0.02, touch: str = "complement"):
    """Render frame `frame`: returns dict(rgb HxWx3 u8, depth HxW f32, ht, lt HxW f32, q, t)."""
    (R_wc, p), (q, t) = pose(frame)
    H, W = cam.height, cam.width
    u, v = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    dc = np.stack([(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, np.ones_like(u)], axis=-1)
    dw = dc.reshape(-1, 3) @ R_wc.T
    o = np.broadcast_to(p, dw.shape)
    s, sid, pts = _ray_scene(p, dw)  # s = depth along camera z because dc.z == 1
    rng = np.random.Generator(np.random.PCG64(SEED + frame))
    depth = s.copy()
    if noise:
        depth = depth + rng.normal(0.0, 0.001, size=depth.shape)
    depth = np.round(depth * DEPTH_FACTOR).clip(0, 65535).astype(np.uint16)
    depth = (depth.astype(np.float32) / np.float32(DEPTH_FACTOR)).astype(np.float32)
    depth[depth > MAX_RANGE] = 0.0
    if holes > 0:
        depth[rng.random(depth.shape) < holes] = 0.0
    # per-surface smooth touch field and checker colour
    wave = np.sin(3.1 * pts[:, 0] + 1.7 * pts[:, 1]) * np.cos(2.3 * pts[:, 2] + 0.4 * pts[:, 0])
    if touch == "complement":
        ht = np.clip(_TOUCH_BASE[sid] + 0.08 * wave, 0.02, 0.98).astype(np.float32)
        lt = (np.float32(1.0) - ht).astype(np.float32)
    else:  # its own generator: the depth noise and holes stay those of the complement stream
        trng = np.random.Generator(np.random.PCG64(SEED + 7919 * (frame + 1)))
        u1, u2 = trng.random(sid.shape), trng.random(sid.shape)
        ht, lt = _touch_fields(np, pts, sid, wave, u1, u2, touch)
    chk = ((np.floor(pts[:, 0] / 0.2) + np.floor(pts[:, 1] / 0.2) + np.floor(pts[:, 2] / 0.2)) % 2)
    shade = 0.75 + 0.25 * chk
    rgb = np.clip(_PALETTE[sid] * shade[:, None] + 10 * wave[:, None], 0, 255).astype(np.uint8)
    del o
    return dict(
        rgb=np.ascontiguousarray(rgb.reshape(H, W, 3)),
        depth=np.ascontiguousarray(depth.reshape(H, W)),
        ht=np.ascontiguousarray(ht.reshape(H, W)),
        lt=np.ascontiguousarray(lt.reshape(H, W)),
        q=q,
        t=t,
    )


def frames(cam: Camera, start: int, count: int, **kw):
    for f in range(start, start + count):
        yield render(cam, f, **kw)


def render_torch(cam: Camera, frame_ids, device="cuda", noise: bool = True, holes: float = 0.02,
                 seed: int = SEED, touch: str = "complement"):
    """Same scene rendered with torch on `device` (float64 geometry) for benchmark streams.

    Returns dict of stacked tensors: rgb (F,H,W,3) u8, depth/ht/lt (F,H,W) f32, and host numpy
    q (F,4) / t (F,3) float32 cam_T_world. Noise comes from a torch generator, so the frames are
    deterministic per (seed, frame) but not bit-identical to render(); parity tests use render().
    """
    import torch

    H, W = cam.height, cam.width
    F = len(frame_ids)
    dd = dict(device=device, dtype=torch.float64)
    v, u = torch.meshgrid(torch.arange(H, **dd), torch.arange(W, **dd), indexing="ij")
    dc = torch.stack([(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, torch.ones_like(u)], -1).reshape(-1, 3)
    out = dict(
        rgb=torch.empty((F, H, W, 3), dtype=torch.uint8, device=device),
        depth=torch.empty((F, H, W), dtype=torch.float32, device=device),
        ht=torch.empty((F, H, W), dtype=torch.float32, device=device),
        lt=torch.empty((F, H, W), dtype=torch.float32, device=device),
        q=np.zeros((F, 4), np.float32),
        t=np.zeros((F, 3), np.float32),
    )
    room_min = torch.tensor(ROOM_MIN, **dd)
    room_max = torch.tensor(ROOM_MAX, **dd)
    pal = torch.tensor(_PALETTE, **dd)
    touch_base = torch.tensor(_TOUCH_BASE, **dd)
    gen = torch.Generator(device=device)
    for k, f in enumerate(frame_ids):
        (R_wc, p), (q, t) = pose(f)
        out["q"][k], out["t"][k] = q, t
        d = dc @ torch.tensor(R_wc.T, **dd)
        o = torch.tensor(p, **dd)
        inv = torch.where(d.abs() > 1e-12, 1.0 / torch.where(d == 0, torch.ones_like(d), d),
                          torch.full_like(d, 1e12))
        t_hi = torch.maximum((room_min - o) * inv, (room_max - o) * inv)
        best, axis = t_hi.min(dim=1)
        positive = d.gather(1, axis[:, None])[:, 0] > 0
        sid = axis * 2 + positive.long()
        for bmin, bmax, ident in BOXES:
            t0 = (torch.tensor(bmin, **dd) - o) * inv
            t1 = (torch.tensor(bmax, **dd) - o) * inv
            tn = torch.minimum(t0, t1).max(dim=1).values
            tf = torch.maximum(t0, t1).min(dim=1).values
            hit = (tn <= tf) & (tn > 1e-6) & (tn < best)
            best = torch.where(hit, tn, best)
            sid = torch.where(hit, torch.full_like(sid, ident), sid)
        for cen, rad, ident in SPHERES:
            oc = o - torch.tensor(cen, **dd)
            a = (d * d).sum(1)
            b = 2.0 * (d @ oc)
            cc = (oc @ oc) - rad * rad
            disc = b * b - 4 * a * cc
            ok = disc >= 0
            sq = torch.sqrt(torch.where(ok, disc, torch.zeros_like(disc)))
            s0 = (-b - sq) / (2 * a)
            hit = ok & (s0 > 1e-6) & (s0 < best)
            best = torch.where(hit, s0, best)
            sid = torch.where(hit, torch.full_like(sid, ident), sid)
        pts = o + best[:, None] * d
        gen.manual_seed(seed + f)
        depth = best
        if noise:
            depth = depth + 0.001 * torch.randn(depth.shape, generator=gen, **dd)
        depth = torch.round(depth * DEPTH_FACTOR).clamp(0, 65535).to(torch.float32) / DEPTH_FACTOR
        depth[depth > MAX_RANGE] = 0.0
        if holes > 0:
            depth[torch.rand(depth.shape, generator=gen, **dd) < holes] = 0.0
        wave = torch.sin(3.1 * pts[:, 0] + 1.7 * pts[:, 1]) * torch.cos(2.3 * pts[:, 2] + 0.4 * pts[:, 0])
        if touch == "complement":
            ht = (touch_base[sid] + 0.08 * wave).clamp(0.02, 0.98).to(torch.float32)
            lt = (1.0 - ht)
        else:
            u1 = torch.rand(sid.shape, generator=gen, **dd)
            u2 = torch.rand(sid.shape, generator=gen, **dd)
            ht, lt = _touch_fields(torch, pts, sid, wave, u1, u2, touch)
        chk = torch.remainder(torch.floor(pts[:, 0] / 0.2) + torch.floor(pts[:, 1] / 0.2)
                              + torch.floor(pts[:, 2] / 0.2), 2)
        shade = 0.75 + 0.25 * chk
        rgb = (pal[sid] * shade[:, None] + 10 * wave[:, None]).clamp(0, 255).to(torch.uint8)
        out["depth"][k] = depth.reshape(H, W)
        out["ht"][k] = ht.reshape(H, W)
        out["lt"][k] = lt.reshape(H, W)
        out["rgb"][k] = rgb.reshape(H, W, 3)
    return out
