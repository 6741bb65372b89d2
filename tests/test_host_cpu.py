"""Host-side (CPU, no GPU) pieces of the drop-in: the C++ pose_manager (utils/rotation_math/
pose_manager.cc) against a Python restatement of the reference's lookup, and the oracle's restatement
of DISINFSystem::feed_rgbd_frame's preprocessing against numpy (OpenCV's fast 2x2 area path; parity
with OpenCV itself unpinned -- it is not installed)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "disinfect-slam_amd", "host")


@pytest.fixture(scope="module")
def pose_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("pm") / "pose_manager_main")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I" + HOST, "-o", out,
                           os.path.join(HOST, "pose_manager.cc"), os.path.join(HOST, "tests", "pose_manager_main.cc"),
                           "-lpthread"])
    return out


def ref_query(reg, ts):
    """pose_manager.cc:16-66 (nearest registered pose; identity when empty; first pose before the
    first timestamp, where the reference reads element -1)."""
    if not reg:
        return (0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0)
    stamps = [r[0] for r in reg]
    lo = int(np.searchsorted(stamps, ts, side="right")) - 1
    if lo < 0:
        return reg[0][1]
    if lo == len(reg) - 1:
        return reg[lo][1]
    return reg[lo][1] if (ts - stamps[lo]) < (stamps[lo + 1] - ts) else reg[lo + 1][1]


def test_pose_manager_nearest_lookup(pose_bin):
    rng = np.random.default_rng(3)
    stamps = np.cumsum(rng.integers(1, 60, size=120)) + 1000
    reg = [(int(t), tuple(float(np.float32(v)) for v in rng.normal(size=7))) for t in stamps]
    queries = [0, 999, 1000, int(stamps[0]), int(stamps[-1]), int(stamps[-1]) + 500]
    queries += [int(t) for t in rng.integers(900, int(stamps[-1]) + 100, size=300)]
    queries += [int((a + b) // 2) for a, b in zip(stamps[:-1], stamps[1:])]  # ties go to the newer
    lines = ["Q 5"]  # empty manager -> identity
    lines += [f"R {t} " + " ".join(repr(v) for v in p) for t, p in reg]
    lines += [f"Q {q}" for q in queries]
    out = subprocess.run([pose_bin], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split("\n")
    got = [tuple(map(float, l.split())) for l in out if l.strip()]
    assert got[0] == (0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0)
    for q, g in zip(queries, got[1:]):
        np.testing.assert_array_equal(np.float32(g), np.float32(ref_query(reg, q)), err_msg=str(q))
    assert len(got) == len(queries) + 1


def test_oracle_rgbd_half_formula():
    from _oracle import rgbd_half
    rng = np.random.default_rng(11)
    H, W = 36, 50
    rgb = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    d = rng.integers(0, 65536, size=(H, W), dtype=np.uint16)
    m = (rng.random((H, W)) < 0.5).astype(np.uint8)
    r2, d2 = rgbd_half(rgb, d, m, 5000.0)
    blk = lambda a: a.reshape(H // 2, 2, W // 2, 2, *a.shape[2:]).astype(np.int64).sum(axis=(1, 3))
    np.testing.assert_array_equal(r2, ((blk(rgb) + 2) >> 2).astype(np.uint8))
    dv = ((blk(d) + 2) >> 2).astype(np.float32) * np.float32(1.0 / 5000.0)
    dv[((blk(m) + 2) >> 2) == 0] = 0.0
    np.testing.assert_array_equal(d2.view(np.uint32), dv.astype(np.float32).view(np.uint32))
    # ties round up: 1 + 1 + 0 + 0 -> (2 + 2) >> 2 == 1
    one = np.zeros((2, 2, 3), np.uint8)
    one[0, :, :] = 1
    assert rgbd_half(one, np.zeros((2, 2), np.uint16), None, 1.0)[0][0, 0, 0] == 1


def _write_log(d, n=3, W=48, H=36, semantic=True, seed=0):
    """A synthetic offline log (examples/tsdf/offline.cc format) of the analytic room."""
    from _png import write_png
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    rng = np.random.default_rng(seed)
    lines, frames = [], []
    for i in range(n):
        fr = synth.render(cam, 3 * i)
        fid = 100 + 7 * i
        (R_wc, p), (_, _) = synth.pose(3 * i)
        R_cw = R_wc.T
        t_cw = -R_cw @ p
        m = np.concatenate([R_cw, t_cw[:, None]], 1).astype(np.float32)
        lines.append(f"{fid} " + " ".join(repr(float(v)) for v in m.reshape(-1)))
        d16 = np.round(fr["depth"] * 5000).astype(np.uint16)
        rgb = fr["rgb"]
        if i == 1:  # an RGBA frame: imread(IMREAD_COLOR) drops alpha
            rgb = np.concatenate([rgb, rng.integers(0, 256, (H, W, 1), dtype=np.uint8)], 2)
        write_png(d / f"{fid}_rgb.png", rgb)
        write_png(d / f"{fid}_depth.png", d16, filters=(4, 3, 2, 1, 0))
        ht16 = lt16 = None
        if semantic:
            ht16 = np.round(fr["ht"] * 65535).astype(np.uint16)
            lt16 = np.round(fr["lt"] * 65535).astype(np.uint16)
            write_png(d / f"{fid}_ht.png", ht16)
            write_png(d / f"{fid}_no_ht.png", lt16, filters=(2, 4))
        frames.append(dict(id=fid, m=m, rgb=fr["rgb"], d16=d16, ht16=ht16, lt16=lt16))
    (d / "trajectory.txt").write_text("\n".join(lines) + "\n")
    return cam, frames


def expected_frame(f):
    """get_images_by_id (offline.cc:65-83) on the frames the log holds."""
    depth = f["d16"].astype(np.float32) * np.float32(1.0 / 5000.0)
    if f["ht16"] is None:
        ht = np.zeros_like(depth)
        lt = np.ones_like(depth)
    else:
        ht = f["ht16"].astype(np.float32) * np.float32(1.0 / 65535)
        lt = f["lt16"].astype(np.float32) * np.float32(1.0 / 65535)
    return f["rgb"], depth, ht, lt


@pytest.mark.parametrize("semantic", [True, False])
def test_offline_log_decoding(tmp_path, semantic):
    """host/offline_log.cc: trajectory parsing (3x4 -> SE3 as Eigen does) and the PNG decoder (all
    five scanline filters, RGB / RGBA / 16-bit grey) against the frames written."""
    from _png import se3_from_matrix
    out = str(tmp_path / "offline_decode")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-DOFFLINE_DECODE_ONLY", "-I" + HOST,
                           "-I" + os.path.join(ROOT, "include"), "-o", out, os.path.join(HOST, "offline_log.cc"),
                           os.path.join(HOST, "tests", "offline_main.cc"), "-lz"])
    cam, frames = _write_log(tmp_path, semantic=semantic)
    subprocess.check_call([out, str(tmp_path), "1", "1", "0", "0", "5000", "0.01", "0.04", "10"])
    poses = [l.split() for l in (tmp_path / "poses.txt").read_text().splitlines()]
    assert len(poses) == len(frames)
    H, W = frames[0]["d16"].shape
    for i, (f, p) in enumerate(zip(frames, poses)):
        q, t = se3_from_matrix(f["m"])
        assert int(p[0]) == f["id"]
        np.testing.assert_array_equal(np.float32([float(v) for v in p[1:]]), np.concatenate([q, t]))
        rgb, depth, ht, lt = expected_frame(f)
        got = lambda k, dt: np.fromfile(tmp_path / f"f{i}_{k}.dec", dt)
        np.testing.assert_array_equal(got("rgb", np.uint8).reshape(H, W, 3), rgb)
        for k, v in (("depth", depth), ("ht", ht), ("lt", lt)):
            np.testing.assert_array_equal(got(k, np.uint32), v.reshape(-1).view(np.uint32), err_msg=k)
