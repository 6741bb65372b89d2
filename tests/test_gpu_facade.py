"""The C++17 facade (TSDFSystem queue + worker thread -> TSDFGrid -> C ABI) against the oracle.

disinfect-slam_amd/facade_main is built with plain g++ against include/disinfect_tsdf.h only.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "disinfect-slam_amd", "facade_main")


@pytest.mark.parametrize("semantic,shards", [(True, 1), (False, 1), (True, 2), (True, 5)])
def test_tsdf_system_matches_oracle(tmp_path, semantic, shards):
    """shards > 1: TSDFSystem over a volume sharded across that many shards of one GPU (the C++
    group constructor, tsdf_group_*): the same voxels (shard by shard, compared as a set), statistics
    and images as the unsharded oracle."""
    from tsdf_amd import synth
    from _oracle import OracleGrid
    W, H, n, voxel, trunc, nb = 96, 72, 5, 0.005, 0.03, 13
    cam = synth.camera(W, H)
    ora = OracleGrid(voxel, trunc, nb)
    k32 = " ".join(repr(float(v)) for v in cam.K)  # float32 values, exact in decimal
    lines = [f"{W} {H} {n} {k32} {voxel} {trunc} 4.0 {int(semantic)} {nb}"]
    for i in range(n):
        fr = synth.render(cam, i)
        for k in ("rgb", "depth", "ht", "lt"):
            fr[k].tofile(tmp_path / f"f{i}_{k}.bin")
        lines.append(" ".join(repr(float(v)) for v in list(fr["q"]) + list(fr["t"])))
        ora.integrate(fr["rgb"], fr["depth"], fr["ht"] if semantic else None,
                      fr["lt"] if semantic else None, 4.0, cam.K, fr["q"], fr["t"])
    (tmp_path / "meta.txt").write_text("\n".join(lines) + "\n")
    r = subprocess.run([BIN, str(tmp_path), str(shards)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(tmp_path / "out_query.bin", np.float32).reshape(-1, 4)
    exp = ora.query(None)
    assert got.shape == exp.shape and got.shape[0] > 0
    if shards > 1:  # shard by shard: the same set of voxels
        got = np.sort(np.ascontiguousarray(got).view(np.uint32).view("V16").ravel())
        exp = np.sort(np.ascontiguousarray(exp).view(np.uint32).view("V16").ravel())
        assert np.array_equal(got, exp)
    else:
        np.testing.assert_array_equal(got[:, :3], exp[:, :3])
        np.testing.assert_array_equal(got[:, 3].view(np.uint32), exp[:, 3].view(np.uint32))
    frames, active, nvis, nupd, status = map(int, (tmp_path / "out_stats.txt").read_text().split())
    so = ora.stats()
    assert (frames, active, nvis, nupd, status) == (n, so["active_blocks"], so["last_num_visible"],
                                                    so["last_num_updated"], 0)
    (_, _), (q, t) = synth.pose(n - 1)
    _, nrm = ora.raycast(cam.K, W, H, q, t, 4.0)
    got_n = np.fromfile(tmp_path / "out_render.bin", np.uint8).reshape(H, W, 4)
    np.testing.assert_array_equal(got_n, nrm)
    ora.close()


def test_disinf_system_feed_rgbd_frame(tmp_path):
    """DISINFSystem (host/disinfect_slam.h): poses registered at tracker timestamps, raw 16-bit
    sensor frames fed at their own timestamps (nearest pose, pose_manager.cc) and preprocessed on the
    GPU (x0.5 resize, depth scale, mask) == the oracle fed the same preprocessing + poses."""
    from tsdf_amd import synth
    from _oracle import OracleGrid, rgbd_half
    from test_host_cpu import ref_query
    W, H, n, voxel, trunc, nb, factor = 192, 144, 5, 0.01, 0.04, 13, 5000.0
    full = synth.camera(W, H)
    half = synth.camera(W // 2, H // 2)
    rng = np.random.default_rng(5)
    reg = []
    for i in range(2 * n + 2):  # tracker poses every 33 ms
        (_, _), (q, t) = synth.pose(i)
        reg.append((1000 + 33 * i, tuple(float(v) for v in list(q) + list(t))))
    ora = OracleGrid(voxel, trunc, nb)
    k32 = " ".join(repr(float(v)) for v in half.K)
    lines = [f"{W} {H} {n} {len(reg)} {k32} {voxel} {trunc} 4.0 {factor} {nb}"]
    lines += [f"{ts} " + " ".join(repr(v) for v in p) for ts, p in reg]
    for i in range(n):
        ts = 1000 + 66 * i + int(rng.integers(-14, 15))  # the depth stream's own clock
        fr = synth.render(full, 2 * i)
        d16 = np.round(fr["depth"] * factor).astype(np.uint16)
        mask = (rng.random((H, W)) < 0.85).astype(np.uint8) if i % 2 else None
        fr["rgb"].tofile(tmp_path / f"f{i}_rgb.bin")
        d16.tofile(tmp_path / f"f{i}_depth.bin")
        if mask is not None:
            mask.tofile(tmp_path / f"f{i}_mask.bin")
        lines.append(f"{ts} {int(mask is not None)}")
        p = ref_query(reg, ts)
        r2, dd = rgbd_half(fr["rgb"], d16, mask, factor)
        ora.integrate(r2, dd, None, None, 4.0, half.K, np.float32(p[:4]), np.float32(p[4:]))
    (tmp_path / "meta.txt").write_text("\n".join(lines) + "\n")
    binp = os.path.join(ROOT, "disinfect-slam_amd", "disinfect_main")
    r = subprocess.run([binp, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(tmp_path / "out_query.bin", np.float32).reshape(-1, 4)
    exp = ora.query(np.array([-1e4, 1e4, -1e4, 1e4, -1e4, 1e4], np.float32))
    assert got.shape == exp.shape and got.shape[0] > 0
    np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))
    frames, active, status = map(int, (tmp_path / "out_stats.txt").read_text().split())
    assert (frames, active, status) == (n, ora.stats()["active_blocks"], 0)
    ora.close()


@pytest.mark.parametrize("semantic", [True, False])
def test_offline_replay_matches_oracle(tmp_path, semantic):
    """examples/tsdf/offline.cc's loop (host/offline_log.cc + TSDFGrid via offline_main): a log
    directory of PNG frames + trajectory.txt replayed on the GPU == the oracle fed the decoded
    frames (absent ht maps read as ht = 0, lt = 1, offline.cc:80-81)."""
    from _oracle import OracleGrid
    from _png import se3_from_matrix
    from test_host_cpu import _write_log, expected_frame
    cam, frames = _write_log(tmp_path, n=4, W=96, H=72, semantic=semantic)
    ora = OracleGrid(0.01, 0.04, 13)
    for f in frames:
        rgb, depth, ht, lt = expected_frame(f)
        q, t = se3_from_matrix(f["m"])
        ora.integrate(rgb, depth, ht, lt, 4.0, cam.K, q, t)
    binp = os.path.join(ROOT, "disinfect-slam_amd", "offline_main")
    K = [repr(float(v)) for v in cam.K]
    r = subprocess.run([binp, str(tmp_path), *K, "5000", "0.01", "0.04", "13"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(tmp_path / "out_query.bin", np.float32).reshape(-1, 4)
    exp = ora.query(None)
    assert got.shape == exp.shape and got.shape[0] > 0
    np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))
    frames_n, active, status = map(int, (tmp_path / "out_stats.txt").read_text().split())
    assert (frames_n, active, status) == (len(frames), ora.stats()["active_blocks"], 0)
    ora.close()
