"""Edge cases of the integrate path against the CPU oracle:

 - ragged image sizes (not multiples of the 16x16 pixel tile, narrow and tall);
 - frames with no usable depth (all holes, all beyond max_depth, half holes): nothing is
   allocated or updated, but the visible blocks are still carve-tested (voxel_tsdf.cu:207-230);
 - a camera looking away from everything allocated (no visible blocks);
 - the reference's largest frame, MAX_IMG = 1920x1080 (voxel_tsdf.cu:10-12), and frames larger
   than the engine was sized for (rejected, volume untouched);
 - device-resident (torch) frames give the same volume as host frames.
Entries, pool indices, free stack, tsdf, colour, weight and probability bit-exact.
"""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _pair(W, H, voxel=0.005, trunc=0.03, nb=14, intr=None):
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    cam = synth.camera(W, H, intr or synth.TUM_FR1)
    return (tsdf_amd.Engine(voxel, trunc, max_width=W, max_height=H, num_block_bits=nb),
            OracleGrid(voxel, trunc, nb), cam)


def _step(eng, ora, cam, fr, q=None, t=None, tag=""):
    import tsdf_amd
    q = fr["q"] if q is None else q
    t = fr["t"] if t is None else t
    eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(q, t), 4.0)
    ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, q, t)
    s, so = eng.stats(), ora.stats()
    assert s["status"] == 0, (tag, s)
    for k in ("last_num_visible", "last_num_updated", "last_num_deleted", "active_blocks"):
        assert s[k] == so[k], (tag, k, s, so)
    return s


@pytest.mark.parametrize("W,H", [(100, 75), (37, 29), (24, 200)])
def test_ragged_image_sizes(W, H):
    from tsdf_amd import synth
    eng, ora, cam = _pair(W, H)
    try:
        for f in range(4):
            _step(eng, ora, cam, synth.render(cam, 3 * f), tag=f"{W}x{H} frame {f}")
        assert eng.stats()["active_blocks"] > 0
        compare(eng, ora, tag=f"{W}x{H}")
    finally:
        eng.close(), ora.close()


def test_frames_without_usable_depth_and_looking_away():
    from tsdf_amd import synth
    eng, ora, cam = _pair(128, 96, voxel=0.01, trunc=0.04, nb=14)
    try:
        for f in range(3):
            _step(eng, ora, cam, synth.render(cam, 2 * f), tag=f"frame {f}")
        before = eng.stats()["active_blocks"]
        assert before > 0
        fr = synth.render(cam, 6)
        holes = dict(fr, depth=np.zeros_like(fr["depth"]))
        s = _step(eng, ora, cam, holes, tag="all holes")
        assert s["last_num_updated"] == 0 and s["last_num_visible"] > 0
        compare(eng, ora, tag="all holes")
        far = dict(fr, depth=np.full_like(fr["depth"], 5.0))  # every pixel beyond max_depth = 4
        s = _step(eng, ora, cam, far, tag="beyond max_depth")
        assert s["last_num_updated"] == 0
        compare(eng, ora, tag="beyond max_depth")
        half = dict(fr, depth=np.where(np.arange(fr["depth"].shape[1])[None, :] < 64, fr["depth"], 0.0)
                    .astype(np.float32))
        s = _step(eng, ora, cam, half, tag="half holes")
        assert s["last_num_updated"] > 0
        # looking straight away from the scene: a camera 100 m outside it (no block in view)
        s = _step(eng, ora, cam, dict(fr, depth=np.zeros_like(fr["depth"])), q=fr["q"],
                  t=np.array([1000.0, 1000.0, 1000.0], np.float32), tag="looking away")
        assert s["last_num_visible"] == 0 and s["last_num_deleted"] == 0
        _step(eng, ora, cam, synth.render(cam, 8), tag="normal again")
        compare(eng, ora, tag="after edge frames")
    finally:
        eng.close(), ora.close()


def test_max_image_1920x1080_and_oversized_frames():
    import tsdf_amd
    from tsdf_amd import synth
    eng, ora, cam = _pair(1920, 1080, intr=synth.L515_FULL, nb=16)
    try:
        for f in range(2):
            _step(eng, ora, cam, synth.render(cam, 4 * f), tag=f"1080p frame {f}")
        s = eng.stats()
        assert s["active_blocks"] > 3000
        compare(eng, ora, tag="1920x1080")
        big = synth.camera(1936, 1080, synth.L515_FULL)
        fr = synth.render(big, 0)
        with pytest.raises(tsdf_amd.TSDFError):
            eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], big.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
        assert eng.stats()["active_blocks"] == s["active_blocks"]
        compare(eng, ora, pool=False, tag="after the rejected frame")
    finally:
        eng.close(), ora.close()


def test_device_frames_match_host_frames():
    """Host frames (pageable numpy, then pinned torch, alternating: the engine's two upload slots are
    each reused several times while the pipelined frames before them run) equal device frames; the
    host buffers are overwritten right after each call (the upload is complete on return)."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H = 160, 120
    cam = synth.camera(W, H, synth.TUM_FR1)
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=14)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=14)
    try:
        for f in range(10):
            fr = synth.render(cam, 2 * f)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            if f % 2:
                hf = {k: torch.from_numpy(np.ascontiguousarray(fr[k])).pin_memory() for k in ("rgb", "depth", "ht", "lt")}
            else:
                hf = {k: np.array(fr[k], copy=True) for k in ("rgb", "depth", "ht", "lt")}
            a.integrate(hf["rgb"], hf["depth"], hf["ht"], hf["lt"], cam.K, pose, 4.0)
            for k in hf:  # (the caller may reuse its buffers at once)
                hf[k][...] = 0
            dv = {k: torch.from_numpy(np.ascontiguousarray(fr[k])).cuda() for k in ("rgb", "depth", "ht", "lt")}
            b.integrate(dv["rgb"], dv["depth"], dv["ht"], dv["lt"], cam.K, pose, 4.0)
        b.synchronize()
        da, db = a.dump(), b.dump()
        for k in ("entry_pos", "entry_idx", "heap", "rgbw"):
            assert np.array_equal(da[k], db[k]), k
        for k in ("tsdf", "prob"):
            assert np.array_equal(da[k].view(np.uint32), db[k].view(np.uint32)), k
    finally:
        a.close(), b.close()


def test_null_arguments_return_invalid_arg():
    """tsdf_integrate with a NULL frame, camera or pose returns TSDF_ERR_INVALID_ARG
    (checked before the pipelining test reads the frame size) and leaves the engine usable."""
    import ctypes as C

    import tsdf_amd
    from tsdf_amd import _lib, synth
    L = _lib.load()
    cam = synth.camera(64, 48, synth.TUM_FR1)
    eng = tsdf_amd.Engine(0.01, 0.04, max_width=64, max_height=48, num_block_bits=14)
    try:
        K = _lib.Intrinsics(*[float(v) for v in cam.K])
        pose = _lib.Pose(0, 0, 0, 1, 0, 0, 0)
        fr = _lib.Frame(64, 48, None, None, None, None, 0)
        assert L.tsdf_integrate(eng._h, None, C.byref(K), C.byref(pose), 4.0) == 1
        assert L.tsdf_integrate(eng._h, C.byref(fr), None, C.byref(pose), 4.0) == 1
        assert L.tsdf_integrate(eng._h, C.byref(fr), C.byref(K), None, 4.0) == 1
        assert L.tsdf_integrate(None, C.byref(fr), C.byref(K), C.byref(pose), 4.0) == 1
        f = synth.render(cam, 0)
        eng.integrate(f["rgb"], f["depth"], f["ht"], f["lt"], cam.K, tsdf_amd.SE3(f["q"], f["t"]), 4.0)
        assert eng.stats()["status"] == 0 and eng.stats()["active_blocks"] > 0
    finally:
        eng.close()
