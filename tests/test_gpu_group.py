"""The library-owned sharded volume (tsdf_group_*, csrc/tsdf_group.hip; SURVEY.md 8b / 8e, VERDICT r5
next item 3): G shard engines in one process, the carve-candidate exchange done by the update kernels
themselves (each writes its slot into every shard's inbox), no collective and no caller-run exchange.
Checked against the UNSHARDED CPU oracle: the union of the shards equals it block for block and voxel
for voxel (tsdf, rgb, weight, probability bit-exact), the statistics, the Query voxels (as a set) and
the raycast images (bit-exact, through render replicas) -- at G = 2 and 8 shards on one GPU, with host
and device frames, heavy carving, and semantic input."""
import numpy as np
import pytest

from _shards import assert_union_equals

pytestmark = pytest.mark.gpu

MAXD = 4.0


def _run(G, W, H, voxel, trunc, frames, nb_bits, shard_bits, stride=1, device_frames=False, touch="complement",
         checks=()):
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    cam = synth.camera(W, H, synth.TUM_FR1)
    g = tsdf_amd.Group([0] * G, voxel, trunc, max_width=W, max_height=H, num_block_bits=shard_bits)
    ora = OracleGrid(voxel, trunc, nb_bits)
    try:
        for f in range(frames):
            fr = synth.render(cam, stride * f, touch=touch)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            if device_frames:
                dv = {k: torch.from_numpy(np.ascontiguousarray(fr[k])).cuda() for k in ("rgb", "depth", "ht", "lt")}
                g.integrate(dv["rgb"], dv["depth"], dv["ht"], dv["lt"], cam.K, pose, MAXD)
            else:
                g.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD)
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], MAXD, cam.K, fr["q"], fr["t"])
            if f in checks or f == frames - 1:
                s, so = g.stats(), ora.stats()  # (completes the pending frames)
                assert s["status"] == 0, s
                assert s["active_blocks"] == so["active_blocks"], (f, s, so)
                assert s["last_num_visible"] == so["last_num_visible"], (f, s, so)
                assert s["last_num_updated"] == so["last_num_updated"], (f, s, so)
                full = ora.dump()
                nb = assert_union_equals([g.shard_dump(i) for i in range(G)], full, tag=f"G={G} frame {f}")
                assert nb == so["active_blocks"]
        return g, ora, cam
    except Exception:
        g.close(), ora.close()
        raise


@pytest.mark.parametrize("G", [1, 2, 8])
def test_group_c3_union_equals_unsharded(G):
    """(G = 1: one unsharded engine behind the group calls.)"""
    g, ora, cam = _run(G, 640, 480, 0.005, 0.03, 8, 18, 16, stride=2, checks=(3,))
    g.close(), ora.close()


def test_group_device_frames_semantic_heavy_carving():
    """2 cm voxels (blocks carved every frame), segmentation-shaped ht / lt with exact zeros, device
    frames, 4 shards."""
    g, ora, cam = _run(4, 96, 72, 0.02, 0.08, 12, 14, 13, device_frames=True, touch="u16z", checks=(4, 8))
    g.close(), ora.close()


def test_group_query_and_raycast_equal_unsharded():
    import tsdf_amd
    from tsdf_amd import synth
    g, ora, cam = _run(3, 160, 120, 0.01, 0.04, 10, 15, 14, stride=3)
    try:
        got = g.query(None)
        exp = ora.query(None)
        assert got.shape[0] == exp.shape[0] > 0
        a = np.sort(np.stack([got[k] for k in ("x", "y", "z", "tsdf")], 1).view(np.uint32).view("V16").ravel())
        b = np.sort(np.ascontiguousarray(exp[:, :4]).view(np.uint32).view("V16").ravel())
        assert np.array_equal(a, b)
        for f in (7, 27):
            (_, _), (q, t) = synth.pose(f)
            rgba, nrm = g.raycast(cam.K, cam.width, cam.height, tsdf_amd.SE3(q, t), MAXD)
            ro, no = ora.raycast(cam.K, cam.width, cam.height, q, t, MAXD)
            assert (rgba[..., 3] == 255).mean() > 0.5
            np.testing.assert_array_equal(rgba, ro)
            np.testing.assert_array_equal(nrm, no)
        # integrating on after the reads (a fresh pipeline) stays equal
        for f in range(30, 36, 2):
            fr = synth.render(cam, f)
            g.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], MAXD, cam.K, fr["q"], fr["t"])
        assert_union_equals([g.shard_dump(i) for i in range(3)], ora.dump(), tag="after reads")
    finally:
        g.close(), ora.close()


def test_group_argument_errors():
    import ctypes as C

    import tsdf_amd
    from tsdf_amd import _lib
    L = _lib.load()
    cfg = _lib.Config()
    L.tsdf_config_default(C.byref(cfg))
    h = C.c_void_p()
    assert L.tsdf_group_create(C.byref(cfg), None, 2, C.byref(h)) == 1  # TSDF_ERR_INVALID_ARG
    devs = (C.c_int * 1)(0)
    assert L.tsdf_group_create(C.byref(cfg), devs, 0, C.byref(h)) == 1  # TSDF_ERR_INVALID_ARG
    g = tsdf_amd.Group([0, 0], 0.01, 0.04, max_width=64, max_height=48, num_block_bits=10)
    try:
        fr = _lib.Frame(128, 96, None, None, None, None, 0)  # larger than the group's maximum
        K = _lib.Intrinsics(50.0, 50.0, 32.0, 24.0)
        assert L.tsdf_group_integrate(g._g, C.byref(fr), C.byref(K), C.byref(tsdf_amd.SE3()._c()),
                                      4.0) == 1  # TSDF_ERR_INVALID_ARG
        assert L.tsdf_group_size(g._g) == 2
        assert g.stats()["status"] == 0
    finally:
        g.close()


def test_group_device_frame_buffers_reused_on_torch_stream():
    """Device frames in ONE set of tensors, overwritten on torch's stream right after every
    tsdf_group_integrate (the group reads them on its own streams after the call returns; Group orders
    torch's stream after that work with tsdf_group_stream_signal): the union still equals the oracle."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    W, H = 160, 120
    cam = synth.camera(W, H, synth.TUM_FR1)
    g = tsdf_amd.Group([0, 0], 0.01, 0.04, max_width=W, max_height=H, num_block_bits=15)
    ora = OracleGrid(0.01, 0.04, 16)
    try:
        frames = [synth.render(cam, 2 * f, touch="independent") for f in range(10)]
        dv = {k: torch.from_numpy(np.ascontiguousarray(frames[0][k])).cuda() for k in ("rgb", "depth", "ht", "lt")}
        junk = {k: torch.full_like(v, 7) for k, v in dv.items()}
        for f, fr in enumerate(frames):
            for k in dv:
                dv[k].copy_(torch.from_numpy(np.ascontiguousarray(fr[k])).cuda())
            g.integrate(dv["rgb"], dv["depth"], dv["ht"], dv["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
            for k in dv:  # overwrite at once, on torch's stream (ordered after the group's reads)
                dv[k].copy_(junk[k])
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], MAXD, cam.K, fr["q"], fr["t"])
        s, so = g.stats(), ora.stats()
        assert s["status"] == 0 and s["active_blocks"] == so["active_blocks"], (s, so)
        assert_union_equals([g.shard_dump(i) for i in range(2)], ora.dump(), tag="reused buffers")
    finally:
        g.close(), ora.close()
