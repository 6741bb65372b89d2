"""DISINFSystem::feed_rgbd_frame on the GPU: the x0.5 resize of rgb / depth /
mask, the depth scale and the mask -> depth 0 loop (tsdf_rgbd_half), and the whole feed (that
preprocessing + TSDFGrid::Integrate with ht = lt = ones) against the CPU oracle, bit for bit.
OpenCV is absent here, so the resize is pinned only by the oracle's restatement of OpenCV's
published fast 2x2 area path (oracle/tsdf_oracle.c ora_rgbd_half): parity unpinned beyond it.
"""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def random_rgbd(rng, W, H, with_mask=True):
    rgb = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    depth = rng.integers(0, 65536, size=(H, W), dtype=np.uint16)
    depth[rng.random((H, W)) < 0.05] = 0
    mask = None
    if with_mask:
        mask = (rng.random((H, W)) < 0.7).astype(np.uint8) * rng.integers(1, 256, size=(H, W), dtype=np.uint8)
        mask[:2, :2] = [[1, 0], [0, 0]]  # (1 + 2) >> 2 == 0: masked
    return rgb, depth, mask


@pytest.mark.parametrize("W,H,with_mask,factor", [(64, 48, True, 5000.0), (1280, 720, True, 4000.0),
                                                  (642, 482, False, 1000.0), (2, 2, True, 5000.0)])
def test_rgbd_half_matches_oracle(W, H, with_mask, factor):
    import torch

    import tsdf_amd
    from _oracle import rgbd_half
    rng = np.random.default_rng(W * H)
    rgb, depth, mask = random_rgbd(rng, W, H, with_mask)
    exp_rgb, exp_d = rgbd_half(rgb, depth, mask, factor)
    with tsdf_amd.Engine(0.01, 0.04, max_width=max(W // 2, 16), max_height=max(H // 2, 16),
                         num_block_bits=10) as eng:
        got_rgb, got_d = eng.rgbd_half(rgb, depth, mask, factor)  # host buffers
        np.testing.assert_array_equal(got_rgb, exp_rgb)
        np.testing.assert_array_equal(got_d.view(np.uint32), exp_d.view(np.uint32))
        dev = torch.device("cuda")
        t = [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rgb, depth.view(np.int16), mask)]
        g_rgb, g_d = eng.rgbd_half(t[0], t[1], t[2], factor)  # device buffers
        torch.cuda.synchronize()
        np.testing.assert_array_equal(g_rgb.cpu().numpy(), exp_rgb)
        np.testing.assert_array_equal(g_d.cpu().numpy().view(np.uint32), exp_d.view(np.uint32))
    if with_mask:
        assert exp_d[0, 0] == 0.0


def test_rgbd_half_rejects_odd_sizes():
    import tsdf_amd
    rng = np.random.default_rng(0)
    rgb, depth, _ = random_rgbd(rng, 63, 48, False)
    with tsdf_amd.Engine(0.01, 0.04, max_width=64, max_height=64, num_block_bits=10) as eng:
        with pytest.raises(tsdf_amd.TSDFError):
            eng.rgbd_half(rgb, depth, None, 5000.0)


def test_feed_rgbd_frame_matches_oracle():
    """Full-resolution 16-bit sensor frames (TUM depth factor 5000) fed through the GPU front end
    equal the oracle's preprocessing + integrate."""
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid, rgbd_half
    W, H, factor = 192, 144, 5000.0
    full = synth.camera(W, H, synth.TUM_FR1)
    half = synth.camera(W // 2, H // 2, synth.TUM_FR1)
    rng = np.random.default_rng(7)
    eng = tsdf_amd.Engine(0.01, 0.04, max_width=W // 2, max_height=H // 2, num_block_bits=13)
    ora = OracleGrid(0.01, 0.04, 13)
    try:
        for f in range(5):
            fr = synth.render(full, 2 * f)
            d16 = np.round(fr["depth"] * factor).astype(np.uint16)  # the sensor's raw depth
            mask = (rng.random((H, W)) < 0.9).astype(np.uint8) if f % 2 else None
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            eng.feed_rgbd_frame(fr["rgb"], d16, mask, factor, half.K, pose, 4.0)
            r2, d2 = rgbd_half(fr["rgb"], d16, mask, factor)
            ora.integrate(r2, d2, None, None, 4.0, half.K, fr["q"], fr["t"])
            s, so = eng.stats(), ora.stats()
            assert s["status"] == 0
            assert s["active_blocks"] == so["active_blocks"] > 0
        compare(eng, ora, tag="feed_rgbd_frame")
    finally:
        eng.close(), ora.close()
