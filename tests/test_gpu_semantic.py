"""Semantic fusion on segmentation-shaped input (Missing 3 / next item 1).

The reference feeds TSDFGrid::Integrate two independent network channels (examples/tsdf/online.cc:59-60,
segmentation/inference.cc:57-65) or uint16 PNG maps read with convertTo(CV_32FC1, 1 / 65535)
(examples/tsdf/offline.cc:76-82), which are exactly 0 where the network is certain; the update
(voxel_tsdf.cu:196-202) is expf((w_old logf(p) + w_new logf(ht)) / wc) / (... + ...). The engine runs
that float chain operation for operation with the oracle's logf / expf (oracle/ora_math.c), so the
probability is compared BIT FOR BIT here (NaN == NaN where the reference's own arithmetic gives 0 / 0:
a voxel that sees ht = lt = 0, or p = 0 then lt = 0 -- input the reference leaves undefined), and the
raycast images (colour blends with p) exactly. Streams (tsdf_amd.synth touch modes):
  independent -- two independent fields over (0, 1], regions and sprinkled pixels at 1e-6, 1 - 1e-6,
                 the largest float below 1 and 1 (p driven to within 1e-6 of 1 and of 0, where the
                 reference's float chain is ill-conditioned);
  u16         -- those fields as uint16 / 65535 maps, exact zeros in lt (p becomes exactly 1);
  u16z        -- and exact zeros in ht too (p exactly 0, and NaN where both meet).
C3 at full size (640 x 480, 5 mm, 2^18 pool) over 120 frames of the bench orbit, integrated back to
back (pipelined k_frame launches), so much of the surface reaches the weight cap (40); and 160 x 120
streams compared after every frame.
"""
import numpy as np
import pytest

from test_gpu_parity import compare, prob_equal, run_sequence

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("touch", ["independent", "u16", "u16z"])
def test_semantic_160x120_every_frame(touch):
    eng, ora, cam = run_sequence(160, 120, 0.005, 0.03, 12, touch=touch, check_every=1)
    try:
        d = eng.dump()
        live = d["entry_idx"][d["entry_idx"] >= 0]
        p = d["prob"].reshape(-1, 512)[live]
        w = d["rgbw"].reshape(-1, 512, 4)[live, :, 3]
        seen = p[w > 0]
        if touch == "independent":
            assert np.isfinite(seen).all()
            assert (seen > 1 - 1e-5).sum() > 100 and (seen < 1e-5).sum() > 100
        else:
            assert (seen == 1).sum() > 100
        if touch == "u16z":
            assert (seen == 0).sum() > 100 and np.isnan(seen).sum() > 0
        from tsdf_amd import synth
        import tsdf_amd
        (_, _), (q, t) = synth.pose(11)
        rgba, nrm = eng.raycast(cam.K, cam.width, cam.height, tsdf_amd.SE3(q, t), 4.0)
        rgba_o, nrm_o = ora.raycast(cam.K, cam.width, cam.height, q, t, 4.0)
        assert (rgba[..., 3] == 255).mean() > 0.5
        np.testing.assert_array_equal(rgba, rgba_o)
        np.testing.assert_array_equal(nrm, nrm_o)
    finally:
        eng.close(), ora.close()


@pytest.mark.parametrize("touch", ["independent", "u16", "u16z"])
def test_semantic_c3_full_size_120_frames(touch):
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid

    def host(x):
        return x.cpu().numpy() if torch.is_tensor(x) else np.asarray(x)

    W, H, n = 640, 480, 120
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    fr = synth.render_torch(cam, list(range(n)), device="cuda", touch=touch)
    eng = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    ora = OracleGrid(0.005, 0.03, 18)
    try:
        for i in range(n):
            q, t = fr["q"][i], fr["t"][i]
            eng.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, tsdf_amd.SE3(q, t), 4.0)
            ora.integrate(host(fr["rgb"][i]), host(fr["depth"][i]), host(fr["ht"][i]), host(fr["lt"][i]), 4.0,
                          cam.K, host(q), host(t))
            if (i + 1) % 40 == 0:
                s, so = eng.stats(), ora.stats()
                assert s["status"] == 0, s
                assert s["active_blocks"] == so["active_blocks"]
                compare(eng, ora, tag=f"{touch} frame {i}")
        d = eng.dump()
        live = d["entry_idx"][d["entry_idx"] >= 0]
        w = d["rgbw"].reshape(-1, 512, 4)[live, :, 3]
        p = d["prob"].reshape(-1, 512)[live][w > 0]
        assert (w == 40).sum() > 100000, "the orbit drives much of the surface to the weight cap"
        if touch == "independent":
            assert (p > 1 - 1e-5).sum() > 1000 and (p < 1e-5).sum() > 1000
        else:
            assert (p == 1).sum() > 1000
        rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        nrm = torch.zeros_like(rgba)
        eng.raycast(K, W, H, tsdf_amd.SE3(fr["q"][n - 1], fr["t"][n - 1]), 4.0, rgba, nrm)
        torch.cuda.synchronize()
        rgba_o, nrm_o = ora.raycast(cam.K, W, H, host(fr["q"][n - 1]), host(fr["t"][n - 1]), 4.0)
        np.testing.assert_array_equal(rgba.cpu().numpy(), rgba_o)
        np.testing.assert_array_equal(nrm.cpu().numpy(), nrm_o)
    finally:
        eng.close()
        ora.close()
