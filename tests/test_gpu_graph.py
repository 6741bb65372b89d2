"""Graph-captured frame loop (tsdf_graph_*, BASELINE config C5): one hipGraph launch per frame
(argument upload, DDA / allocation, update, carving, raycast of a render camera) must give exactly
what tsdf_integrate + tsdf_raycast give on the same device frames, frame after frame."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("semantic", [True, False])
def test_graph_loop_matches_eager_calls(semantic):
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, n = 160, 120, 9
    cam = synth.camera(W, H, synth.TUM_FR1)
    fr = synth.render_torch(cam, list(range(n + 3)), device="cuda")
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=15)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=15)
    g = b.frame_graph(W, H, W, H)
    try:
        img = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
        hits = 0
        for i in range(n):
            pose = tsdf_amd.SE3(fr["q"][i], fr["t"][i])
            rpose = tsdf_amd.SE3(fr["q"][i + 3], fr["t"][i + 3])
            ht = fr["ht"][i] if semantic else None
            lt = fr["lt"][i] if semantic else None
            a.integrate(fr["rgb"][i], fr["depth"][i], ht, lt, K, pose, 4.0)
            a.raycast(K, W, H, rpose, 4.0, rgba=img[0], normal=img[1])
            g.frame(fr["rgb"][i], fr["depth"][i], ht, lt, K, pose, 4.0, K, rpose, img[2], img[3])
            a.synchronize()
            b.synchronize()
            assert torch.equal(img[0], img[2]) and torch.equal(img[1], img[3]), f"frame {i}"
            hits += int((img[2][..., 3] == 255).sum())
            sa, sb = a.stats(), b.stats()
            for k in ("active_blocks", "last_num_visible", "last_num_updated", "last_num_deleted", "status"):
                assert sa[k] == sb[k], (i, k, sa[k], sb[k])
        assert hits > W * H  # the render camera sees the surface
        da, db = a.dump(), b.dump()
        for k in ("entry_pos", "entry_idx", "heap", "rgbw"):
            assert np.array_equal(da[k], db[k]), k
        for k in ("tsdf", "prob"):
            assert np.array_equal(da[k].view(np.uint32), db[k].view(np.uint32)), k
    finally:
        g.close()
        a.close(), b.close()


def test_graph_rejects_host_frames_and_wrong_size():
    import tsdf_amd
    from tsdf_amd import synth
    cam = synth.camera(64, 48, synth.TUM_FR1)
    fr = synth.render(cam, 0)
    with tsdf_amd.Engine(0.01, 0.04, max_width=64, max_height=48, num_block_bits=10) as e:
        g = e.frame_graph(64, 48)
        try:
            with pytest.raises(ValueError):
                g.frame(fr["rgb"], fr["depth"], None, None, cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
        finally:
            g.close()
        with pytest.raises(tsdf_amd.TSDFError):
            e.frame_graph(128, 48)


def test_pipelined_graph_frames_equal_unpipelined():
    """Graph frames without a render camera are pipelined like tsdf_integrate (one k_frame_g launch per
    frame: the pending frames' carving / allocation / update beside this frame's ingest). Mixed with
    eager frames (every transition of the pending state: a graph frame after a flush, after an eager
    frame, an eager frame after a graph frame) and reads that flush, the whole state must equal an
    unpipelined engine's bit for bit."""
    import os

    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from test_gpu_pipeline import _engine, _same
    W, H, n = 320, 240, 24
    cam = synth.camera(W, H, synth.TUM_FR1)
    fr = synth.render_torch(cam, list(range(n)), device="cuda")
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = _engine(True, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=16)
    b = _engine(False, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=16)
    g = a.frame_graph(W, H)
    eager = {3, 4, 9, 15, 16, 17}  # frames a integrates eagerly (the others through the graph)
    try:
        for i in range(n):
            pose = tsdf_amd.SE3(fr["q"][i], fr["t"][i])
            args = (fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, pose, 4.0)
            (a.integrate if i in eager else g.frame)(*args)
            b.integrate(*args)
            if i in (7, 12, n - 1):  # (reads flush the pending frames)
                torch.cuda.synchronize()
                _same(a, b, f"frame {i}")
        assert a.stats()["status"] == 0
    finally:
        g.close()
        a.close(), b.close()


@pytest.mark.parametrize("batch", [3, 8])
def test_batched_graph_frames_equal_eager(batch):
    """tsdf_graph_create_batch: `batch` pipelined C3 frames per graph launch == eager tsdf_integrate, bit
    for bit, also when other calls (stats, query) launch a partly filled batch in between."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, n = 160, 120, 29
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    fr = synth.render_torch(cam, list(range(n)), device="cuda")
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=15)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=15)
    g = b.frame_graph(W, H, batch=batch)
    try:
        for i in range(n):
            pose = tsdf_amd.SE3(fr["q"][i], fr["t"][i])
            a.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, pose, 4.0)
            g.frame(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, pose, 4.0)
            if i in (4, 13):  # a partly filled batch, launched by the read
                sa, sb = a.stats(), b.stats()
                assert sa["active_blocks"] == sb["active_blocks"] and sb["status"] == 0, (i, sa, sb)
                qa, qb = a.query(None), b.query(None)
                assert qa.shape == qb.shape and np.array_equal(qa["tsdf"].view(np.uint32), qb["tsdf"].view(np.uint32))
        b.synchronize()
        torch.cuda.synchronize()
        da, db = a.dump(), b.dump()
        for k in ("entry_pos", "entry_idx", "heap", "rgbw"):
            assert np.array_equal(da[k], db[k]), k
        for k in ("tsdf", "prob"):
            assert np.array_equal(da[k].view(np.uint32), db[k].view(np.uint32)), k
        assert da["free"] == db["free"]
    finally:
        g.close()
        a.close(), b.close()
