"""BASELINE configs C5 and C3 at their workload against the CPU oracle:

 - the 640x480 render() stream integrated for 30 frames into a 2^18-block pool, eager engine and
   oracle compared every 10 frames (hash table, free stack, every voxel);
 - C5 on the same stream: the graph-captured frame (integrate + raycast of the frame's camera in one
   hipGraph launch) and the eager chain render every frame identically, the 640x480 raycast equals
   the oracle's at frames 0, 14 and 29, and marching cubes at frame 30 equals the oracle's mesh bit
   for bit (tsdf_extract_mesh, voxel_tsdf.cu's caller ros_offline.cc:279-287);
 - the raycast view grid (tsdf_kernels.h ViewGrid) against the hash-lookup path it replaces: views
   too deep for the grid, cameras outside the volume, and more calls than the grid has generations.
"""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _check_render(rgba, nrm, rgba_o, nrm_o, tag):
    hit = rgba[..., 3] == 255
    assert np.array_equal(rgba[..., 3], rgba_o[..., 3]), f"{tag}: hit mask differs"
    # colour / shading blend with the probability: bit-exact (the reference's own chain)
    np.testing.assert_array_equal(rgba, rgba_o, err_msg=tag)
    np.testing.assert_array_equal(nrm, nrm_o, err_msg=tag)
    return hit.mean()


def test_c5_640x480_stream_graph_eager_oracle():
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    W, H, n = 640, 480, 30
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    ora = OracleGrid(0.005, 0.03, 18)
    g = b.frame_graph(W, H, W, H)
    try:
        img = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
        dev = {}
        for i in range(n):
            fr = synth.render(cam, i)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            for k in ("rgb", "depth", "ht", "lt"):  # the graph takes device frames
                dev[k] = torch.from_numpy(fr[k]).to("cuda")
            a.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
            a.raycast(K, W, H, pose, 4.0, rgba=img[0], normal=img[1])
            g.frame(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], K, pose, 4.0, K, pose, img[2], img[3])
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            torch.cuda.synchronize()
            assert torch.equal(img[0], img[2]) and torch.equal(img[1], img[3]), f"frame {i}: graph != eager"
            s, so = a.stats(), ora.stats()
            assert s["status"] == 0 and b.stats()["status"] == 0
            for k in ("last_num_visible", "last_num_updated", "last_num_deleted", "active_blocks"):
                assert s[k] == so[k] == b.stats()[k], (i, k, s[k], so[k])
            if i in (0, 14, n - 1):
                ro, no = ora.raycast(cam.K, W, H, fr["q"], fr["t"], 4.0)
                frac = _check_render(img[0].cpu().numpy(), img[1].cpu().numpy(), ro, no, f"frame {i}")
                assert frac > 0.5
            if (i + 1) % 10 == 0:
                compare(a, ora, tag=f"frame {i}")
        # marching cubes every 30 frames (C5): the whole volume
        m_a = a.extract_mesh(None, 0.99, 0)
        m_b = b.extract_mesh(None, 0.99, 0)
        m_o = ora.extract_mesh(None, 0.99, 0)
        assert m_a.shape[0] > 100000
        np.testing.assert_array_equal(np.asarray(m_a).view(np.uint32), np.asarray(m_o).view(np.uint32))
        np.testing.assert_array_equal(np.asarray(m_b).view(np.uint32), np.asarray(m_o).view(np.uint32))
    finally:
        g.close()
        a.close(), b.close(), ora.close()


@pytest.mark.parametrize("max_depth", [2.0, 4.0, 9.0])
def test_raycast_view_grid_depths_and_outside_cameras(max_depth):
    """4 m and 2 m use the view grid, 9 m exceeds it (hash lookups); cameras inside the volume,
    behind it and far outside it (no block within reach) render like the oracle."""
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    W, H = 160, 120
    cam = synth.camera(W, H, synth.TUM_FR1)
    eng = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=15)
    ora = OracleGrid(0.01, 0.04, 15)
    try:
        for f in range(0, 24, 3):
            fr = synth.render(cam, f)
            eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
        rng = np.random.default_rng(5)
        views = [synth.pose(f)[1] for f in (2, 11, 40)]
        for _ in range(3):  # random orientations at random places, some far outside the room
            q = rng.normal(size=4)
            q = (q / np.linalg.norm(q)).astype(np.float32)
            t = rng.uniform(-12, 12, size=3).astype(np.float32)
            views.append((q, t))
        hits = 0.0
        for q, t in views:
            rgba, nrm = eng.raycast(cam.K, W, H, tsdf_amd.SE3(q, t), max_depth)
            ro, no = ora.raycast(cam.K, W, H, q, t, max_depth)
            hits += _check_render(rgba, nrm, ro, no, f"view {q} {t} depth {max_depth}")
        assert hits > 0.5
    finally:
        eng.close(), ora.close()


def test_raycast_view_grid_generations_wrap():
    """More raycasts than the view grid has generations (1023): cells of earlier calls never read
    as this call's blocks, also after blocks were carved away and the cells were zeroed."""
    import tsdf_amd
    from tsdf_amd import synth
    W, H = 32, 24
    cam = synth.camera(W, H, synth.TUM_FR1)
    eng = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=14)
    try:
        fr = synth.render(cam, 0)
        pose = tsdf_amd.SE3(fr["q"], fr["t"])
        eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
        ref = eng.raycast(cam.K, W, H, pose, 4.0)
        assert (ref[0][..., 3] == 255).mean() > 0.5
        away = tsdf_amd.SE3(fr["q"], np.asarray(fr["t"]) + np.float32(0.5))
        for i in range(1100):
            img = eng.raycast(cam.K, W, H, pose if i % 2 else away, 4.0)
            if i % 2 and i % 97 == 1:
                assert np.array_equal(img[0], ref[0]) and np.array_equal(img[1], ref[1]), i
        eng.reset()  # every block gone: the same view must now see nothing
        img = eng.raycast(cam.K, W, H, pose, 4.0)
        assert (img[0][..., 3] == 0).all()
        eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
        img = eng.raycast(cam.K, W, H, pose, 4.0)
        assert np.array_equal(img[0], ref[0]) and np.array_equal(img[1], ref[1])
    finally:
        eng.close()


def test_c5_deferred_raycast_equals_immediate():
    """tsdf_raycast_deferred (the raycast launched beside the next frame's ingest, k_render_ingest)
    renders what tsdf_raycast renders, frame by frame over the 640x480 C5 stream; also when the next
    call is not an integrate (stats, a second raycast, mesh extraction, flush: the pending raycast is
    launched alone first) and with host frames (the upload ring) for the fused ingest."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, n = 640, 480, 24
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    try:
        ref = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
        out = [[torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)] for _ in range(3)]
        pending = None  # (frame, image pair, the immediate render's copies)
        for i in range(n):
            fr = synth.render(cam, i)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            src = fr if i % 3 == 2 else {k: torch.from_numpy(fr[k]).to("cuda") for k in ("rgb", "depth", "ht", "lt")}
            a.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
            b.integrate(src["rgb"], src["depth"], src["ht"], src["lt"], cam.K, pose, 4.0)
            if pending is not None:  # the previous deferred raycast is written by now
                j, o, r0, r1 = pending
                torch.cuda.synchronize()
                assert torch.equal(o[0], r0) and torch.equal(o[1], r1), f"frame {j}: deferred != immediate"
            a.raycast(K, W, H, pose, 4.0, rgba=ref[0], normal=ref[1])
            o = out[i % 3]
            b.raycast(K, W, H, pose, 4.0, rgba=o[0], normal=o[1], deferred=True)
            pending = (i, o, ref[0].clone(), ref[1].clone())
            if i == 7:
                assert b.stats()["status"] == 0  # (joins the pending raycast)
            elif i == 12:  # a second deferred raycast: the first is launched alone
                o2 = out[(i + 1) % 3]
                b.raycast(K, W, H, pose, 4.0, rgba=o2[0], normal=o2[1], deferred=True)
                torch.cuda.synchronize()
                assert torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]), "first of two deferred"
                pending = (i, o2, ref[0].clone(), ref[1].clone())
            elif i == 17:
                m_a, m_b = a.extract_mesh(None, 0.99, 0), b.extract_mesh(None, 0.99, 0)
                np.testing.assert_array_equal(np.asarray(m_a).view(np.uint32), np.asarray(m_b).view(np.uint32))
        b.flush()
        torch.cuda.synchronize()
        j, o, r0, r1 = pending
        assert torch.equal(o[0], r0) and torch.equal(o[1], r1), "last frame after flush"
        assert (r0[..., 3] == 255).float().mean().item() > 0.5
        assert a.stats()["status"] == 0 and b.stats()["status"] == 0
        with pytest.raises(ValueError):
            b.raycast(K, W, H, pose, 4.0, deferred=True)  # (host images: immediate only)
    finally:
        a.close(), b.close()


def test_c5_deferred_graph_equals_graph():
    """tsdf_graph_create_deferred: frame i's raycast runs in graph launch i + 1 (k_render_ingest_g) or
    in the engine's next other call; images equal the immediate graph's frame by frame, the volume
    equals it block for block (mesh), also across a stats() call, a far view (hash-lookup raycast, not
    deferred) and the final flush."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, n = 640, 480, 20
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
    ga, gb = a.frame_graph(W, H, W, H), b.frame_graph(W, H, W, H, deferred=True)
    try:
        ref = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
        out = [[torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)] for _ in range(3)]
        pending = None
        frames = []
        for i in range(n):
            fr = synth.render(cam, i)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            dev = {k: torch.from_numpy(fr[k]).to("cuda") for k in ("rgb", "depth", "ht", "lt")}
            frames.append(dev)  # (graph frames stay valid until they have run)
            md = 9.0 if i == 11 else 4.0  # frame 11: too deep for a view grid
            ga.frame(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], K, pose, md, K, pose, ref[0], ref[1])
            o = out[i % 3]
            gb.frame(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], K, pose, md, K, pose, o[0], o[1])
            if pending is not None:
                j, po, r0, r1 = pending
                torch.cuda.synchronize()
                assert torch.equal(po[0], r0) and torch.equal(po[1], r1), f"frame {j}: deferred graph != graph"
            torch.cuda.synchronize()
            pending = (i, o, ref[0].clone(), ref[1].clone())
            if i == 6:
                assert b.stats()["status"] == 0  # launches the pending raycast alone
                torch.cuda.synchronize()
                assert torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]), "frame 6 after stats"
        b.flush()
        torch.cuda.synchronize()
        j, po, r0, r1 = pending
        assert torch.equal(po[0], r0) and torch.equal(po[1], r1), "last frame after flush"
        assert (r0[..., 3] == 255).float().mean().item() > 0.5
        sa, sb = a.stats(), b.stats()
        assert sa["status"] == 0 and sb["status"] == 0 and sa["active_blocks"] == sb["active_blocks"]
        m_a, m_b = a.extract_mesh(None, 0.99, 0), b.extract_mesh(None, 0.99, 0)
        np.testing.assert_array_equal(np.asarray(m_a).view(np.uint32), np.asarray(m_b).view(np.uint32))
    finally:
        ga.close(), gb.close()
        a.close(), b.close()


def test_deferred_raycast_heavy_carving():
    """The C5 loop's view grid built inside the update launch (k_integrate_vg) before that launch's
    carving, which then clears the cells of the blocks it released: 2 cm voxels at 96x72 carve many
    blocks per frame; the deferred images equal the immediate raycast's frame by frame (also with
    TSDF_FUSE_VIEW_GRID's separate launch as the reference, the immediate path)."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, n = 96, 72, 16
    cam = synth.camera(W, H)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.02, 0.08, max_width=W, max_height=H, num_block_bits=13)
    b = tsdf_amd.Engine(0.02, 0.08, max_width=W, max_height=H, num_block_bits=13)
    try:
        ref = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
        out = [[torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)] for _ in range(2)]
        pending = None
        deleted = 0
        for i in range(n):
            fr = synth.render(cam, i)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            dev = {k: torch.from_numpy(fr[k]).to("cuda") for k in ("rgb", "depth", "ht", "lt")}
            a.integrate(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], cam.K, pose, 4.0)
            b.integrate(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], cam.K, pose, 4.0)
            if pending is not None:
                j, o, r0, r1 = pending
                torch.cuda.synchronize()
                assert torch.equal(o[0], r0) and torch.equal(o[1], r1), f"frame {j}"
            a.raycast(K, W, H, pose, 4.0, rgba=ref[0], normal=ref[1])
            deleted += a.stats()["last_num_deleted"]
            o = out[i % 2]
            b.raycast(K, W, H, pose, 4.0, rgba=o[0], normal=o[1], deferred=True)
            pending = (i, o, ref[0].clone(), ref[1].clone())
        b.flush()
        torch.cuda.synchronize()
        j, o, r0, r1 = pending
        assert torch.equal(o[0], r0) and torch.equal(o[1], r1), "last frame"
        assert deleted > 20, deleted  # (the carving ran inside the fused launches)
        assert (r0[..., 3] == 255).float().mean().item() > 0.3
        sa, sb = a.stats(), b.stats()
        assert sa["status"] == 0 and sb["status"] == 0 and sa["total_deleted"] == sb["total_deleted"]
    finally:
        a.close(), b.close()


def test_deferred_raycast_images_without_device_sync():
    """a deferred raycast into temporaries the caller drops at once, on an engine-owned
    stream, read on torch's current stream after a HOST-frame integrate (the call that renders them)
    -- no torch.cuda.synchronize in between: the engine keeps the tensors referenced until that call
    and orders torch's stream after it, so the images equal the immediate raycast. Then the same
    through flush() and through stats()."""
    import gc

    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H = 160, 120
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=15)
    b = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=15)
    try:
        frames = [synth.render(cam, f) for f in range(0, 30, 3)]
        for i, fr in enumerate(frames[:-1]):
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            for e in (a, b):
                e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], K, pose, 4.0)
            out = b.raycast(K, W, H, pose, 4.0, rgba=torch.empty((H, W, 4), dtype=torch.uint8, device="cuda"),
                            normal=torch.empty((H, W, 4), dtype=torch.uint8, device="cuda"), deferred=True)
            keep = [t.data_ptr() for t in out]
            del out
            gc.collect()
            # torch reuses freed blocks at once: garbage written into any block the images sat in
            junk = [torch.full((H, W, 4), 7, dtype=torch.uint8, device="cuda") for _ in range(4)]
            assert not any(j.data_ptr() in keep for j in junk), "the deferred images were freed early"
            nxt = frames[i + 1]
            how = i % 3
            if how == 0:  # a host-frame integrate renders the images
                b.integrate(nxt["rgb"], nxt["depth"], nxt["ht"], nxt["lt"], K, tsdf_amd.SE3(nxt["q"], nxt["t"]), 4.0)
                a.integrate(nxt["rgb"], nxt["depth"], nxt["ht"], nxt["lt"], K, tsdf_amd.SE3(nxt["q"], nxt["t"]), 4.0)
            elif how == 1:
                b.flush()
            else:
                b.stats()
            del junk
            assert b._pending is None  # rendered by that call, reference dropped
    finally:
        a.close(), b.close()


def test_deferred_raycast_read_on_torch_stream():
    """The deferred images read on torch's stream right after the engine's next call equal the
    immediate raycast (no device synchronisation)."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H = 160, 120
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    eng = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=15)
    try:
        frames = [synth.render(cam, f) for f in range(0, 24, 3)]
        for i, fr in enumerate(frames):
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], K, pose, 4.0)
            rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            nrm = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            eng.raycast(K, W, H, pose, 4.0, rgba=rgba, normal=nrm, deferred=True)
            eng.flush() if i % 2 else eng.stats()
            got = (rgba.clone(), nrm.clone())  # on torch's stream, after the call that rendered them
            ref = eng.raycast(K, W, H, pose, 4.0)
            np.testing.assert_array_equal(got[0].cpu().numpy(), ref[0])
            np.testing.assert_array_equal(got[1].cpu().numpy(), ref[1])
    finally:
        eng.close()


def test_deferred_graph_across_grid_growth_and_generation_wrap():
    """a deferred graph frame pending while the next frame's view grid is reallocated (a
    deeper render camera: the cube grows) or its generations wrap (more than kViewGenMax = 1023 grid
    builds): the pending raycast must run before the grid it reads is reset (view_grid_resets, one
    shape computation with view_grid_for). Images equal the immediate graph's frame by frame."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H = 32, 24
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    a = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=14)
    b = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=14)
    ga, gb = a.frame_graph(W, H, W, H), b.frame_graph(W, H, W, H, deferred=True)
    try:
        fr0 = [synth.render(cam, f) for f in range(0, 30, 3)]
        dev = [{k: torch.from_numpy(fr[k]).to("cuda") for k in ("rgb", "depth", "ht", "lt")} for fr in fr0]
        ref = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
        out = [[torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)] for _ in range(2)]
        pending = None
        n = 1040  # > kViewGenMax grid builds in b
        checked = 0
        for i in range(n):
            d = dev[i % len(dev)]
            pose = tsdf_amd.SE3(fr0[i % len(fr0)]["q"], fr0[i % len(fr0)]["t"])
            md = 2.0 if i < 5 else (4.0 if i < 600 else 3.0)  # frame 5: the cube grows
            ga.frame(d["rgb"], d["depth"], d["ht"], d["lt"], K, pose, md, K, pose, ref[0], ref[1])
            o = out[i % 2]
            gb.frame(d["rgb"], d["depth"], d["ht"], d["lt"], K, pose, md, K, pose, o[0], o[1])
            if pending is not None and (i < 12 or i % 97 == 0 or 1015 <= i <= 1035):
                j, po, r0, r1 = pending
                torch.cuda.synchronize()
                assert torch.equal(po[0], r0) and torch.equal(po[1], r1), f"frame {j}: deferred graph != graph"
                checked += 1
            ra, rn = ref[0].clone(), ref[1].clone()
            pending = (i, o, ra, rn)
        b.flush()
        torch.cuda.synchronize()
        j, po, r0, r1 = pending
        assert torch.equal(po[0], r0) and torch.equal(po[1], r1), "last frame after flush"
        assert checked > 40 and (r0[..., 3] == 255).float().mean().item() > 0.3
    finally:
        ga.close(), gb.close()
        a.close(), b.close()


@pytest.mark.parametrize("batch", [4])
def test_c5_batched_deferred_graph_equals_eager(batch):
    """The C5 loop as a batched, render-deferring graph (tsdf_graph_create_batch(deferred=1)): frames'
    images equal the eager loop's (integrate + immediate raycast) once their batch has run; a far view
    (hash-lookup raycast) and the render camera's cube growing mid-batch break a batch early; marching
    cubes at the end equal."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, n = 160, 120, 22
    cam = synth.camera(W, H, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    fr = synth.render_torch(cam, list(range(n)), device="cuda")
    a = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=15)
    b = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=15)
    g = b.frame_graph(W, H, W, H, deferred=True, batch=batch)
    outs = [(torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda"),
             torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")) for _ in range(n)]
    refs = []
    try:
        for i in range(n):
            pose = tsdf_amd.SE3(fr["q"][i], fr["t"][i])
            md = 9.0 if i == 9 else (2.0 if i < 3 else 4.0)  # 9: no view grid; 3: the cube grows
            a.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, pose, md)
            refs.append(a.raycast(K, W, H, pose, md))
            g.frame(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, pose, md, K, pose, outs[i][0], outs[i][1])
        b.flush()
        torch.cuda.synchronize()
        for i in range(n):
            np.testing.assert_array_equal(outs[i][0].cpu().numpy(), refs[i][0], err_msg=f"rgba {i}")
            np.testing.assert_array_equal(outs[i][1].cpu().numpy(), refs[i][1], err_msg=f"normal {i}")
        m_a, m_b = a.extract_mesh(None, 0.99, 0), b.extract_mesh(None, 0.99, 0)
        np.testing.assert_array_equal(np.asarray(m_a).view(np.uint32), np.asarray(m_b).view(np.uint32))
    finally:
        g.close()
        a.close(), b.close()
