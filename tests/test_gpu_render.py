"""Raycast of a spatially sharded volume (SURVEY.md 8e raycast composite).

The sharded volumes here are tsdf_amd.ShardGroup volumes (one GPU, exchanged slots), whose union is
the unsharded volume (tests/test_gpu_sharded.py); the two-process test runs the same frames
through tsdf_amd.dist.integrate_sharded over gloo.

Every shard packs the blocks a raycast of the render camera can read (tsdf_render_blocks, a
conservative view-pyramid selection), the union is imported into a scratch replica engine
(tsdf_import_blocks) and rendered there with the unchanged raycast kernel. The images must equal the
unsharded engine's tsdf_raycast bit for bit: ray_cast_kernel (voxel_tsdf.cu:232-307) reads only
voxels inside the selection, and a missing block reads as the default voxel on both sides.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, VOXEL, TRUNC = 96, 72, 0.01, 0.04


def _engines(G, nb_bits=13, w=W, h=H, voxel=VOXEL, trunc=TRUNC):
    """(unsharded engine, G-shard group of one volume or None, replica engine)."""
    import tsdf_amd
    full = tsdf_amd.Engine(voxel, trunc, max_width=w, max_height=h, num_block_bits=nb_bits)
    group = tsdf_amd.ShardGroup(G, voxel, trunc, max_width=w, max_height=h, num_block_bits=nb_bits) if G else None
    replica = tsdf_amd.Engine(voxel, trunc, max_width=w, max_height=h, num_block_bits=nb_bits)
    return full, group, replica


def _integrate(engines, cam, frames, stride=2):
    import tsdf_amd
    from tsdf_amd import synth
    for f in range(frames):
        fr = synth.render(cam, stride * f)
        for e in engines:
            e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K,
                        tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)


def _views(cam):
    """Render cameras: a mapped pose, an in-between pose, and a narrow (4x focal) view."""
    import tsdf_amd
    from tsdf_amd import synth
    out = []
    for f, zoom in ((8, 1.0), (3, 1.0), (5, 4.0)):
        fr = synth.render(cam, f)
        K = np.array(cam.K, np.float32).copy()
        K[:2] *= zoom
        out.append((K, tsdf_amd.SE3(fr["q"], fr["t"])))
    return out


def _close(*engines):
    for e in engines:
        e.close()


def test_replica_of_unsharded_volume_renders_identically():
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, _, replica = _engines(0)
    try:
        _integrate([full], cam, 6)
        active = full.stats()["active_blocks"]
        for K, pose in _views(cam):
            recs = full.render_blocks(K, W, H, pose, 4.0)
            assert 0 < recs.shape[0] <= active
            replica.reset()
            assert replica.stats()["active_blocks"] == 0
            replica.import_blocks(recs)
            assert replica.stats()["active_blocks"] == recs.shape[0]
            exp = full.raycast(K, W, H, pose, 4.0)
            got = replica.raycast(K, W, H, pose, 4.0)
            assert (exp[0][..., 3] == 255).sum() > 0.3 * W * H  # the view hits the surface
            np.testing.assert_array_equal(got[0], exp[0])
            np.testing.assert_array_equal(got[1], exp[1])
        # the narrow view selects a strict subset of the volume
        K, pose = _views(cam)[2]
        assert full.render_blocks(K, W, H, pose, 4.0).shape[0] < active
    finally:
        _close(full, replica)


def test_imported_blocks_equal_their_source():
    """Imported payload = source payload: Query of the replica is a subset of the source's Query
    (positions and tsdf bit-exact), one whole block per record; keys already present are kept."""
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, _, replica = _engines(0)
    try:
        _integrate([full], cam, 4)
        K, pose = _views(cam)[0]
        recs = full.render_blocks(K, W, H, pose, 4.0)
        replica.import_blocks(recs)
        replica.import_blocks(recs[: recs.shape[0] // 2])  # re-import: no new blocks
        assert replica.stats()["active_blocks"] == recs.shape[0]
        key = lambda a: {bytes(r) for r in a.view(np.uint8).reshape(a.shape[0], -1)}
        got = replica.query(None)
        assert got.shape[0] == 512 * recs.shape[0]
        assert key(got) <= key(full.query(None))
        hdr = recs[:, :16].view(np.int16)[:, :4]
        assert (hdr[:, 3] == 0).all() and len({tuple(h) for h in hdr[:, :3]}) == recs.shape[0]
    finally:
        _close(full, replica)


@pytest.mark.parametrize("G", [2, 3])
def test_sharded_render_equals_unsharded(G):
    import torch

    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, group, replica = _engines(G)
    shards = group.engines
    try:
        _integrate([full, group], cam, 6)
        for K, pose in _views(cam):
            parts = [e.render_blocks(K, W, H, pose, 4.0, device=True) for e in shards]
            assert sum(p.shape[0] for p in parts) == full.render_blocks(K, W, H, pose, 4.0).shape[0]
            replica.import_blocks(torch.cat(parts), replace=True)  # drops the previous view's blocks
            assert replica.stats()["active_blocks"] == sum(p.shape[0] for p in parts)
            exp = full.raycast(K, W, H, pose, 4.0)
            got = replica.raycast(K, W, H, pose, 4.0)
            np.testing.assert_array_equal(got[0], exp[0])
            np.testing.assert_array_equal(got[1], exp[1])
    finally:
        _close(full, replica, group)


def test_sharded_render_bench_scale():
    """C3 geometry (640x480, 5 mm, 3 cm truncation), 8 shards after 12 frames of the orbit."""
    import torch

    from tsdf_amd import synth
    w, h, G = 640, 480, 8
    cam = synth.camera(w, h, synth.TUM_FR1)
    full, group, replica = _engines(G, nb_bits=16, w=w, h=h, voxel=0.005, trunc=0.03)
    shards = group.engines
    try:
        _integrate([full, group], cam, 12, stride=3)
        fr = synth.render(cam, 20)
        import tsdf_amd
        pose = tsdf_amd.SE3(fr["q"], fr["t"])
        parts = [e.render_blocks(cam.K, w, h, pose, 4.0, device=True) for e in shards]
        replica.import_blocks(torch.cat(parts))
        exp = full.raycast(cam.K, w, h, pose, 4.0)
        got = replica.raycast(cam.K, w, h, pose, 4.0)
        assert (exp[0][..., 3] == 255).sum() > 0.5 * w * h
        np.testing.assert_array_equal(got[0], exp[0])
        np.testing.assert_array_equal(got[1], exp[1])
    finally:
        _close(full, replica, group)


def test_replica_random_views():
    """Selection superset property under arbitrary cameras: random positions in the room, random
    orientations (including views of unmapped space and of the room from outside it), random focal
    lengths and image sizes -- the replica always renders what the volume renders."""
    import tsdf_amd
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, _, replica = _engines(0)
    rng = np.random.default_rng(0x5EED)
    try:
        _integrate([full], cam, 8)
        hits = 0
        for _ in range(24):
            q = rng.normal(size=4).astype(np.float32)
            q /= np.linalg.norm(q)
            x, y, z, qw = (float(v) for v in q)
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * qw), 2 * (x * z + y * qw)],
                          [2 * (x * y + z * qw), 1 - 2 * (x * x + z * z), 2 * (y * z - x * qw)],
                          [2 * (x * z - y * qw), 2 * (y * z + x * qw), 1 - 2 * (x * x + y * y)]])
            centre = rng.uniform([-1.0, -1.0, -0.5], [7.0, 6.0, 3.5])  # camera centre in the world
            t = (-R @ centre).astype(np.float32)  # cam_T_world translation
            w, h = int(rng.integers(16, W + 1)), int(rng.integers(12, H + 1))
            f = float(rng.uniform(20.0, 400.0))
            K = np.array([f, f * float(rng.uniform(0.8, 1.2)), w / 2 - 0.5, h / 2 - 0.5], np.float32)
            pose = tsdf_amd.SE3(q, t)
            recs = full.render_blocks(K, w, h, pose, 4.0)
            replica.import_blocks(recs, replace=True)
            exp = full.raycast(K, w, h, pose, 4.0)
            got = replica.raycast(K, w, h, pose, 4.0)
            hits += int((exp[0][..., 3] == 255).sum())
            np.testing.assert_array_equal(got[0], exp[0])
            np.testing.assert_array_equal(got[1], exp[1])
        assert hits > 0
    finally:
        _close(full, replica)


def _tri_set(t):
    t = np.ascontiguousarray(t, dtype=np.float32).reshape(-1, 9)
    return t[np.lexsort(t.view(np.uint32).T[::-1])].view(np.uint32)


@pytest.mark.parametrize("G", [2, 3])
def test_sharded_mesh_equals_unsharded(G):
    """tsdf_pack_blocks (all live blocks) -> replica -> tsdf_extract_mesh = the unsharded mesh as a
    set of triangles; the union of the shards' own meshes is not (cells across owners are lost)."""
    import torch

    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, group, replica = _engines(G)
    shards = group.engines
    try:
        _integrate([full, group], cam, 6)
        xyz = full.query(None).view(np.float32).reshape(-1, 4)[:, :3]
        lo, hi = np.percentile(xyz, 20, axis=0), np.percentile(xyz, 80, axis=0)
        box = np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], np.float32)
        parts = [e.pack_blocks(None, device=True) for e in shards]
        assert sum(p.shape[0] for p in parts) == full.stats()["active_blocks"]
        replica.import_blocks(torch.cat(parts), replace=True)
        for bounds in (None, box):
            exp = full.extract_mesh(bounds)
            got = replica.extract_mesh(bounds)
            assert exp.shape[0] > 100
            np.testing.assert_array_equal(_tri_set(got), _tri_set(exp))
        own = _tri_set(np.concatenate([e.extract_mesh(None) for e in shards]))
        ref = _tri_set(full.extract_mesh(None))
        assert own.shape != ref.shape or not np.array_equal(own, ref)
        # bounded packing selects the Query blocks of the box
        sel = full.pack_blocks(box)
        assert 0 < sel.shape[0] < full.stats()["active_blocks"]
        assert sel.shape[0] * 512 == full.query(box).shape[0]
    finally:
        _close(full, replica, group)


def test_import_errors():
    import tsdf_amd
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, _, _ = _engines(0)
    small = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=6)
    try:
        _integrate([full], cam, 4)
        K, pose = _views(cam)[0]
        recs = full.render_blocks(K, W, H, pose, 4.0)
        assert recs.shape[0] > 64
        with pytest.raises(tsdf_amd.TSDFError):
            small.import_blocks(recs)  # 64-block pool
        small.reset()
        small.import_blocks(recs[:10])
        assert small.stats()["active_blocks"] == 10
    finally:
        _close(full, small)


def _render_worker(rank, world, port, q, pipe=False):
    import os
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "disinfect-slam_amd"))
    import torch
    import torch.distributed as dist

    import tsdf_amd
    from tsdf_amd import dist as tdist
    from tsdf_amd import synth
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cam = synth.camera(W, H, synth.TUM_FR1)
        shard = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=13,
                                shard_index=rank, shard_count=world,
                                stream=torch.cuda.current_stream().cuda_stream)
        replica = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=13)
        engines = [shard]
        bufs = tdist.ShardBuffers(shard, world, key_cap=8192, cand_cap=4096)
        if rank == 0:
            full = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=13)
            engines.append(full)
            _integrate([full], cam, 6)
        for f in range(6):  # the sharded frames: key and candidate slots all-gathered over gloo
            fr = synth.render(cam, 2 * f)
            if pipe:  # one k_frame and one candidate all-gather per frame (tsdf_integrate_shard_pipe)
                tdist.integrate_sharded_pipe(shard, bufs, fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K,
                                             tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
            else:
                tdist.integrate_sharded(shard, bufs, fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K,
                                        tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
        if pipe:
            tdist.flush_sharded_pipe(shard, bufs)
        for K, pose in _views(cam):
            got = tdist.render_sharded(shard, replica, K, W, H, pose, 4.0, device=False)
            if rank == 0:
                exp = full.raycast(K, W, H, pose, 4.0)
                assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
        tris = tdist.mesh_sharded(shard, replica, device=False)
        if rank == 0:
            assert np.array_equal(_tri_set(tris), _tri_set(full.extract_mesh(None)))
        dist.barrier()
        for e in engines + [replica]:
            e.close()
        q.put((rank, "ok"))
    except BaseException as ex:  # report to the parent instead of hanging the spawn
        q.put((rank, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipe", [False, True])
def test_render_sharded_two_ranks(pipe):
    """tsdf_amd.dist.render_sharded across 2 processes (gloo all-gather of host records, both ranks
    on this GPU): rank 0's image equals its unsharded engine's raycast bit for bit, and the mesh its
    mesh. pipe: the frames through integrate_sharded_pipe (one candidate exchange per frame, across
    the processes) and flush_sharded_pipe."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_render_worker, args=(2, port, q, pipe), nprocs=2, join=True, start_method="spawn")
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: "ok", 1: "ok"}, res


def _banded_render(shards, replica, K, w, h, pose, rows):
    """The sharded render of tsdf_amd.dist.render_sharded with the all-to-all done in-process:
    band b's replica imports band b's records of every shard and renders band b's rows."""
    import torch
    G = len(shards)
    parts = [e.render_bands(K, w, h, pose, 4.0, rows, device=True) for e in shards]
    rgba = np.zeros((h, w, 4), np.uint8)
    normal = np.zeros((h, w, 4), np.uint8)
    received = []
    for b in range(G):
        recs = []
        for counts, r in parts:
            off = int(counts[:b].sum())
            recs.append(r[off:off + int(counts[b])])
        recs = torch.cat(recs)
        received.append(int(recs.shape[0]))
        replica.import_blocks(recs, replace=True)
        got = replica.raycast_rows(K, w, h, pose, 4.0, rows[b], rows[b + 1] - rows[b])
        rgba[rows[b]:rows[b + 1]] = got[0]
        normal[rows[b]:rows[b + 1]] = got[1]
    return rgba, normal, received


@pytest.mark.parametrize("G", [2, 3])
def test_banded_sharded_render_equals_unsharded(G):
    """Sharded render that splits the image: band b of the rows is rendered from the
    blocks every shard selects for that band's sub-pyramid (tsdf_render_bands) -- bit-identical to
    the unsharded raycast, and tsdf_raycast_rows equals the rows of a whole raycast."""
    from tsdf_amd import dist as tdist
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, group, replica = _engines(G)
    try:
        _integrate([full, group], cam, 6)
        for K, pose in _views(cam):
            exp = full.raycast(K, W, H, pose, 4.0)
            r0, n = 17, 23
            part = full.raycast_rows(K, W, H, pose, 4.0, r0, n)
            np.testing.assert_array_equal(part[0], exp[0][r0:r0 + n])
            np.testing.assert_array_equal(part[1], exp[1][r0:r0 + n])
            got = _banded_render(group.engines, replica, K, W, H, pose, tdist.band_rows(H, G))
            np.testing.assert_array_equal(got[0], exp[0])
            np.testing.assert_array_equal(got[1], exp[1])
    finally:
        _close(full, replica, group)


def test_banded_sharded_render_bench_scale():
    """C3 / C5 geometry, 8 shards: the banded render equals the unsharded raycast bit for bit, and a
    band's replica holds a fraction of the view's blocks (the render work and the records each rank
    receives shrink with the shard count)."""
    import tsdf_amd
    from tsdf_amd import dist as tdist
    from tsdf_amd import synth
    w, h, G = 640, 480, 8
    cam = synth.camera(w, h, synth.TUM_FR1)
    full, group, replica = _engines(G, nb_bits=16, w=w, h=h, voxel=0.005, trunc=0.03)
    try:
        _integrate([full, group], cam, 12, stride=3)
        fr = synth.render(cam, 20)
        pose = tsdf_amd.SE3(fr["q"], fr["t"])
        exp = full.raycast(cam.K, w, h, pose, 4.0)
        got = _banded_render(group.engines, replica, cam.K, w, h, pose, tdist.band_rows(h, G))
        assert (exp[0][..., 3] == 255).sum() > 0.5 * w * h
        np.testing.assert_array_equal(got[0], exp[0])
        np.testing.assert_array_equal(got[1], exp[1])
        view = full.render_blocks(cam.K, w, h, pose, 4.0).shape[0]
        received = got[2]
        assert max(received) < 0.5 * view, (received, view)
        assert sum(received) < 2.0 * view, (received, view)
    finally:
        _close(full, replica, group)


@pytest.mark.parametrize("G", [2, 3])
def test_halo_sharded_mesh_equals_unsharded(G):
    """Sharded marching cubes that splits the work: shard s meshes only its own blocks, in a replica
    holding them plus the halo of neighbouring blocks the other shards send it (tsdf_pack_halo) --
    the union of the shards' triangles is the unsharded mesh, and the halo is smaller than the
    volume."""
    import torch

    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, group, replica = _engines(G)
    shards = group.engines
    try:
        _integrate([full, group], cam, 6)
        xyz = full.query(None).view(np.float32).reshape(-1, 4)[:, :3]
        lo, hi = np.percentile(xyz, 20, axis=0), np.percentile(xyz, 80, axis=0)
        box = np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], np.float32)
        halos = [e.pack_halo(device=True) for e in shards]
        active = full.stats()["active_blocks"]
        for bounds in (None, box):
            tris = []
            for s, e in enumerate(shards):
                own = e.pack_blocks(None, device=True)
                got = [r[int(c[:s].sum()):int(c[:s + 1].sum())] for c, r in halos]
                halo = torch.cat(got)
                assert halo.shape[0] < active - own.shape[0]
                replica.import_blocks(torch.cat([own, halo]), replace=True)
                tris.append(replica.extract_mesh(bounds, owner=(s, G)))
            exp = full.extract_mesh(bounds)
            assert exp.shape[0] > 100
            np.testing.assert_array_equal(_tri_set(np.concatenate(tris)), _tri_set(exp))
    finally:
        _close(full, replica, group)


def _halo_mesh(shards, replica):
    """tsdf_amd.dist.mesh_sharded with the all-to-all done in-process: shard s meshes its own blocks
    in a replica holding them plus the halo the other shards send it."""
    import torch
    G = len(shards)
    halos = [e.pack_halo(device=True) for e in shards]
    tris = []
    for s, e in enumerate(shards):
        own = e.pack_blocks(None, device=True)
        halo = torch.cat([r[int(c[:s].sum()):int(c[:s + 1].sum())] for c, r in halos])
        replica.import_blocks(torch.cat([own, halo]), replace=True)
        tris.append(replica.extract_mesh(None, owner=(s, G)))
    return np.concatenate(tris)


def test_halo_sharded_mesh_equals_unsharded_eight_shards():
    """The halo mesh at G = 8: the union of the 8 shards' triangles is the
    unsharded mesh."""
    from tsdf_amd import synth
    cam = synth.camera(W, H, synth.TUM_FR1)
    full, group, replica = _engines(8)
    try:
        _integrate([full, group], cam, 6)
        exp = full.extract_mesh(None)
        assert exp.shape[0] > 100
        np.testing.assert_array_equal(_tri_set(_halo_mesh(group.engines, replica)), _tri_set(exp))
    finally:
        _close(full, replica, group)


def test_c5_loop_eight_shards_graph_frames():
    """BASELINE C5 on an 8-way sharded volume as one loop: 640x480 frames of the
    bench stream through each shard's graph-captured sharded frame (ShardGroup graph=...), the banded
    render of the sharded volume every 10 frames equal to the unsharded engine's raycast bit for bit,
    and at frame 30 the halo mesh of the 8 shards equal to the unsharded mesh and to the CPU oracle's."""
    import torch

    import tsdf_amd
    from tsdf_amd import dist as tdist
    from tsdf_amd import synth
    from _oracle import OracleGrid
    w, h, G, n = 640, 480, 8, 30
    cam = synth.camera(w, h, synth.TUM_FR1)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    full = tsdf_amd.Engine(0.005, 0.03, max_width=w, max_height=h, num_block_bits=18)
    group = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=w, max_height=h, num_block_bits=16,
                                graph=(w, h))
    replica = tsdf_amd.Engine(0.005, 0.03, max_width=w, max_height=h, num_block_bits=18)
    ora = OracleGrid(0.005, 0.03, 18)
    try:
        rows = tdist.band_rows(h, G)
        for i in range(n):
            fr = synth.render(cam, i)
            dev = {k: torch.from_numpy(fr[k]).to("cuda") for k in ("rgb", "depth", "ht", "lt")}
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            full.integrate(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], K, pose, 4.0)
            group.integrate(dev["rgb"], dev["depth"], dev["ht"], dev["lt"], K, pose, 4.0)
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            if (i + 1) % 10 == 0:
                exp = full.raycast(K, w, h, pose, 4.0)
                got = _banded_render(group.engines, replica, K, w, h, pose, rows)
                assert (exp[0][..., 3] == 255).mean() > 0.5, i
                np.testing.assert_array_equal(got[0], exp[0])
                np.testing.assert_array_equal(got[1], exp[1])
        for e in group.engines:
            assert e.stats()["status"] == 0
        exp = full.extract_mesh(None, 0.99, 0)
        m_o = ora.extract_mesh(None, 0.99, 0)
        assert exp.shape[0] > 100000
        np.testing.assert_array_equal(np.asarray(exp).view(np.uint32), np.asarray(m_o).view(np.uint32))
        np.testing.assert_array_equal(_tri_set(_halo_mesh(group.engines, replica)), _tri_set(exp))
    finally:
        _close(full, replica, group)
        ora.close()
