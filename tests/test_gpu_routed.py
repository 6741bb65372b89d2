"""Routed frames (SURVEY.md 8e option 2) on one GPU: G shard engines each run the block-allocation
DDA over their own slice of pixel-tile rows and route the visible keys other shards own through an
outbox / inbox exchange (done here with device copies; the bench does it with an RCCL all-to-all).
The result must equal the replicated-frame sharded integrate (option 1), whose shards the CPU
oracle reproduces: entries, pool indices, free stack and voxels bit-exact per shard.
"""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def exchange(outboxes):
    """inbox_j slot s = outbox_s slot j (what dist.all_to_all_single does across ranks)."""
    import torch
    G = len(outboxes)
    torch.cuda.synchronize()
    inboxes = [torch.stack([outboxes[s][j] for s in range(G)]).contiguous() for j in range(G)]
    torch.cuda.synchronize()
    return inboxes


def run_routed(G, W, H, voxel, trunc, frames, nb_bits, cap=4096, stride=1):
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    cam = synth.camera(W, H, synth.TUM_FR1)
    nbytes = tsdf_amd.Engine.route_buffer_bytes(G, cap)
    engs = [tsdf_amd.Engine(voxel, trunc, max_width=W, max_height=H, num_block_bits=nb_bits,
                            shard_index=i, shard_count=G) for i in range(G)]
    oras = [OracleGrid(voxel, trunc, nb_bits, shard_index=i, shard_count=G) for i in range(G)]
    outs = [torch.zeros((G, nbytes // G), dtype=torch.uint8, device="cuda") for _ in range(G)]
    routed = 0
    try:
        for f in range(frames):
            fr = synth.render(cam, stride * f)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            for i, e in enumerate(engs):
                e.integrate_route_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0,
                                        i, G, outs[i], cap)
                e.synchronize()
            for o in outs:  # count headers: record 0 of each slot
                routed += int(o.view(G, -1, 16)[:, 0, 8:12].contiguous().view(torch.int32).sum())
            inboxes = exchange(outs)
            for j, e in enumerate(engs):
                e.integrate_route_end(inboxes[j], cap)
            for o in oras:
                o.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            for i, (e, o) in enumerate(zip(engs, oras)):
                s, so = e.stats(), o.stats()
                assert s["status"] == 0, (f, i, s)
                assert s["active_blocks"] == so["active_blocks"], (f, i, s, so)
                assert s["last_num_visible"] == so["last_num_visible"], (f, i, s, so)
        for i, (e, o) in enumerate(zip(engs, oras)):
            compare(e, o, tag=f"routed shard {i}/{G}")
        return routed
    finally:
        for e in engs:
            e.close()
        for o in oras:
            o.close()


@pytest.mark.parametrize("G", [2, 3])
def test_routed_shards_match_sharded_oracle(G):
    routed = run_routed(G, 96, 72, 0.01, 0.04, 5, nb_bits=13, stride=2)
    assert routed > 100  # keys really crossed shards


def test_routed_5mm_160x120():
    routed = run_routed(2, 160, 120, 0.005, 0.03, 4, nb_bits=15)
    assert routed > 500


def test_route_overflow_and_misuse():
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, G, cap = 96, 72, 2, 4
    cam = synth.camera(W, H, synth.TUM_FR1)
    fr = synth.render(cam, 0)
    pose = tsdf_amd.SE3(fr["q"], fr["t"])
    e = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=12, shard_index=0,
                        shard_count=G)
    try:
        buf = torch.zeros(tsdf_amd.Engine.route_buffer_bytes(G, cap), dtype=torch.uint8, device="cuda")
        with pytest.raises(tsdf_amd.TSDFError):
            e.integrate_route_end(buf, cap)  # no routed frame pending
        e.integrate_route_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0, 0, G, buf, cap)
        with pytest.raises(tsdf_amd.TSDFError):  # pending routed frame blocks other integrates
            e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
        e.integrate_route_end(torch.zeros_like(buf), cap)
        assert e.stats(clear_status=True)["status"] & tsdf_amd.STATUS_ROUTE_OVERFLOW
    finally:
        e.close()
    u = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=12)
    try:
        with pytest.raises(tsdf_amd.TSDFError):  # unsharded engines have no routed frames
            u.integrate_route_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0, 0, 1,
                                    torch.zeros(64, dtype=torch.uint8, device="cuda"), 1)
    finally:
        u.close()


def test_sharded_query_union_equals_unsharded_query():
    """SURVEY 8e Query gather on the engine: the shard engines' Query results, concatenated the way
    tsdf_amd.dist.gather_query concatenates ranks, equal the unsharded engine's Query as a set."""
    import tsdf_amd
    from tsdf_amd import synth
    W, H, G = 96, 72, 3
    cam = synth.camera(W, H, synth.TUM_FR1)
    full = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=13)
    shards = [tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=13, shard_index=i,
                              shard_count=G) for i in range(G)]
    try:
        for f in range(5):
            fr = synth.render(cam, 2 * f)
            for e in [full] + shards:
                e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
        srt = lambda a: a[np.lexsort(a.view(np.uint32).T[::-1])]
        xyz = full.query(None).view(np.float32).reshape(-1, 4)[:, :3]
        lo, hi = np.percentile(xyz, 10, axis=0), np.percentile(xyz, 90, axis=0)
        for bounds in (None, np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], np.float32)):
            exp = full.query(bounds).view(np.float32).reshape(-1, 4)
            got = np.concatenate([e.query(bounds).view(np.float32).reshape(-1, 4) for e in shards])
            assert got.shape == exp.shape and exp.shape[0] > 0
            np.testing.assert_array_equal(srt(got).view(np.uint32), srt(exp).view(np.uint32))
    finally:
        full.close()
        for e in shards:
            e.close()
