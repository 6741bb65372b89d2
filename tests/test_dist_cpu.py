"""Multi-rank (world_size 2, gloo, CPU) coverage of the N>1 path.

 - the bench's rank bookkeeping (tsdf_amd.dist): max-over-ranks timing, whole-job units, stream
   offsets, shard assignment, and the routed-frame key exchange (all-to-all of the outboxes);
 - spatial sharding semantics on the CPU oracle: two shard engines fed the same frames own
   disjoint block sets, each block lives on its owner, and the union equals the unsharded volume
   with bit-identical voxels (integration of a block reads only its own state + the frame).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

W, H, VOXEL, TRUNC, NB, FRAMES = 64, 48, 0.01, 0.04, 13, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _live(ora):
    d = ora.dump()
    live = np.flatnonzero(d["entry_idx"] >= 0)
    idx = d["entry_idx"][live]
    pos = d["entry_pos"][live, :3]
    order = np.lexsort(pos.T[::-1])
    tsdf = d["tsdf"].reshape(-1, 512)[idx][order]
    rgbw = d["rgbw"].reshape(-1, 512, 4)[idx][order]
    return pos[order], tsdf, rgbw


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tests"), os.path.join(root, "disinfect-slam_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from tsdf_amd import dist as tdist
    from tsdf_amd import synth
    from _oracle import OracleGrid, block_owner

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, lr, w = tdist.env_rank_world()
        assert (r, lr, w) == (rank, rank, world)
        assert tdist.max_over_ranks(1.5 + rank) == 1.5 + world - 1
        assert tdist.sum_over_ranks([1, rank]) == [world, sum(range(world))]
        assert tdist.units("streams", 300, world) == 300 * world
        assert tdist.units("sharded", 300, world) == 300
        assert tdist.shard_of("sharded", rank, world) == (rank, world)
        assert tdist.shard_of("streams", rank, world) == (0, 1)
        assert tdist.units("routed", 300, world) == 300
        assert tdist.shard_of("routed", rank, world) == (rank, world)
        # routed frames' key exchange (bench --mode routed): inbox slot s = rank s's outbox slot rank
        import torch
        slot = 48
        out = torch.stack([torch.full((slot,), rank * world + j, dtype=torch.uint8) for j in range(world)])
        inbox = tdist.route_exchange(out, torch.empty_like(out))
        for src in range(world):
            assert bool((inbox[src] == src * world + rank).all()), (rank, src, inbox[src][:4])
        # render replicas (tsdf_amd.dist.render_sharded): all-gather-v of ragged record rows, rank order
        rows = np.full((rank + 1, 6160), rank + 1, np.uint8)
        rows[:, 0] = np.arange(rank + 1)
        got = tdist.gather_rows(rows).numpy()
        assert got.shape == (world * (world + 1) // 2, 6160)
        exp = np.concatenate([np.full((r + 1, 6160), r + 1, np.uint8) for r in range(world)])
        exp[:, 0] = np.concatenate([np.arange(r + 1) for r in range(world)])
        np.testing.assert_array_equal(got, exp)
        assert tdist.gather_rows(np.zeros((0, 6160), np.uint8)).shape == (0, 6160)
        offs = [None] * world
        dist.all_gather_object(offs, tdist.stream_offset("streams", rank, world))
        assert len(set(offs)) == world

        cam = synth.camera(W, H, synth.TUM_FR1)
        shard = OracleGrid(VOXEL, TRUNC, NB, shard_index=rank, shard_count=world)
        for f in range(FRAMES):
            fr = synth.render(cam, 2 * f)
            shard.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
        pos, tsdf, rgbw = _live(shard)
        shard.close()
        assert all(block_owner(*map(int, p), world) == rank for p in pos)
        # whole-volume Query of the sharded volume = union of the shard queries (SURVEY 8e gather)
        qshard = OracleGrid(VOXEL, TRUNC, NB, shard_index=rank, shard_count=world)
        for f in range(FRAMES):
            fr = synth.render(cam, 2 * f)
            qshard.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
        union = tdist.gather_query(qshard.query(None))
        qshard.close()
        sets = tdist.gather_block_sets(pos)
        tsdfs = [None] * world
        dist.all_gather_object(tsdfs, (tsdf, rgbw))
        if rank == 0:
            keys = [set(map(tuple, s.tolist())) for s in sets]
            assert not (keys[0] & keys[1])
            full = OracleGrid(VOXEL, TRUNC, NB)
            for f in range(FRAMES):
                fr = synth.render(cam, 2 * f)
                full.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            fpos, ftsdf, frgbw = _live(full)
            fq = full.query(None)
            full.close()
            srt = lambda a: a[np.lexsort(a.view(np.uint32).T[::-1])]
            assert union.shape == fq.shape and fq.shape[0] > 0
            np.testing.assert_array_equal(srt(union).view(np.uint32), srt(fq).view(np.uint32))
            fkeys = list(map(tuple, fpos.tolist()))
            assert set(fkeys) == keys[0] | keys[1]
            where = {k: i for i, k in enumerate(fkeys)}
            for s, (t, c) in zip(sets, tsdfs):
                sel = [where[tuple(p)] for p in s.tolist()]
                np.testing.assert_array_equal(t.view(np.uint32), ftsdf[sel].view(np.uint32))
                np.testing.assert_array_equal(c, frgbw[sel])
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_two_rank_sharding_and_bookkeeping(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)
