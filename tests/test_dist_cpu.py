"""Multi-rank (world_size 2, gloo, CPU) coverage of the N>1 path.

 - the bench's rank bookkeeping (tsdf_amd.dist): max-over-ranks timing, whole-job units, stream
   offsets, shard assignment, the slot all-gather of sharded frames, the ragged row gather;
 - the sharded-volume protocol itself on the CPU oracle (tests/_shards.py restates the engine's
   tsdf_integrate_shard_* phases): each rank is one shard of one volume, runs the DDA over its band
   of pixel rows, and the ranks all-gather their new keys and their carve candidates over gloo.
   Every rank's hash index equals the unsharded table, every block it holds equals the unsharded
   block, and the union of the ranks' blocks is the unsharded volume -- at a size where keys of
   the two ranks contend for bucket locks (cross-shard lock losses > 0, asserted).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

W, H, VOXEL, TRUNC, NB, FRAMES = 160, 120, 0.005, 0.03, 15, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tests"), os.path.join(root, "disinfect-slam_amd")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from tsdf_amd import dist as tdist
    from tsdf_amd import synth
    from _oracle import OracleGrid, lib
    from _shards import assert_shard_matches, row_slices

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, lr, w = tdist.env_rank_world()
        assert (r, lr, w) == (rank, rank, world)
        assert tdist.max_over_ranks(1.5 + rank) == 1.5 + world - 1
        assert tdist.sum_over_ranks([1, rank]) == [world, sum(range(world))]
        assert tdist.units("streams", 300, world) == 300 * world
        for mode in ("sharded", "routed"):
            assert tdist.units(mode, 300, world) == 300
            assert tdist.shard_of(mode, rank, world) == (rank, world)
        assert tdist.shard_of("streams", rank, world) == (0, 1)
        # the exchange of sharded frames: slot all-gather in rank order
        slot = torch.full((48,), rank + 7, dtype=torch.uint8)
        out = torch.empty((world, 48), dtype=torch.uint8)
        tdist.all_gather_slots(slot, out)
        for src in range(world):
            assert bool((out[src] == src + 7).all()), (rank, src, out[src][:4])
        # banded render / mesh halo (tsdf_amd.dist.exchange_groups): all-to-all-v of grouped rows --
        # rank r's group d (d + 1 + r rows tagged (r, d)) arrives at rank d, in source-rank order
        counts = [d + 1 + rank for d in range(world)]
        recs = torch.cat([torch.full((counts[d], 16), 16 * rank + d, dtype=torch.uint8) for d in range(world)])
        got, rc = tdist.exchange_groups(counts, recs)
        assert rc == [rank + 1 + src for src in range(world)], rc
        off = 0
        for src in range(world):
            assert bool((got[off:off + rc[src]] == 16 * src + rank).all())
            off += rc[src]
        assert off == got.shape[0]
        assert tdist.band_rows(480, world)[-1] == 480
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

        # ---- the sharded volume, one shard per rank ----
        cam = synth.camera(W, H, synth.TUM_FR1)
        shard = OracleGrid(VOXEL, TRUNC, NB)
        lib().ora_set_shard(shard.h, rank, world)
        full = OracleGrid(VOXEL, TRUNC, NB)  # every rank checks its own shard against one volume
        lo, hi = row_slices(H, world)[rank]
        cross = 0
        for f in range(FRAMES):
            fr = synth.render(cam, f)
            full.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            keys, orders = shard.shard_keys(fr["depth"], cam.K, fr["q"], fr["t"], 4.0, lo, hi)
            parts = [None] * world
            dist.all_gather_object(parts, (keys, orders))  # the key all-gather
            cpos, cent = shard.shard_update(np.concatenate([p[0] for p in parts]),
                                            np.concatenate([p[1] for p in parts]), fr["rgb"],
                                            fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            cands = [None] * world
            dist.all_gather_object(cands, (cpos, cent))  # the carve-candidate all-gather
            shard.shard_delete(np.concatenate([c[0] for c in cands]), np.concatenate([c[1] for c in cands]))
            cross += shard.stats()["last_cross_losses"]
        fd = full.dump()
        mine = assert_shard_matches(shard.dump(), fd, tag=f"rank {rank}")
        assert mine and cross > 0, (len(mine), cross)
        # whole-volume Query of the sharded volume = union of the shard queries (SURVEY 8e gather)
        union = tdist.gather_query(shard.query(None))
        fq = full.query(None)
        sets = [None] * world
        dist.all_gather_object(sets, sorted(mine))
        if rank == 0:
            keys = [set(s) for s in sets]
            assert not (keys[0] & keys[1])
            idx = fd["entry_idx"]
            live = fd["entry_pos"][(idx >= 0), :3]
            assert keys[0] | keys[1] == {tuple(map(int, p)) for p in live}
            srt = lambda a: a[np.lexsort(a.view(np.uint32).T[::-1])]
            assert union.shape == fq.shape and fq.shape[0] > 0
            np.testing.assert_array_equal(srt(union).view(np.uint32), srt(fq).view(np.uint32))
        shard.close()
        full.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_two_rank_sharding_and_bookkeeping(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)
