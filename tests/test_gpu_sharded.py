"""Spatially sharded volume on one GPU: G shard engines of ONE volume, exchanging
their key and carve-candidate slots by device copies where a multi-GPU job all-gathers them
(tsdf_amd.ShardGroup; tsdf_amd.dist.integrate_sharded over RCCL).

The bar (SURVEY 8e "compared to single-GPU as sets keyed by block position"):
the union of the shards equals the UNSHARDED volume -- the same live block positions, every voxel's
tsdf / rgb / weight bit-identical, probability within 1e-4 -- and every shard's hash index equals
the unsharded table. Each shard is also bit-exact against the oracle's sharded restatement
(tests/_shards.py: pool indices and free stacks included). The configurations are ones where
keys of different owners contend for bucket locks (the oracle counts those cross-shard lock
losses), which a shard that allocates only its own keys would resolve differently.
"""
import numpy as np
import pytest

from _shards import assert_union_equals, oracle_shard_frame
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

MAXD = 4.0


def _run(G, W, H, voxel, trunc, frames, nb_bits, shard_bits, split=True, stride=1, intrinsics=None,
         oracle_shards=True, semantic=True):
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid, lib
    cam = synth.camera(W, H, intrinsics or synth.TUM_FR1)
    group = tsdf_amd.ShardGroup(G, voxel, trunc, max_width=W, max_height=H, num_block_bits=shard_bits,
                                split=split)
    full = OracleGrid(voxel, trunc, nb_bits)
    oshards = []
    if oracle_shards:
        for i in range(G):
            o = OracleGrid(voxel, trunc, shard_bits)
            lib().ora_set_shard(o.h, i, G)
            oshards.append(o)
    cross = 0
    try:
        for f in range(frames):
            fr = synth.render(cam, stride * f)
            ht, lt = (fr["ht"], fr["lt"]) if semantic else (None, None)
            fr = dict(fr, ht=ht, lt=lt)
            group.integrate(fr["rgb"], fr["depth"], ht, lt, cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD,
                            count=True)
            full.integrate(fr["rgb"], fr["depth"], ht, lt, MAXD, cam.K, fr["q"], fr["t"])
            if oshards:
                oracle_shard_frame(oshards, fr, cam, MAXD, split=split)
                cross += oshards[0].stats()["last_cross_losses"]
            st = group.stats()
            assert all(s["status"] == 0 for s in st), (f, st)
            fs = full.stats()
            assert sum(s["last_num_visible"] for s in st) == fs["last_num_visible"], (f, st, fs)
            assert sum(s["last_num_updated"] for s in st) == fs["last_num_updated"], (f, st, fs)
            assert sum(s["active_blocks"] for s in st) == fs["active_blocks"], (f, st, fs)
        dumps = [e.dump() for e in group.engines]
        nblk = assert_union_equals(dumps, full.dump(), tag=f"G={G}")
        for i, o in enumerate(oshards):
            compare(group.engines[i], o, tag=f"shard {i}/{G}")
        return nblk, cross, group
    except Exception:
        group.close()
        raise
    finally:
        full.close()
        for o in oshards:
            o.close()


@pytest.mark.parametrize("G", [2, 8])
def test_sharded_c3_union_equals_unsharded(G):
    """C3 geometry (640x480 + ht/lt, 5 mm, 3 cm), 10 frames, DDA split by tile rows: the union of
    the shards is the unsharded oracle volume; each shard equals the oracle's shard."""
    nblk, cross, group = _run(G, 640, 480, 0.005, 0.03, 10, nb_bits=16, shard_bits=16 if G == 2 else 14)
    try:
        assert nblk > 5000
        assert cross > 0, "no cross-shard bucket contention: the test would not catch a per-shard resolver"
        assert group.keys_exchanged > nblk  # (few carve candidates at 5 mm in 10 frames)
    finally:
        group.close()


def test_sharded_replicated_dda_union_equals_unsharded():
    """split=False: every shard runs the whole frame's DDA (no key exchange), only carve candidates
    are exchanged; same volume. 2 cm voxels with heavy carving."""
    nblk, cross, group = _run(3, 160, 120, 0.02, 0.06, 8, nb_bits=14, shard_bits=13, split=False, stride=3)
    try:
        assert nblk > 200 and group.cands_exchanged > 50
    finally:
        group.close()


def test_sharded_c4_l515_union_equals_unsharded():
    """C4 shape: 1280x720 L515 intrinsics, 8 shards, 4 frames, depth-only."""
    from tsdf_amd import synth
    nblk, cross, group = _run(8, 1280, 720, 0.005, 0.03, 4, nb_bits=16, shard_bits=14,
                              intrinsics=synth.L515_FULL, oracle_shards=False, semantic=False)
    try:
        assert nblk > 5000
    finally:
        group.close()


def test_sharded_query_union_equals_unsharded_query():
    """SURVEY 8e Query gather: the shards' Query results, concatenated the way
    tsdf_amd.dist.gather_query concatenates ranks, equal the unsharded engine's Query as a set."""
    import tsdf_amd
    from tsdf_amd import synth
    W, H, G = 96, 72, 3
    cam = synth.camera(W, H, synth.TUM_FR1)
    full = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=13)
    group = tsdf_amd.ShardGroup(G, 0.01, 0.04, max_width=W, max_height=H, num_block_bits=13)
    try:
        for f in range(5):
            fr = synth.render(cam, 2 * f)
            for e in (full, group):
                e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
        srt = lambda a: a[np.lexsort(a.view(np.uint32).T[::-1])]
        xyz = full.query(None).view(np.float32).reshape(-1, 4)[:, :3]
        lo, hi = np.percentile(xyz, 10, axis=0), np.percentile(xyz, 90, axis=0)
        for bounds in (None, np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], np.float32)):
            exp = full.query(bounds).view(np.float32).reshape(-1, 4)
            got = np.concatenate([e.query(bounds).view(np.float32).reshape(-1, 4) for e in group.engines])
            assert got.shape == exp.shape and exp.shape[0] > 0
            np.testing.assert_array_equal(srt(got).view(np.uint32), srt(exp).view(np.uint32))
    finally:
        full.close()
        group.close()


def test_shard_protocol_misuse_and_overflow():
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, G, cap = 96, 72, 2, 4
    cam = synth.camera(W, H, synth.TUM_FR1)
    fr = synth.render(cam, 0)
    pose = tsdf_amd.SE3(fr["q"], fr["t"])
    e = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=12, shard_index=0,
                        shard_count=G)
    slot = lambda c, n=1: torch.zeros((n, tsdf_amd.Engine.shard_slot_bytes(c)), dtype=torch.uint8, device="cuda")
    try:
        with pytest.raises(tsdf_amd.TSDFError):  # a shard integrates only through the three phases
            e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD)
        with pytest.raises(tsdf_amd.TSDFError):  # no frame pending
            e.integrate_shard_update(slot(cap, G), cap, slot(cap)[0], cap)
        with pytest.raises(tsdf_amd.TSDFError):  # a split DDA needs a key slot
            e.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD, 0, G)
        keys = slot(cap, G)
        e.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD, 0, G, keys[0], cap)
        with pytest.raises(tsdf_amd.TSDFError):  # pending frame blocks snapshots / other frames
            e.snapshot()
        with pytest.raises(tsdf_amd.TSDFError):  # the key inbox is required after a packed slot
            e.integrate_shard_update(None, cap, slot(cap)[0], cap)
        cands = slot(cap, G)
        e.integrate_shard_update(keys, cap, cands[0], cap)
        with pytest.raises(tsdf_amd.TSDFError):
            e.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD, 0, G, keys[0], cap)
        e.integrate_shard_end(cands, cap)
        assert e.stats(clear_status=True)["status"] & tsdf_amd.STATUS_SHARD_OVERFLOW
    finally:
        e.close()
    u = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=12)
    try:
        with pytest.raises(tsdf_amd.TSDFError):  # an unsharded engine has no sharded frames
            u.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD)
    finally:
        u.close()


def test_sharded_snapshot_resume():
    """A shard's snapshot carries its index (foreign entries included) and restores only into the
    same shard layout; the restored shards continue the stream equal to the unsharded volume."""
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    W, H, G = 160, 120, 2
    cam = synth.camera(W, H, synth.TUM_FR1)
    group = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=14)
    other = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=14)
    full = OracleGrid(0.005, 0.03, 15)
    u = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=14)
    try:
        for f in range(6):
            fr = synth.render(cam, f)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            group.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD)
            full.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], MAXD, cam.K, fr["q"], fr["t"])
            if f == 2:
                snaps = [e.snapshot() for e in group.engines]
        with pytest.raises(tsdf_amd.TSDFError):  # shard 0's snapshot into an unsharded engine
            u.restore(snaps[0])
        with pytest.raises(tsdf_amd.TSDFError):  # into another shard index
            other.engines[1].restore(snaps[0])
        for e, s in zip(other.engines, snaps):
            e.restore(s)
        for f in range(3, 6):
            fr = synth.render(cam, f)
            other.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
        assert_union_equals([e.dump() for e in other.engines], full.dump(), tag="resumed")
    finally:
        group.close(), other.close(), full.close(), u.close()
