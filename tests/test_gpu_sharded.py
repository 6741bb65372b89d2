"""Spatially sharded volume on one GPU: G shard engines of ONE volume, exchanging
their key and carve-candidate slots by device copies where a multi-GPU job all-gathers them
(tsdf_amd.ShardGroup; tsdf_amd.dist.integrate_sharded over RCCL).

The bar (SURVEY 8e "compared to single-GPU as sets keyed by block position"):
the union of the shards equals the UNSHARDED volume -- the same live block positions, every voxel's
tsdf / rgb / weight / probability bit-identical -- and every shard's hash index equals
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
         oracle_shards=True, semantic=True, graph=False, pipe=False, checks=None):
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid, lib
    cam = synth.camera(W, H, intrinsics or synth.TUM_FR1)
    group = tsdf_amd.ShardGroup(G, voxel, trunc, max_width=W, max_height=H, num_block_bits=shard_bits,
                                split=split, graph=(W, H) if graph else None, pipe=pipe)
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
            if graph:  # graph frames take device frames
                dv = {k: None if fr[k] is None else torch.from_numpy(np.ascontiguousarray(fr[k])).cuda()
                      for k in ("rgb", "depth", "ht", "lt")}
                group.integrate(dv["rgb"], dv["depth"], dv["ht"], dv["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]),
                                MAXD, count=True)
            else:
                group.integrate(fr["rgb"], fr["depth"], ht, lt, cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD,
                                count=True)
            full.integrate(fr["rgb"], fr["depth"], ht, lt, MAXD, cam.K, fr["q"], fr["t"])
            if oshards:
                oracle_shard_frame(oshards, fr, cam, MAXD, split=split)
                cross += oshards[0].stats()["last_cross_losses"]
            if checks is not None and f not in checks:  # (pipelined: a read completes the frames)
                continue
            st = group.stats()
            assert all(s["status"] == 0 for s in st), (f, st)
            fs = full.stats()
            assert sum(s["last_num_visible"] for s in st) == fs["last_num_visible"], (f, st, fs)
            assert sum(s["last_num_updated"] for s in st) == fs["last_num_updated"], (f, st, fs)
            assert sum(s["active_blocks"] for s in st) == fs["active_blocks"], (f, st, fs)
        group.flush()
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
    """C4 as configured: 1280x720 L515 intrinsics, depth + ht / lt, 8 routed shards (DDA split by
    tile rows, keys and candidates exchanged), 10 frames: the union equals the unsharded oracle and
    every shard its oracle shard."""
    from tsdf_amd import synth
    nblk, cross, group = _run(8, 1280, 720, 0.005, 0.03, 10, nb_bits=17, shard_bits=14,
                              intrinsics=synth.L515_FULL, oracle_shards=True, semantic=True)
    try:
        assert nblk > 5000
        assert cross > 0
    finally:
        group.close()


def test_sharded_routed_heavy_carving():
    """Routed exchange (split DDA) under heavy carving: 8 shards, 2 cm voxels, 20 frames of a fast
    orbit -- carve candidates of several shards are deleted from every shard's index each frame; the
    union stays the unsharded oracle volume and every shard its oracle shard."""
    nblk, cross, group = _run(8, 160, 120, 0.02, 0.06, 20, nb_bits=14, shard_bits=12, split=True, stride=3)
    try:
        assert nblk > 200
        assert group.cands_exchanged > 100, group.cands_exchanged
        assert sum(1 for c in group.cands_by_shard if c > 0) >= 4, group.cands_by_shard
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


def _no_owned_voxelless_entries(group):
    """No shard keeps an entry of a block it owns without voxels (an exhausted owner's
    kForeignIdx entry would hide the key from the DDA forever)."""
    import tsdf_amd
    for i, e in enumerate(group.engines):
        d = e.dump(pool=False)
        foreign = np.flatnonzero(d["entry_idx"] == tsdf_amd.FOREIGN_IDX)
        for p in d["entry_pos"][foreign, :3]:
            assert tsdf_amd.block_owner(int(p[0]), int(p[1]), int(p[2]), group.G) != i, \
                f"shard {i} owns block {tuple(p)} but holds no voxels for it"


def test_sharded_pool_exhaustion_matches_oracle_shards():
    """Shard pools far smaller than the scene: owned keys an exhausted pool cannot hold are carved in
    the same frame on every shard (the key is retried when the DDA meets it again, as one volume
    retries a dropped insert). Every shard stays bit-exact against the oracle's shard, and no shard
    is left with a voxel-less entry of a block it owns."""
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid, lib
    W, H, G, bits = 160, 120, 3, 8
    cam = synth.camera(W, H, synth.TUM_FR1)
    group = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=bits)
    oshards = []
    for i in range(G):
        o = OracleGrid(0.005, 0.03, bits)
        lib().ora_set_shard(o.h, i, G)
        oshards.append(o)
    try:
        exhausted = 0
        for f in range(8):
            fr = synth.render(cam, 2 * f)
            group.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
            oracle_shard_frame(oshards, fr, cam, MAXD, split=True)
            st = group.stats()
            assert all((s["status"] & ~tsdf_amd.STATUS_POOL_EXHAUSTED) == 0 for s in st), [s["status"] for s in st]
            exhausted += sum(bool(s["status"] & tsdf_amd.STATUS_POOL_EXHAUSTED) for s in st)
            for i, o in enumerate(oshards):
                compare(group.engines[i], o, tag=f"frame {f} shard {i}/{G}")
            _no_owned_voxelless_entries(group)
        assert exhausted > 0, "the pools never ran out: the test would not exercise exhaustion"
    finally:
        group.close()
        for o in oshards:
            o.close()


def test_sharded_candidate_union_overflow_is_clamped():
    """the union of the shards' candidate slots can exceed the records a shard's
    carving list holds. It is clamped with TSDF_STATUS_SHARD_OVERFLOW instead of
    being written past the list; later frames still run and every pool index stays in range."""
    import tsdf_amd
    from tsdf_amd import synth
    import os
    W, H, G, bits, cap = 640, 480, 8, 8, 1024  # pools of 256: thousands of voxel-less entries to carve
    cam = synth.camera(W, H, synth.TUM_FR1)
    os.environ["TSDF_CAND_CAP"] = str(cap)  # a 1024-record carving list (default: 2^17)
    try:
        group = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=bits,
                                    key_cap=16384, cand_cap=16384)
    finally:
        del os.environ["TSDF_CAND_CAP"]
    try:
        prev, big = 0, False
        for f in range(4):
            fr = synth.render(cam, 4 * f)
            group.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]),
                            MAXD, count=True)
            n = group.cands_exchanged - prev
            prev = group.cands_exchanged
            st = group.stats()
            if n > cap:
                big = True
                assert all(s["status"] & tsdf_amd.STATUS_SHARD_OVERFLOW for s in st), (f, n, st)
            for e in group.engines:
                e.stats(clear_status=True)
        assert big, "no frame exchanged more candidates than the list holds"
        for e in group.engines:
            d = e.dump(pool=False)
            idx = d["entry_idx"]
            ok = (idx == -1) | (idx == tsdf_amd.FOREIGN_IDX) | ((idx >= 0) & (idx < (1 << bits)))
            assert ok.all()
    finally:
        group.close()


def test_shard_abort_returns_engine_between_frames():
    """a failed exchange between the phases must not strand the engine in a pending frame.
    tsdf_integrate_shard_abort clears it (STATUS_SHARD_ABORTED set); new frames, snapshots and reset
    work again."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, G, cap = 96, 72, 2, 4096
    cam = synth.camera(W, H, synth.TUM_FR1)
    fr = synth.render(cam, 0)
    pose = tsdf_amd.SE3(fr["q"], fr["t"])
    e = tsdf_amd.Engine(0.01, 0.04, max_width=W, max_height=H, num_block_bits=12, shard_index=0,
                        shard_count=G)
    slot = lambda n=1: torch.zeros((n, tsdf_amd.Engine.shard_slot_bytes(cap)), dtype=torch.uint8, device="cuda")
    try:
        e.integrate_shard_abort()  # nothing pending: a no-op
        assert e.stats()["status"] == 0
        for phases in (1, 2):
            keys, cands = slot(G), slot(G)
            e.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD, 0, G, keys[0], cap)
            if phases == 2:
                e.integrate_shard_update(keys, cap, cands[0], cap)
            with pytest.raises(tsdf_amd.TSDFError):
                e.snapshot()
            e.integrate_shard_abort()
            assert e.stats(clear_status=True)["status"] & tsdf_amd.STATUS_SHARD_ABORTED
            e.snapshot()
        e.reset()
        # a whole frame runs after the aborts, and the per-frame state was cleared (no stale keys)
        keys, cands = slot(G), slot(G)
        e.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD, 0, G, keys[0], cap)
        e.integrate_shard_update(keys, cap, cands[0], cap)
        e.integrate_shard_end(cands, cap)
        assert e.stats()["status"] == 0 and e.stats()["active_blocks"] > 0
    finally:
        e.close()


def test_shard_pipe_abort_mid_step_and_recover():
    """a failure part-way through a pipelined sharded step (one shard has launched its
    k_frame, the next raises) aborts every shard -- the pending pipelined frames are dropped with
    STATUS_SHARD_ABORTED, nothing stays stuck (stats / snapshot / reset work) -- and after a reset the
    group integrates a stream exactly like a fresh group (every shard's table and voxels). count=True
    counts the pipelined slots' candidates."""
    import tsdf_amd
    from tsdf_amd import synth
    W, H, G = 160, 120, 2
    cam = synth.camera(W, H, synth.TUM_FR1)
    frames = [synth.render(cam, 3 * f) for f in range(6)]
    mk = lambda: tsdf_amd.ShardGroup(G, 0.01, 0.04, max_width=W, max_height=H, num_block_bits=13, split=False,
                                     pipe=True, cand_cap=4096)
    step = lambda g, fr, **kw: g.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K,
                                           tsdf_amd.SE3(fr["q"], fr["t"]), MAXD, **kw)
    group, fresh = mk(), mk()
    try:
        for fr in frames[:3]:
            step(group, fr, count=True)
        assert group.cands_exchanged >= 0 and len(group.cands_by_shard) == G
        real = group.engines[1].integrate_shard_pipe

        def boom(*a, **k):
            raise RuntimeError("injected exchange failure")
        group.engines[1].integrate_shard_pipe = boom
        with pytest.raises(RuntimeError, match="injected"):
            step(group, frames[3])
        group.engines[1].integrate_shard_pipe = real
        for e in group.engines:  # both shards dropped their pending frames
            assert e.stats(clear_status=True)["status"] & tsdf_amd.STATUS_SHARD_ABORTED
            e.snapshot()  # (between frames again: no pending frame to flush)
            e.reset()
        for fr in frames:
            step(group, fr)
            step(fresh, fr)
        group.flush()
        fresh.flush()
        for a, b in zip(group.engines, fresh.engines):
            assert a.stats()["status"] == 0 and b.stats()["status"] == 0
            da, db = a.dump(), b.dump()
            for k in ("entry_pos", "entry_idx", "heap", "tsdf", "rgbw"):
                assert np.array_equal(da[k], db[k]), k
            assert a.stats()["active_blocks"] > 0
    finally:
        group.close()
        fresh.close()


@pytest.mark.parametrize("split", [True, False])
def test_sharded_graph_frames_equal_oracle(split):
    """C5 on a sharded volume: every shard's frame as its three captured graph segments
    (tsdf_graph_create_shard) around the exchanges -- each shard still equals the oracle's shard and
    the union the unsharded oracle volume."""
    nblk, cross, group = _run(3, 160, 120, 0.005, 0.03, 6, nb_bits=15, shard_bits=14, split=split, graph=True)
    try:
        assert nblk > 500
    finally:
        group.close()


@pytest.mark.parametrize("G", [2, 8])
def test_sharded_pipe_c3_union_equals_unsharded(G):
    """Pipelined sharded frames (tsdf_integrate_shard_pipe: one exchange per frame, every shard runs
    the whole DDA): C3 640x480, 12 frames back to back with one mid-stream read (which completes the
    pending frames through the exchange protocol): the union is the unsharded oracle volume, each
    shard its oracle shard."""
    nblk, cross, group = _run(G, 640, 480, 0.005, 0.03, 12, nb_bits=16, shard_bits=16 if G == 2 else 14,
                              split=False, pipe=True, checks={5})
    try:
        assert nblk > 5000
    finally:
        group.close()


def test_sharded_pipe_heavy_carving():
    """Pipelined sharded frames under heavy carving (2 cm, fast orbit, 8 shards, 20 frames back to
    back): carvings of every shard's candidates run a frame late beside the next frame's update,
    deleted keys the next frame's DDA had found are re-inserted; shards stay bit-exact against the
    oracle's."""
    nblk, cross, group = _run(8, 160, 120, 0.02, 0.06, 20, nb_bits=14, shard_bits=12, split=False, stride=3,
                              pipe=True, checks={9})
    try:
        assert nblk > 200
    finally:
        group.close()


def test_sharded_pipe_pool_exhaustion_matches_oracle_shards():
    """Pipelined sharded frames with shard pools far smaller than the scene: the owned entries an
    exhausted pool leaves without voxels go out with the candidates and are carved on every shard."""
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid, lib
    W, H, G, bits = 160, 120, 3, 8
    cam = synth.camera(W, H, synth.TUM_FR1)
    group = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=bits, split=False,
                                pipe=True)
    oshards = []
    for i in range(G):
        o = OracleGrid(0.005, 0.03, bits)
        lib().ora_set_shard(o.h, i, G)
        oshards.append(o)
    try:
        for f in range(8):
            fr = synth.render(cam, 2 * f)
            group.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
            oracle_shard_frame(oshards, fr, cam, MAXD, split=False)
        st = group.stats()
        assert any(s["status"] & tsdf_amd.STATUS_POOL_EXHAUSTED for s in st)
        assert all((s["status"] & ~tsdf_amd.STATUS_POOL_EXHAUSTED) == 0 for s in st), [s["status"] for s in st]
        for i, o in enumerate(oshards):
            compare(group.engines[i], o, tag=f"shard {i}/{G}")
        _no_owned_voxelless_entries(group)
    finally:
        group.close()
        for o in oshards:
            o.close()


def test_sharded_pipe_protocol():
    """Reads are refused while pipelined sharded frames are pending (only the exchange protocol can
    complete them); flush() completes them, after which reads work and a new stream starts."""
    import tsdf_amd
    from tsdf_amd import synth
    cam = synth.camera(80, 60, synth.TUM_FR1)
    group = tsdf_amd.ShardGroup(2, 0.01, 0.04, max_width=80, max_height=60, num_block_bits=12, split=False,
                                pipe=True)
    try:
        for f in range(3):
            fr = synth.render(cam, f)
            group.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
        with pytest.raises(tsdf_amd.TSDFError):
            group.engines[0].dump()
        group.flush()
        assert all(s["status"] == 0 and s["frames"] == 3 for s in group.stats())
        fr = synth.render(cam, 3)
        group.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), MAXD)
        assert all(s["frames"] == 4 for s in group.stats())
    finally:
        group.close()


def test_shard_frame_buffers_may_be_dropped_after_begin():
    """a shard's update reads the raw device frame it was given at _begin. The
    Python wrapper keeps that frame referenced until _update, so a caller may pass temporaries and
    drop them at once; here every frame tensor is a temporary, torch's cache is emptied and refilled
    with garbage of the same size between _begin and _update, and the volume still equals a
    ShardGroup's (which holds its frames)."""
    import gc

    import torch

    import tsdf_amd
    from tsdf_amd import synth
    W, H, G = 160, 120, 2
    cam = synth.camera(W, H, synth.TUM_FR1)
    ref = tsdf_amd.ShardGroup(G, 0.02, 0.08, max_width=W, max_height=H, num_block_bits=12, split=False)
    eng = [tsdf_amd.Engine(0.02, 0.08, W, H, 12, 0, shard_index=i, shard_count=G,
                           stream=torch.cuda.current_stream(0)) for i in range(G)]
    cap = 4096
    cands = torch.zeros((G, tsdf_amd.Engine.shard_slot_bytes(cap)), dtype=torch.uint8, device="cuda")
    try:
        for f in range(6):
            fr = synth.render(cam, 3 * f)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            ref.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, MAXD)
            dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
            for e in eng:
                e.integrate_shard_begin(dev(fr["rgb"]), dev(fr["depth"]), dev(fr["ht"]), dev(fr["lt"]), cam.K,
                                        pose, MAXD)
            gc.collect()
            torch.cuda.empty_cache()
            junk = [torch.full((H, W), -7.0, device="cuda") for _ in range(16)]
            junk += [torch.full((H, W, 3), 255, dtype=torch.uint8, device="cuda") for _ in range(8)]
            for i, e in enumerate(eng):
                e.integrate_shard_update(None, 0, cands[i], cap)
            for e in eng:
                e.integrate_shard_end(cands, cap)
            del junk
        ref.flush()
        for a, b in zip(ref.engines, eng):
            da, db = a.dump(), b.dump()
            assert set(da) == set(db)
            for k in da:
                np.testing.assert_array_equal(np.asarray(da[k]), np.asarray(db[k]), err_msg=k)
    finally:
        ref.close()
        for e in eng:
            e.close()
