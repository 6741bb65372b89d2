"""Sharded-volume test helpers (TEST INFRASTRUCTURE): the CPU oracle's three-phase sharded frame
driven for G shards in one process, and the block-keyed view of a volume that the sharded ==
unsharded comparisons use ("compared to single-GPU as sets keyed by block position").
"""
from __future__ import annotations

import numpy as np

FOREIGN = 0x7FFFFFFF  # entry of a block another shard owns (ORA_FOREIGN / kForeignIdx)


def row_slices(H: int, G: int, rows_per_tile: int = 16):
    """Pixel rows of each shard's DDA slice: contiguous bands of 16-row tile rows, the engine's
    split (tsdf_integrate_shard_begin, slice i of G)."""
    tiles_y = (H + rows_per_tile - 1) // rows_per_tile
    per = (tiles_y + G - 1) // G
    return [(min(tiles_y, i * per) * rows_per_tile, min(H, min(tiles_y, (i + 1) * per) * rows_per_tile))
            for i in range(G)]


def oracle_shard_frame(shards, fr, cam, max_depth=4.0, split=True):
    """One sharded frame of the oracle shards (one process): keys of every slice, union, update,
    union of the carve candidates, delete. Returns (#keys exchanged, #candidates exchanged)."""
    G = len(shards)
    H = fr["depth"].shape[0]
    K = cam.K
    if split:
        parts = [s.shard_keys(fr["depth"], K, fr["q"], fr["t"], max_depth, lo, hi)
                 for s, (lo, hi) in zip(shards, row_slices(H, G))]
    else:  # replicated DDA: every shard computes the same keys; one copy stands for all
        parts = [shards[0].shard_keys(fr["depth"], K, fr["q"], fr["t"], max_depth, 0, H)]
    keys = np.concatenate([p[0] for p in parts])
    orders = np.concatenate([p[1] for p in parts])
    cands = [s.shard_update(keys, orders, fr["rgb"], fr["depth"], fr["ht"], fr["lt"], max_depth, K,
                            fr["q"], fr["t"]) for s in shards]
    cpos = np.concatenate([c[0] for c in cands])
    cent = np.concatenate([c[1] for c in cands])
    for s in shards:
        s.shard_delete(cpos, cent)
    return keys.shape[0], cent.shape[0]


def live_blocks(dump):
    """{block position: (tsdf[512] u32 bits, rgbw[512, 4], prob[512])} of the blocks a volume
    (or shard) holds voxels for."""
    idx = dump["entry_idx"]
    live = np.flatnonzero((idx >= 0) & (idx != FOREIGN))
    pos = dump["entry_pos"][live, :3]
    pidx = idx[live]
    tsdf = dump["tsdf"].reshape(-1, 512)[pidx].view(np.uint32)
    rgbw = dump["rgbw"].reshape(-1, 512, 4)[pidx]
    prob = dump["prob"].reshape(-1, 512)[pidx]
    return {tuple(map(int, p)): (t, c, q) for p, t, c, q in zip(pos, tsdf, rgbw, prob)}


def _prob_same(a, b):
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def assert_shard_matches(shard_dump, full_dump, full=None, prob_atol=0.0, tag=""):
    """One shard against the unsharded volume: its hash index (occupied entries, positions, list
    offsets) equals the unsharded table, and each block it holds equals the unsharded block (tsdf /
    rgb / weight bit-identical; probability bit-identical, NaN == NaN, or within prob_atol > 0).
    Returns its block positions."""
    full = live_blocks(full_dump) if full is None else full
    focc = full_dump["entry_idx"] >= 0
    occ = shard_dump["entry_idx"] >= 0
    assert np.array_equal(occ, focc), f"{tag}: index occupancy differs"
    np.testing.assert_array_equal(shard_dump["entry_pos"][occ], full_dump["entry_pos"][focc],
                                  err_msg=f"{tag}: index entries differ")
    mine = live_blocks(shard_dump)
    for k, v in mine.items():
        assert k in full, f"{tag}: block {k} is not in the unsharded volume"
        ft, fc, fq = full[k]
        np.testing.assert_array_equal(v[0], ft, err_msg=f"{tag}: tsdf of block {k}")
        np.testing.assert_array_equal(v[1], fc, err_msg=f"{tag}: rgbw of block {k}")
        if prob_atol > 0:
            np.testing.assert_allclose(v[2], fq, atol=prob_atol, rtol=0, err_msg=f"{tag}: prob of block {k}")
        else:
            assert _prob_same(v[2], fq), f"{tag}: prob of block {k}"
    return set(mine)


def assert_union_equals(shard_dumps, full_dump, prob_atol=0.0, tag=""):
    """Every shard matches the unsharded volume (assert_shard_matches), the shards' blocks are
    disjoint, and their union has exactly the unsharded volume's block positions."""
    full = live_blocks(full_dump)
    seen = {}
    for i, d in enumerate(shard_dumps):
        for k in assert_shard_matches(d, full_dump, full, prob_atol, tag=f"{tag} shard {i}"):
            assert k not in seen, f"{tag}: block {k} on shards {seen[k]} and {i}"
            seen[k] = i
    missing = set(full) - set(seen)
    assert not missing, f"{tag}: {len(missing)} unsharded blocks on no shard, e.g. {sorted(missing)[:3]}"
    return len(full)
