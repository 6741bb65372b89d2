"""The CPU oracle against the committed golden fixtures (tests/golden/, made by make_golden.py).

kat_reference.json holds the reference's own known-answer vectors (voxel_hash_test.cu /
voxel_mem_test.cu) as data; integrate_48x36.npz holds a small synthetic stream and the oracle's
outputs, which pins the restatement against drift (parity unpinned vs the CUDA reference itself,
which cannot run here -- SURVEY.md 8c).
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

from _oracle import OracleGrid, hash_block

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


STREAMS = ["integrate_48x36.npz", "integrate_48x36_independent.npz", "integrate_48x36_u16.npz",
           "integrate_48x36_u16z.npz"]


def load_stream(name="integrate_48x36.npz"):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


def prob_same(a, b):
    """Bit-identical where both are numbers, NaN where either is (any payload)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32)))


def test_reference_kat_vectors():
    kat = json.load(open(os.path.join(GOLD, "kat_reference.json")))
    for h in kat["hash"]:
        assert hash_block(*h["key"]) == h["bucket"]
    col = kat["collision"]
    keys = np.asarray(col["keys"], np.int16)
    # the reference's four threads race; the canonical linearisation must give 2 -> 3 -> 4 for
    # every order of the launch's four keys
    for perm in itertools.permutations(range(4)):
        g = OracleGrid(0.01, 0.06, num_block_bits=12)
        try:
            for launch in range(col["launches"]):
                g.hash_allocate(keys[list(perm)])  # all four keys, one Allocate launch
                assert g.num_active_blocks() == col["active_after_each"][launch], (perm, launch)
            points = keys.astype(np.int32) * 8  # the first voxel of each block (:157-161)
            rgbw = np.asarray(col["assign_rgbw"], np.uint8)
            assert g.hash_assign(points, rgbw) == 0
            r = g.hash_retrieve(points)
            np.testing.assert_array_equal(r["rgbw"], rgbw)
            np.testing.assert_array_equal(r["block_pos_off"][:, :3], keys)
        finally:
            g.close()


def run_oracle(G):
    ora = OracleGrid(float(G["voxel"]), float(G["trunc"]), int(G["num_block_bits"]))
    stats = []
    for f in range(G["depth"].shape[0]):
        ora.integrate(G["rgb"][f], G["depth"][f], G["ht"][f], G["lt"][f], float(G["max_depth"]),
                      G["K"], G["q"][f], G["t"][f])
        s = ora.stats()
        stats.append([s["last_num_visible"], s["last_num_updated"], s["last_num_deleted"],
                      s["active_blocks"]])
    return ora, np.asarray(stats)


@pytest.mark.parametrize("name", STREAMS)
def test_oracle_reproduces_golden_stream(name):
    G = load_stream(name)
    ora, stats = run_oracle(G)
    try:
        np.testing.assert_array_equal(stats, G["stats"])
        d = ora.dump()
        live = np.flatnonzero(d["entry_idx"] >= 0)
        np.testing.assert_array_equal(live, G["live_entry"])
        np.testing.assert_array_equal(d["entry_pos"][live], G["live_pos"])
        idx = d["entry_idx"][live]
        np.testing.assert_array_equal(idx, G["live_idx"])
        np.testing.assert_array_equal(d["heap"], G["heap"])
        assert d["free"] == int(G["free"])
        blk = lambda a: a.reshape(-1, 512, *a.shape[1:])[idx]
        np.testing.assert_array_equal(blk(d["tsdf"]).view(np.uint32), G["tsdf"].view(np.uint32))
        np.testing.assert_array_equal(blk(d["rgbw"]), G["rgbw"])
        assert prob_same(blk(d["prob"]), G["prob"])
        rgba, normal = ora.raycast(G["K"], int(G["W"]), int(G["H"]), G["q"][-1], G["t"][-1],
                                   float(G["max_depth"]))
        np.testing.assert_array_equal(rgba, G["rgba"])
        np.testing.assert_array_equal(normal, G["normal"])
        q = ora.query(None)
        assert q.shape[0] == int(G["query_count"])
        assert hashlib.sha256(np.ascontiguousarray(q)).digest() == G["query_sha256"].tobytes()
    finally:
        ora.close()
