"""HIP engine vs CPU oracle parity on identical synthetic frames.

Bar: hash entries, pool indices, free-block stack, TSDF values, RGB, weights AND the semantic
probability bit-exact (BASELINE.json north_star asks 1e-4 for the probability; the engine computes the
reference's own float chain with the oracle's logf / expf, oracle/ora_math.c, so it is exact -- NaN
where the reference's chain is 0 / 0 compares equal to NaN); raycast images bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PROB_TOL = 0.0  # the probability is bit-exact (NaN == NaN); kept for the tests that print a bound


def prob_equal(a, b):
    """Bit-identical float arrays where NaN (any payload) equals NaN: the reference's chain gives
    0 / 0 = NaN where a voxel sees ht = lt = 0, and NaN payloads differ between x86 and gfx950."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32)))


def prob_diff(a, b):
    """(voxels whose probability bits differ, NaN-pattern mismatches, largest |difference|)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    both = ~na & ~nb
    bad = both & (a.view(np.uint32) != b.view(np.uint32))
    return int(bad.sum()), int((na != nb).sum()), float(np.abs(a[both] - b[both]).max()) if both.any() else 0.0


def np_hash(k):
    u = k.astype(np.int64) & 0xFFFFFFFF
    M = 0xFFFFFFFF
    return (((u[:, 0] * 73856093) & M) ^ ((u[:, 1] * 19349669) & M) ^ ((u[:, 2] * 83492791) & M)) & ((1 << 21) - 1)


def compare(eng, ora, pool=True, tag=""):
    a, b = eng.dump(pool=pool), ora.dump(pool=pool)
    assert np.array_equal(a["entry_pos"], b["entry_pos"]), f"{tag}: entries differ"
    assert np.array_equal(a["entry_idx"], b["entry_idx"]), f"{tag}: pool indices differ"
    assert a["free"] == b["free"], f"{tag}: free count {a['free']} vs {b['free']}"
    assert np.array_equal(a["heap"], b["heap"]), f"{tag}: heap differs"
    if pool:
        ta, tb = a["tsdf"].view(np.uint32), b["tsdf"].view(np.uint32)
        bad = np.flatnonzero(ta != tb)
        assert bad.size == 0, f"{tag}: {bad.size} tsdf voxels differ, first {bad[:5]}: {a['tsdf'][bad[:5]]} vs {b['tsdf'][bad[:5]]}"
        assert np.array_equal(a["rgbw"], b["rgbw"]), f"{tag}: rgbw differs"
        assert prob_equal(a["prob"], b["prob"]), f"{tag}: prob differs (bits, NaN pattern, max): {prob_diff(a['prob'], b['prob'])}"


def run_sequence(W, H, voxel, trunc, frames, nb_bits=14, semantic=True, check_every=1,
                 intrinsics=None, start=0, touch="complement"):
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    cam = synth.camera(W, H, intrinsics or synth.TUM_FR1)
    eng = tsdf_amd.Engine(voxel, trunc, max_width=W, max_height=H, num_block_bits=nb_bits)
    ora = OracleGrid(voxel, trunc, nb_bits)
    try:
        for f in range(start, start + frames):
            fr = synth.render(cam, f, touch=touch)
            ht = fr["ht"] if semantic else None
            lt = fr["lt"] if semantic else None
            eng.integrate(fr["rgb"], fr["depth"], ht, lt, cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
            ora.integrate(fr["rgb"], fr["depth"], ht, lt, 4.0, cam.K, fr["q"], fr["t"])
            s, so = eng.stats(), ora.stats()
            assert s["status"] == 0, s
            assert s["last_num_visible"] == so["last_num_visible"], (f, s, so)
            assert s["last_num_updated"] == so["last_num_updated"], (f, s, so)
            assert s["last_num_deleted"] == so["last_num_deleted"], (f, s, so)
            assert s["active_blocks"] == so["active_blocks"], (f, s, so)
            if (f - start + 1) % check_every == 0 or f == start + frames - 1:
                compare(eng, ora, tag=f"frame {f}")
        return eng, ora, cam
    except Exception:
        eng.close()
        ora.close()
        raise


def test_integrate_semantic_160x120():
    eng, ora, cam = run_sequence(160, 120, 0.005, 0.03, 6, check_every=2)
    eng.close(), ora.close()


def test_integrate_depth_only_80x60():
    """Config C2 shape: ht = lt = NULL -> ones (tsdf_module.cc:29-33), p stays 0.5 exactly."""
    eng, ora, cam = run_sequence(80, 60, 0.005, 0.03, 5, semantic=False, check_every=5)
    a = eng.dump()
    live = a["entry_idx"][a["entry_idx"] >= 0]
    probs = a["prob"].reshape(-1, 512)[live]
    assert np.all(probs == 0.5)
    eng.close(), ora.close()


def test_integrate_coarse_voxels_carving():
    """2 cm voxels / 8 cm truncation: more DDA samples per pixel and blocks carved every frame."""
    eng, ora, cam = run_sequence(96, 72, 0.02, 0.08, 8, nb_bits=13, check_every=4)
    eng.close(), ora.close()


def test_raycast_and_query_parity():
    import tsdf_amd
    from tsdf_amd import synth
    eng, ora, cam = run_sequence(120, 90, 0.005, 0.03, 4, check_every=4)
    try:
        for f in (3, 7):
            (_, _), (q, t) = synth.pose(f)
            rgba, nrm = eng.raycast(cam.K, cam.width, cam.height, tsdf_amd.SE3(q, t), 4.0)
            rgba_o, nrm_o = ora.raycast(cam.K, cam.width, cam.height, q, t, 4.0)
            hit = rgba[..., 3] == 255
            assert hit.mean() > 0.5
            assert np.array_equal(rgba[..., 3], rgba_o[..., 3])
            # colour and shading blend with the probability (alpha): exact with the exact probability
            np.testing.assert_array_equal(rgba, rgba_o)
            np.testing.assert_array_equal(nrm, nrm_o)
        got = eng.query(None)
        exp = ora.query(None)
        assert got.shape[0] == exp.shape[0] > 0
        np.testing.assert_array_equal(np.stack([got[k] for k in "xyz"], 1), exp[:, :3])
        np.testing.assert_array_equal(got["tsdf"].view(np.uint32), exp[:, 3].view(np.uint32))
        xyz = np.stack([got[k] for k in "xyz"], 1)
        lo, hi = np.percentile(xyz, 20, axis=0), np.percentile(xyz, 80, axis=0)
        bounds = tsdf_amd.BoundingCube(lo[0], hi[0], lo[1], hi[1], lo[2], hi[2])
        got = eng.query(bounds)
        exp = ora.query(bounds.as_array())
        assert got.shape[0] == exp.shape[0] > 0
        np.testing.assert_array_equal(got["tsdf"].view(np.uint32), exp[:, 3].view(np.uint32))
        np.testing.assert_array_equal(np.stack([got[k] for k in "xyz"], 1), exp[:, :3])
    finally:
        eng.close(), ora.close()


def _colliding_keys(rng, n_buckets=400, per_bucket=4):
    g = np.stack(np.meshgrid(*(np.arange(-48, 48),) * 3, indexing="ij"), -1).reshape(-1, 3).astype(np.int16)
    h = np_hash(g)
    order = np.argsort(h, kind="stable")
    hs = h[order]
    starts = np.flatnonzero(np.r_[True, hs[1:] != hs[:-1]])
    counts = np.diff(np.r_[starts, hs.size])
    multi = starts[counts >= per_bucket]
    pick = rng.choice(multi, size=min(n_buckets, multi.size), replace=False)
    keys = np.concatenate([g[order[s:s + per_bucket]] for s in pick])
    # neighbours of last buckets exercise the wrap-around of the list probe
    return keys


def test_hash_stress_allocate_delete():
    """Random launches of colliding keys: chains, appends, head / element deletes, lock losses."""
    import tsdf_amd
    from _oracle import OracleGrid
    rng = np.random.default_rng(1234)
    eng = tsdf_amd.Engine(0.01, 0.06, max_width=128, max_height=128, num_block_bits=14)
    ora = OracleGrid(0.01, 0.06, 14)
    try:
        keys = _colliding_keys(rng)
        extra = rng.integers(-300, 300, size=(4000, 3)).astype(np.int16)
        allkeys = np.concatenate([keys, extra])
        for it in range(12):
            batch = allkeys[rng.choice(allkeys.shape[0], size=3000)]
            eng.hash_allocate(batch)
            ora.hash_allocate(batch)
            compare(eng, ora, pool=False, tag=f"alloc {it}")
            if it % 3 == 2:
                dk = allkeys[rng.choice(allkeys.shape[0], size=700, replace=False)]
                eng.hash_delete(dk)
                ora.hash_delete(dk)
                compare(eng, ora, pool=False, tag=f"delete {it}")
        assert eng.num_active_blocks() == ora.num_active_blocks() > 1000
    finally:
        eng.close(), ora.close()


def test_pool_exhaustion_is_reported():
    import tsdf_amd
    from _oracle import OracleGrid
    eng = tsdf_amd.Engine(0.01, 0.06, max_width=64, max_height=64, num_block_bits=6)
    ora = OracleGrid(0.01, 0.06, 6)
    try:
        keys = np.array([[i, 2 * i, 3] for i in range(200)], np.int16)
        eng.hash_allocate(keys)
        ora.hash_allocate(keys)
        assert eng.num_active_blocks() == 64
        assert eng.stats()["status"] & tsdf_amd.STATUS_POOL_EXHAUSTED
        compare(eng, ora, pool=False, tag="exhausted")
    finally:
        eng.close(), ora.close()


@pytest.mark.parametrize("min_weight,bounded,grid", [(0, False, 0), (1, False, 0), (1, True, 0), (0, False, 7)])
def test_marching_cubes_matches_oracle(min_weight, bounded, grid, monkeypatch):
    """GPU marching cubes (tsdf_extract_mesh) == the oracle's restatement, bit for bit and in
    the same order (KrisLibrary itself is absent: parity unpinned). grid: k_mesh
    workgroups (TSDF_MESH_GRID; 7 walks the selection grid-stride, as selections past kMeshGrid do)."""
    import tsdf_amd
    if grid:
        monkeypatch.setenv("TSDF_MESH_GRID", str(grid))
    eng, ora, cam = run_sequence(96, 72, 0.01, 0.04, 4, nb_bits=13, check_every=4)
    try:
        bounds = None
        if bounded:
            d = ora.dump(pool=False)
            pos = d["entry_pos"][d["entry_idx"] >= 0, :3].astype(np.float32) * 8 * 0.01
            lo, hi = np.percentile(pos, 5, axis=0), np.percentile(pos, 95, axis=0) + 0.08
            bounds = np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], np.float32)
        got = eng.extract_mesh(bounds, 0.99, min_weight)
        exp = ora.extract_mesh(bounds, 0.99, min_weight)
        assert exp.shape[0] > (20 if bounded else 100)
        assert got.shape == exp.shape
        np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))
        # the one-call device form (count, scan and emission enqueued together) gives the same
        # triangles; too small a buffer raises and is left untouched
        import torch
        n = exp.shape[0]
        out = torch.full((9 * n + 90,), -7.0, dtype=torch.float32, device="cuda")
        dev = eng.extract_mesh(bounds, 0.99, min_weight, out=out)
        np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint32), exp.view(np.uint32))
        assert bool((out[9 * n:] == -7.0).all())
        small = torch.full((9 * (n - 1),), -7.0, dtype=torch.float32, device="cuda")
        with pytest.raises(tsdf_amd._lib.TSDFError):
            eng.extract_mesh(bounds, 0.99, min_weight, out=small)
        assert bool((small == -7.0).all())
    finally:
        eng.close(), ora.close()
