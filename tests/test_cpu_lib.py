"""CPU-only checks of the boundary: the C-ABI library loads and exports every symbol that
include/disinfect_tsdf.h declares, and the pure host helpers agree with the oracle. No GPU calls."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "disinfect_tsdf.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tsdf_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header():
    import ctypes
    import tsdf_amd
    from tsdf_amd import _lib
    L = tsdf_amd.load_library()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), f"missing export {s}"
    assert sorted(_lib.EXPORTS) == syms
    assert isinstance(L._name, str) and L._name.endswith("libdisinfect_tsdf.so")
    del ctypes


def test_config_default_is_reference():
    import ctypes as C
    from tsdf_amd import _lib
    L = _lib.load()
    c = _lib.Config()
    L.tsdf_config_default(C.byref(c))
    assert abs(c.voxel_size - 0.005) < 1e-9 and abs(c.truncation - 0.03) < 1e-9
    assert (c.max_width, c.max_height, c.num_block_bits) == (1920, 1080, 18)
    assert (c.shard_index, c.shard_count) == (0, 1)


def test_hash_matches_oracle():
    import tsdf_amd
    from _oracle import hash_block
    rng = np.random.default_rng(7)
    for k in rng.integers(-32768, 32767, size=(500, 3)):
        assert tsdf_amd.hash_block(*map(int, k)) == hash_block(*map(int, k))


def test_block_owner_balanced():
    import tsdf_amd
    rng = np.random.default_rng(3)
    keys = rng.integers(-400, 400, size=(4000, 3))
    own = np.array([tsdf_amd.block_owner(*map(int, k), 8) for k in keys])
    assert own.min() == 0 and own.max() == 7
    counts = np.bincount(own, minlength=8)
    assert counts.min() > 350
    # bricks of 4^3 blocks stay on one shard
    for k in keys[:50]:
        b = (k // 4) * 4
        o = {tsdf_amd.block_owner(int(b[0] + dx), int(b[1] + dy), int(b[2] + dz), 8)
             for dx in range(4) for dy in range(4) for dz in range(4)}
        assert len(o) == 1
    assert tsdf_amd.block_owner(5, 6, 7, 1) == 0


def test_se3_matches_reference_formulas():
    """SE3 composition / inverse keep the reference's host float order (lie_group.cuh)."""
    import tsdf_amd
    from tsdf_amd import synth
    (_, _), (q, t) = synth.pose(11)
    T = tsdf_amd.SE3(q, t)
    I = T * T.Inverse()
    assert np.allclose(I.q, [0, 0, 0, 1], atol=1e-6) and np.allclose(I.t, 0, atol=1e-5)
    v = np.array([0.3, -1.2, 2.5], np.float32)
    assert np.allclose(T.Inverse().Apply(T.Apply(v)), v, atol=1e-5)


def test_synth_deterministic():
    from tsdf_amd import synth
    cam = synth.camera(64, 48)
    a, b = synth.render(cam, 5), synth.render(cam, 5)
    for k in ("rgb", "depth", "ht", "lt", "q", "t"):
        assert np.array_equal(a[k], b[k])
    d = a["depth"]
    assert d.dtype == np.float32 and d.max() <= synth.MAX_RANGE and (d > 0).mean() > 0.9
    assert np.all(a["ht"] >= 0.02) and np.all(a["ht"] <= 0.98)
    assert np.allclose(a["ht"] + a["lt"], 1.0, atol=1e-6)


def test_block_owner_matches_oracle():
    import tsdf_amd
    from _oracle import block_owner
    rng = np.random.default_rng(7)
    for k in rng.integers(-2000, 2000, size=(500, 3)):
        for n in (2, 3, 8):
            assert tsdf_amd.block_owner(*map(int, k), n) == block_owner(*map(int, k), n)


def test_weight_rounding_identity():
    """k_integrate's weight update min(roundf(wc), 40) (voxel_tsdf.cu:188) is computed as
    trunc(RN(wc + 0x1.fffffep-2)) (csrc/tsdf_device.h weight_round_cap): exhaustive over every
    float wc in [0, 64) -- weights are at most 40 + 4 -- against roundf (half away from zero)."""
    c = np.float32(float.fromhex("0x1.fffffep-2"))
    hi = int(np.float32(64.0).view(np.uint32))
    step = 1 << 24
    for lo in range(0, hi, step):
        w = np.arange(lo, min(hi, lo + step), dtype=np.uint32).view(np.float32)
        fast = (w + c).astype(np.uint32)  # float32 add (RN), truncating convert
        ref = np.floor(w.astype(np.float64) + 0.5).astype(np.uint32)  # roundf for w >= 0
        bad = np.nonzero(fast != ref)[0]
        assert bad.size == 0, f"mismatch at w={w[bad[0]]!r}"
