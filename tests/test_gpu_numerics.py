"""Bit-exactness of the engine's fast quotient / conversion helpers (csrc/tsdf_device.h) on the GPU.

The integrate and ingest kernels replace the 11-op IEEE divide where an exact shortcut exists:
 - quot_const(a, b, RN(1/b))  -- Markstein-corrected quotient for frame-constant divisors
   (truncation, voxel size, max depth); checked EXHAUSTIVELY over every float a of both signs in
   the normal range for the divisors the tests and the bench use;
 - round_quot(a, b, rcp(b))   -- roundf(a / b) from a reciprocal estimate with an IEEE fallback
   near rounding boundaries (projection to pixels, colour averages); checked on 2^28 random and
   boundary-adversarial pairs per divisor range;
 - quot_for_cmp(a, b, rcp(b), c) -- a / b where only its order against 0 and c matters
   (voxel_visible's frustum test); adversarial samples at both thresholds;
 - div_pair(a, b, rcp(b))     -- the IEEE divide expansion without its range scaling (tsdf
   running average); every a in the fast range against fixed divisors, 2^28 random pairs;
 - f2i / f2s / f2u8 via v_cvt_{i,u}32_f32, and round_s16 (= f2s(roundf(f)), the raycast's voxel
   rounding) -- checked on every float bit pattern.
Each must agree bit for bit with the correctly rounded divide / cvt.rzi semantics.
And the semantic update's sem_logf / sem_expf (and the update's unit-interval logf form) must return
the oracle's bits (oracle/ora_math.c) for EVERY float input: digests of all 2^32 results per function,
in chunks of 2^24, against the committed oracle digests (tests/golden/sem_math_digests.json).
"""
import ctypes as C
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "disinfect-slam_amd", "libtsdf_selfcheck.so")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    # torch's HIP runtime first (conftest._torch_hip_first runs after module fixtures): loaded before
    # it, this library would bring up the /opt/rocm runtime as a second one in the process
    import torch
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")
    L = C.CDLL(LIB)
    u32, u64, f = C.c_uint32, C.c_uint64, C.c_float
    P64, P32 = C.POINTER(C.c_ulonglong), C.POINTER(C.c_uint32)
    L.tsdf_selfcheck_quot_const.argtypes = [f, u32, u32, P64, P32]
    L.tsdf_selfcheck_round_quot.argtypes = [u32, u64, f, f, f, P64, P32]
    L.tsdf_selfcheck_convert.argtypes = [u32, u32, P64, P32]
    L.tsdf_selfcheck_quot_cmp.argtypes = [u32, u64, f, f, f, P64, P32]
    L.tsdf_selfcheck_div_pair.argtypes = [f, u32, u32, u32, u64, f, f, P64, P32]
    L.tsdf_selfcheck_sem_digest.argtypes = [C.c_int, u64, u64, P64]
    return L


def _run(fn, *args):
    bad, first = C.c_ulonglong(), C.c_uint32()
    assert fn(*args, C.byref(bad), C.byref(first)) == 0
    return bad.value, first.value


# positive and negative normal floats up to 2^100 (larger |a| takes the IEEE path anyway)
RANGES = [(0x00800000, 0x71800000), (0x80800000, 0xF1800000)]


@pytest.mark.parametrize("b", [0.03, 0.005, 0.02, 0.04, 0.08, 0.01, 4.0, 3.0, 5.0, 0.1])
def test_quot_const_exhaustive(lib, b):
    for lo, hi in RANGES:
        bad, first = _run(lib.tsdf_selfcheck_quot_const, b, lo, hi)
        assert bad == 0, f"b={b}: {bad} mismatches, first a bits {first:#x}"


def test_quot_const_edges(lib):
    # zero, denormals, huge values, inf, NaN: the helper must route them to the IEEE divide
    for lo, hi in [(0, 0x00800000), (0x80000000, 0x80800000), (0x71800000, 0x80000000),
                   (0xF1800000, 0xFFFFFFFF)]:
        bad, first = _run(lib.tsdf_selfcheck_quot_const, 0.03, lo, hi)
        assert bad == 0, f"{bad} mismatches, first a bits {first:#x}"


@pytest.mark.parametrize("bmin,bmax,qmax", [
    (0.05, 10.0, 2000.0),     # projection: hz in metres, pixel coordinates
    (1e-3, 0.05, 2000.0),     # voxels close to the camera plane
    (1e-4, 44.0, 256.0),      # colour averages: wc = w_old + w_new in (0, 44]
    (0.5, 44.0, 300.0),
])
def test_round_quot_random(lib, bmin, bmax, qmax):
    bad, first = _run(lib.tsdf_selfcheck_round_quot, 12345, 1 << 28, bmin, bmax, qmax)
    assert bad == 0, f"{bad} mismatches, first sample {first}"


def test_convert_all_floats(lib):
    bad, first = _run(lib.tsdf_selfcheck_convert, 0, 0xFFFFFFFF)
    assert bad == 0, f"{bad} mismatches, first bits {first:#x}"


@pytest.mark.parametrize("c", [639.0, 479.0, 79.0, 1279.0, 1919.0, 1079.0])
def test_quot_for_cmp(lib, c):
    for bmin, bmax in [(1e-3, 0.05), (0.05, 20.0)]:
        bad, first = _run(lib.tsdf_selfcheck_quot_cmp, 777, 1 << 27, bmin, bmax, c)
        assert bad == 0, f"c={c}: {bad} mismatches, first sample {first}"


# |a| in [2^-44, 2^44] both signs: the whole fast range plus 4 binades of fallback on either side
DIV_RANGES = [(0x29800000, 0x55800000), (0xA9800000, 0xD5800000)]


@pytest.mark.parametrize("b", [4.0, 1.0, 3.9999998, 40.5, 44.0, 7.3125, 0.0137, 2.3841858e-7, 1.5e-12])
def test_div_pair_sweep(lib, b):
    for lo, hi in DIV_RANGES:
        bad, first = _run(lib.tsdf_selfcheck_div_pair, b, lo, hi, 0, 0, 0.0, 0.0)
        assert bad == 0, f"b={b}: {bad} mismatches, first a bits {first:#x}"


@pytest.mark.parametrize("bmin,bmax", [(2.0**-22, 44.0), (2.0**-44, 2.0**44)])
def test_div_pair_random(lib, bmin, bmax):
    bad, first = _run(lib.tsdf_selfcheck_div_pair, 0.0, 0, 0, 4242, 1 << 28, bmin, bmax)
    assert bad == 0, f"{bad} mismatches, first sample {first}"


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_semantic_math_matches_oracle_on_every_input(lib, kind):
    """kind 0: sem_logf (pixels' ht / lt), 1: sem_expf, 2: the update's logf of p and 1 - p (inputs
    [0, 1] and NaN): every chunk's digest equals the oracle's."""
    import json
    dig = json.load(open(os.path.join(ROOT, "tests", "golden", "sem_math_digests.json")))[str(kind)]
    bad = []
    for lo, hi, d in dig:
        got = C.c_ulonglong()
        assert lib.tsdf_selfcheck_sem_digest(kind, lo, hi, C.byref(got)) == 0
        if got.value != int(d):
            bad.append((hex(lo), hex(hi)))
    assert not bad, f"{len(bad)} chunks differ from the oracle, first {bad[:4]}"
