"""The oracle's logf / expf of the semantic update (oracle/ora_math.c), CPU only.

The reference fuses ht / lt with CUDA's logf / expf (utils/tsdf/voxel_tsdf.cu:196-202), which no
other platform reproduces bit for bit; the oracle fixes both as explicit single-precision algorithms
and the engine restates them operation for operation (csrc/tsdf_device.h sem_logf / sem_expf;
tests/test_gpu_numerics.py compares the two over every input). Here: their accuracy against the
correctly rounded functions (a full scan of all 2^32 inputs gave max 0.862 / 0.988 ulp and 0.31 % /
0.40 % of results differing from the correctly rounded ones -- CUDA's own are specified to 1 / 2 ulp),
on a strided sample; the special values; and the committed digests the GPU check compares with
(tests/golden/sem_math_digests.json, make_golden.py --digests) against the current oracle code.
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

from _oracle import lib

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _acc(kind, step):
    out = (C.c_double * 3)()
    lib().ora_math_accuracy(kind, 0, 1 << 32, step, out)
    return list(out)


@pytest.mark.parametrize("kind,max_ulp,max_frac", [(0, 0.87, 0.005), (1, 0.99, 0.006)])
def test_accuracy_against_correct_rounding(kind, max_ulp, max_frac):
    n, bad, worst = _acc(kind, 1021)  # ~4.2 M inputs spread over every binade and sign
    assert n > 4e6
    assert worst < max_ulp, worst
    assert bad / n < max_frac, bad / n


def test_special_values():
    L = lib()
    inf = float("inf")
    assert L.ora_logf(1.0) == 0.0 and math.copysign(1, L.ora_logf(1.0)) > 0
    assert L.ora_logf(0.0) == -inf and L.ora_logf(-0.0) == -inf
    assert math.isnan(L.ora_logf(-1.0)) and math.isnan(L.ora_logf(float("nan")))
    assert L.ora_logf(inf) == inf
    tiny = float(np.float32(1.4e-45))  # the smallest subnormal
    assert L.ora_logf(tiny) == pytest.approx(math.log(tiny), rel=1e-6)
    assert L.ora_expf(0.0) == 1.0
    assert L.ora_expf(-inf) == 0.0 and L.ora_expf(inf) == inf and math.isnan(L.ora_expf(float("nan")))
    assert L.ora_expf(89.0) == inf and L.ora_expf(-104.0) == 0.0
    big = float(np.float32(88.72))
    assert L.ora_expf(big) == pytest.approx(math.exp(big), rel=1e-6)
    assert 0 < L.ora_expf(-100.0) < 1e-43  # subnormal result
    # the update's exact cases: p = 0.5 stays 0.5 when ht == lt (P == N)
    lnp = L.ora_logf(0.5)
    a = np.float32(np.float32(3.0) * np.float32(lnp)) / np.float32(3.5)
    P = np.float32(L.ora_expf(float(a)))
    assert P / (P + P) == np.float32(0.5)


def test_digest_fixture_pins_the_oracle():
    dig = json.load(open(os.path.join(GOLD, "sem_math_digests.json")))
    assert sorted(dig) == ["0", "1", "2"] and len(dig["0"]) == len(dig["1"]) == 256
    rng = np.random.default_rng(7)
    for kind in ("0", "1", "2"):
        rows = dig[kind]
        for r in rng.choice(len(rows), size=3, replace=False):
            lo, hi, d = rows[r]
            if hi - lo > (1 << 24):
                continue
            assert int(lib().ora_math_digest(int(kind), lo, hi)) == int(d), (kind, lo, hi)
