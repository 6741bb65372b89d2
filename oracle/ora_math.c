/*
 * ora_math.c -- the oracle's logf / expf for the semantic probability update (TEST INFRASTRUCTURE).
 *
 * tsdf_integrate_kernel fuses the high / low-touch maps with CUDA's logf / expf
 * (utils/tsdf/voxel_tsdf.cu:196-202):
 *   p' = P / (P + N),  P = expf((w_old logf(p) + w_new logf(ht)) / wc),
 *                      N = expf((w_old logf(1 - p) + w_new logf(lt)) / wc).
 * That chain is ill-conditioned once p comes within ~1e-5 of 1: a float p there keeps only a few
 * bits of 1 - p, so one ulp of difference in p (or in a logf / expf result) moves a later p by up to
 * ~1e-2. CUDA's logf / expf (<= 1 / 2 ulp, NVIDIA libdevice) are not reproducible off NVIDIA
 * hardware, and glibc's are not reproducible on a GPU, so no implementation can match "the"
 * reference bit for bit on such inputs. The oracle therefore fixes the two functions as the explicit
 * float algorithms below -- IEEE single-precision operations only (frexpf, rintf, ldexpf, fmaf and
 * + - * with one rounding each), so the engine's HIP restatement (csrc/tsdf_device.h sem_logf /
 * sem_expf, written separately) returns the same bits for every input: tests/test_gpu_numerics.py
 * compares the two over all 2^32 inputs of each. Accuracy against the correctly rounded functions is
 * measured by ora_math_accuracy (tests/test_oracle_math.py; the full scan is in DESIGN.md 2).
 *
 *   logf(x): x = m 2^e, m in [sqrt(1/2), sqrt(2)), f = m - 1 (exact);
 *            log(1 + f) = f - f^2 / 2 + f^3 Q(f), Q a degree-8 fit of (log1p(f) - f + f^2/2) / f^3;
 *            result e ln2_hi + ((e ln2_lo + (f^3 Q - f^2/2)) + f)  (e ln2_hi exact in float).
 *   expf(x): n = rint(x / ln 2), r = (x - n ln2_hi) - n ln2_lo, e^r = 1 + (r + r^2 E(r)), E a
 *            degree-5 fit of (expm1(r) - r) / r^2, result ldexpf(e^r, n); x > 89 -> inf, x < -104 -> 0.
 * Compile with -ffp-contract=off (no fused operation but the explicit fmaf).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "tsdf_oracle.h"

static const float kQ[9] = {0x1.555554p-2f,  -0x1.fffffcp-3f, 0x1.999d5ap-3f,  -0x1.555b4ap-3f, 0x1.23d21ap-3f,
                            -0x1.fcf4c6p-4f, 0x1.dea282p-4f,  -0x1.d635bcp-4f, 0x1.1d8ea4p-4f};
static const float kE[6] = {0x1p-1f, 0x1.555556p-3f, 0x1.5554eap-5f, 0x1.1110e0p-7f, 0x1.6d4316p-10f,
                            0x1.a124e4p-13f};
#define LN2_HI 0x1.62e4p-1f      /* 16 significant bits: e * LN2_HI is exact for |e| < 2^8 */
#define LN2_LO 0x1.7f7d1cp-20f   /* ln 2 - LN2_HI, rounded */
#define INV_LN2 0x1.715476p+0f
#define SQRT_HALF 0x1.6a09e6p-1f

float ora_logf(float x) {
  if (!(x > 0.0f)) return x == 0.0f ? -INFINITY : NAN; /* negative, -0 -> -inf, NaN */
  if (x == INFINITY) return x;
  int e;
  float m = frexpf(x, &e); /* [1/2, 1), exact for subnormal x too */
  if (m < SQRT_HALF) {
    m = m + m;
    e = e - 1;
  }
  const float f = m - 1.0f; /* exact */
  float q = kQ[8];
  for (int i = 7; i >= 0; --i) q = fmaf(q, f, kQ[i]);
  const float f2 = f * f;
  const float hf2 = 0.5f * f2;
  const float t = fmaf(f2 * f, q, -hf2);
  const float dk = (float)e;
  return fmaf(dk, LN2_HI, fmaf(dk, LN2_LO, t) + f);
}

float ora_expf(float x) {
  if (x != x) return x + x;
  if (x > 89.0f) return INFINITY;
  if (x < -104.0f) return 0.0f;
  const float n = rintf(x * INV_LN2);
  float r = fmaf(-n, LN2_HI, x);
  r = fmaf(-n, LN2_LO, r);
  float p = kE[5];
  for (int i = 4; i >= 0; --i) p = fmaf(p, r, kE[i]);
  const float s = fmaf(r * r, p, r);
  return ldexpf(1.0f + s, (int)n);
}

/* ---- test support ---- */
static uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static float bitsf(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

/* Order-independent digest of fn(x) over the inputs x = bits lo .. hi - 1 (NaN results as one
 * pattern): sum of mix(i, bits) mod 2^64, the same sum the GPU self-check forms. kind 0 and 2: logf
 * (2 is the GPU's form for the update's p and 1 - p, compared on [0, 1] and NaN), 1: expf. */
uint64_t ora_math_digest(int kind, uint64_t lo, uint64_t hi) {
  uint64_t h = 0;
  for (uint64_t i = lo; i < hi; ++i) {
    const float x = bitsf((uint32_t)i);
    const float y = kind == 1 ? ora_expf(x) : ora_logf(x);
    uint32_t b = fbits(y);
    if (y != y) b = 0x7fc00000u;
    h += ((uint64_t)b ^ (i * 0x9E3779B97F4A7C15ull)) * 0xBF58476D1CE4E5B9ull;
  }
  return h;
}

/* Accuracy over inputs lo .. hi - 1 (stride `step`) against the correctly rounded value (the double
 * log / exp, whose error is far below a float ulp, rounded to float): out[0] = inputs compared,
 * out[1] = results that differ, out[2] = the largest difference in ulps (of the float result's
 * binade), specials (NaN, inf, 0 results) compared for equality. */
void ora_math_accuracy(int kind, uint64_t lo, uint64_t hi, uint64_t step, double* out) {
  double n = 0, bad = 0, worst = 0;
  for (uint64_t i = lo; i < hi; i += step) {
    const float x = bitsf((uint32_t)i);
    const float y = kind == 0 ? ora_logf(x) : ora_expf(x);
    const double ref = kind == 0 ? log((double)x) : exp((double)x);
    const float yr = (float)ref;
    n += 1;
    if (y != y || yr != yr) {
      if ((y != y) != (yr != yr)) bad += 1, worst = INFINITY;
      continue;
    }
    if (y == yr) continue;
    bad += 1;
    if (isinf(y) || isinf(yr)) {
      worst = INFINITY;
      continue;
    }
    int e;
    (void)frexp(ref, &e);
    double ulp = ldexp(1.0, e - 24);
    if (ulp < 0x1p-149) ulp = 0x1p-149;
    const double d = fabs((double)y - ref) / ulp;
    if (d > worst) worst = d;
  }
  out[0] = n;
  out[1] = bad;
  out[2] = worst;
}
