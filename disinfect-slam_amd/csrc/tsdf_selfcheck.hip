// tsdf_selfcheck.hip -- test-only library (libtsdf_selfcheck.so): checks the engine's fast exact
// quotient helpers (tsdf_device.h: round_quot_i/_u8/_pos2, div_pair, quot_const, quot_for_cmp,
// f2i / f2u8 / round_s16) bit-for-bit against the
// correctly rounded IEEE divide and the saturating conversions, on the GPU, over exhaustive and
// adversarial input sets; and digests the semantic update's sem_logf / sem_expf over every input for
// comparison with the oracle's (ora_math_digest). Not part of the product library; tests/test_gpu_numerics.py drives it.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "tsdf_device.h"

using namespace tsdf;

namespace {

__device__ __forceinline__ uint32_t pcg(uint32_t v) {
  const uint32_t s = v * 747796405u + 2891336453u;
  const uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
  return (w >> 22u) ^ w;
}

__device__ __forceinline__ bool same_bits(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

// every a with bits in [lo, hi) against divisor b (rb = RN(1/b) computed on the host)
__global__ void k_quot_const(float b, float rb, uint32_t lo, uint32_t hi,
                             unsigned long long* bad, uint32_t* first) {
  const uint64_t n = (uint64_t)hi - lo;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t bits = lo + (uint32_t)i;
    const float a = __uint_as_float(bits);
    const v2f a2 = v2(a, __uint_as_float(bits ^ 0x80000000u));  // pair: a and -a
    const v2f q2 = quot_const2(a2, b, rb, true, true);
    if (!same_bits(quot_const(a, b, rb), a / b) || !same_bits(q2.x, a / b) ||
        !same_bits(q2.y, a2.y / b)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, bits);
    }
  }
}

// random (a, b) with b in [bmin, bmax) and a = (k + 1/2 + tiny) * b: quotients at and around the
// rounding boundaries of roundf, plus uniformly random quotients in [-qmax, qmax]
__global__ void k_round_quot(uint32_t seed, uint64_t n, float bmin, float bmax, float qmax,
                             unsigned long long* bad, uint32_t* first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h0 = pcg((uint32_t)i ^ seed), h1 = pcg(h0 + 0x9e3779b9u), h2 = pcg(h1 ^ 0x85ebca6bu);
    const float b = bmin + (bmax - bmin) * ((h0 >> 8) * 0x1p-24f);
    float a;
    if (h2 & 1u) {
      const float k = floorf((h1 >> 8) * 0x1p-24f * qmax);
      const float half = (k + 0.5f) * b;
      // perturb by up to +-8 ulps around the exact boundary product
      const int32_t d = (int32_t)((h2 >> 1) & 15u) - 8;
      a = __uint_as_float(__float_as_uint(half) + d);
      if (h2 & 0x100u) a = -a;
    } else {
      a = ((h1 >> 8) * 0x1p-23f - 1.0f) * qmax * b;
    }
    const float rb = __builtin_amdgcn_rcpf(b);
    const int32_t fast_i = round_quot_i(a, b, rb), ref_i = f2i(roundf(a / b));
    const uint32_t fast_u = round_quot_u8(a, b, rb), ref_u = f2u8(roundf(a / b));
    int32_t p0, p1;  // the packed-pair form on (a, b) and (-a, b)
    round_quot_i2(v2(a, -a), v2(b, b), v2(rb, rb), true, true, p0, p1);
    int32_t n0, n1;  // the non-negative form on (|a|, b) twice
    const float fa = fabsf(a);
    round_quot_pos2(v2(fa, fa), v2(b, b), v2(rb, rb), true, true, n0, n1);
    const int32_t ref_pos = f2i(roundf(fa / b));
    if (fast_i != ref_i || fast_u != ref_u || p0 != ref_i || p1 != f2i(roundf(-a / b)) ||
        n0 != ref_pos || n1 != ref_pos) {
      atomicAdd(bad, 1ull);
      atomicMin(first, (uint32_t)i);
    }
  }
}

// div_pair(a, b, v_rcp(b)) == a / b: every a with bits in [lo, hi) (both signs) against a fixed
// divisor b, or (lo == hi) n random pairs with b log-uniform in [bmin, bmax) and a log-uniform in
// [2^-44, 2^44] of random sign (covers the fast range and both edges of it)
__global__ void k_div_pair(float b, uint32_t lo, uint32_t hi, uint32_t seed, uint64_t n, float bmin,
                           float bmax, unsigned long long* bad, uint32_t* first) {
  const bool sweep = hi > lo;
  const uint64_t cnt = sweep ? (uint64_t)hi - lo : n;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cnt;
       i += (uint64_t)gridDim.x * blockDim.x) {
    float a, bb = b;
    if (sweep) {
      a = __uint_as_float(lo + (uint32_t)i);
    } else {
      const uint32_t h0 = pcg((uint32_t)i ^ seed), h1 = pcg(h0 + 0x9e3779b9u);
      bb = bmin * exp2f(log2f(bmax / bmin) * ((h0 >> 8) * 0x1p-24f));
      a = exp2f(-44.0f + 88.0f * ((h1 >> 8) * 0x1p-24f));
      if (h1 & 1u) a = -a;
    }
    const float y = __builtin_amdgcn_rcpf(bb);
    const v2f q = div_pair(v2(a, -a), v2(bb, bb), v2(y, y), true, true);
    if (!same_bits(q.x, a / bb) || !same_bits(q.y, -a / bb)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, sweep ? lo + (uint32_t)i : (uint32_t)i);
    }
  }
}

// voxel_visible's comparisons: RN(a/b) >= 0 and <= c, with a / b near c, near 0 and uniform
__global__ void k_quot_cmp(uint32_t seed, uint64_t n, float bmin, float bmax, float c,
                           unsigned long long* bad, uint32_t* first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h0 = pcg((uint32_t)i ^ seed), h1 = pcg(h0 + 0x9e3779b9u), h2 = pcg(h1 ^ 0x85ebca6bu);
    float b = bmin + (bmax - bmin) * ((h0 >> 8) * 0x1p-24f);
    if (h2 & 0x200u) b = -b;
    float a;
    const uint32_t mode = h2 & 3u;
    if (mode == 0) {
      a = __uint_as_float(__float_as_uint(c * b) + (int32_t)((h2 >> 2) & 15u) - 8);
    } else if (mode == 1) {
      a = ((h1 >> 8) * 0x1p-24f - 0.5f) * 1e-30f * b;
      if (h2 & 0x400u) a = 0.0f;
      if (h2 & 0x800u) a = -a;
    } else {
      a = ((h1 >> 8) * 0x1p-23f - 1.0f) * 2.0f * c * b;
    }
    const float rb = __builtin_amdgcn_rcpf(b);
    const float qf = quot_for_cmp(a, b, rb, c), qe = a / b;
    if ((qf >= 0) != (qe >= 0) || (qf <= c) != (qe <= c)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, (uint32_t)i);
    }
  }
}

// conversions on every float bit pattern in [lo, hi) against the reference semantics spelled out
__global__ void k_convert(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
  const uint64_t n = (uint64_t)hi - lo;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t bits = lo + (uint32_t)i;
    const float f = __uint_as_float(bits);
    const float t = truncf(f);
    const int32_t ei = f != f ? 0 : t >= 2147483648.0f ? 2147483647
                       : t <= -2147483648.0f ? (-2147483647 - 1) : (int32_t)t;
    const int32_t es = f != f ? 0 : t >= 32767.0f ? 32767 : t <= -32768.0f ? -32768 : (int32_t)t;
    const uint32_t eu = !(t > 0.0f) ? 0u : t >= 255.0f ? 255u : (uint32_t)t;
    if (f2i(f) != ei || f2s(f) != es || f2u8(f) != eu || round_s16(f) != f2s(roundf(f))) {
      atomicAdd(bad, 1ull);
      atomicMin(first, bits);
    }
  }
}

// order-independent digest of the semantic-update functions over the input bit patterns [lo, hi)
// (NaN results as one pattern): the sum ora_math_digest forms. kind 0: sem_logf2 (any float),
// 1: sem_expf2, 2: sem_log_unit2 (the update's p and 1 - p: meant for [0, 1] and NaN). Pairs are
// two consecutive inputs, so both lanes of the packed forms are exercised.
__device__ __forceinline__ unsigned long long sem_mix(uint64_t i, float y) {
  const uint32_t b = y != y ? 0x7fc00000u : __float_as_uint(y);
  return ((unsigned long long)b ^ (i * 0x9E3779B97F4A7C15ull)) * 0xBF58476D1CE4E5B9ull;
}
__global__ void k_sem_digest(int kind, uint64_t lo, uint64_t hi, unsigned long long* out) {
  unsigned long long h = 0;
  for (uint64_t i = lo + 2 * (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x); i < hi;
       i += 2 * (uint64_t)gridDim.x * blockDim.x) {
    const bool two = i + 1 < hi;
    const v2f x = v2(__uint_as_float((uint32_t)i), __uint_as_float((uint32_t)(two ? i + 1 : i)));
    const v2f y = kind == 0 ? sem_logf2(x) : kind == 1 ? sem_expf2(x) : sem_log_unit2(x);
    h += sem_mix(i, y.x);
    if (two) h += sem_mix(i + 1, y.y);
  }
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, h);
}

struct Out {
  unsigned long long bad;
  uint32_t first;
};

int finish(Out* d, unsigned long long* bad, uint32_t* first) {
  Out h{};
  hipError_t err = hipGetLastError();
  if (err == hipSuccess) err = hipDeviceSynchronize();
  if (err != hipSuccess) {
    std::fprintf(stderr, "tsdf_selfcheck: %s\n", hipGetErrorString(err));
    return -2;
  }
  if (hipMemcpy(&h, d, sizeof(Out), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  (void)hipFree(d);
  *bad = h.bad;
  *first = h.first;
  return 0;
}

Out* start() {
  Out* d = nullptr;
  hipError_t err = hipMalloc(&d, sizeof(Out));
  Out h{0ull, 0xFFFFFFFFu};
  if (err == hipSuccess) err = hipMemcpy(d, &h, sizeof(Out), hipMemcpyHostToDevice);
  if (err != hipSuccess) {
    std::fprintf(stderr, "tsdf_selfcheck: %s\n", hipGetErrorString(err));
    return nullptr;
  }
  return d;
}

}  // namespace

extern "C" {

// quot_const(a, b, RN(1/b)) == a / b for every a whose bit pattern lies in [lo, hi)
int tsdf_selfcheck_quot_const(float b, uint32_t lo, uint32_t hi, unsigned long long* bad,
                              uint32_t* first) {
  Out* d = start();
  if (!d) return -1;
  const float rb = 1.0f / b;
  hipLaunchKernelGGL(k_quot_const, dim3(8192), dim3(256), 0, 0, b, rb, lo, hi, &d->bad, &d->first);
  return finish(d, bad, first);
}

int tsdf_selfcheck_round_quot(uint32_t seed, uint64_t n, float bmin, float bmax, float qmax,
                              unsigned long long* bad, uint32_t* first) {
  Out* d = start();
  if (!d) return -1;
  hipLaunchKernelGGL(k_round_quot, dim3(8192), dim3(256), 0, 0, seed, n, bmin, bmax, qmax, &d->bad,
                     &d->first);
  return finish(d, bad, first);
}

int tsdf_selfcheck_quot_cmp(uint32_t seed, uint64_t n, float bmin, float bmax, float c,
                            unsigned long long* bad, uint32_t* first) {
  Out* d = start();
  if (!d) return -1;
  hipLaunchKernelGGL(k_quot_cmp, dim3(8192), dim3(256), 0, 0, seed, n, bmin, bmax, c, &d->bad,
                     &d->first);
  return finish(d, bad, first);
}

// div_pair == IEEE a / b: sweep (lo < hi, fixed b) or random (lo == hi, n pairs, b in [bmin, bmax))
int tsdf_selfcheck_div_pair(float b, uint32_t lo, uint32_t hi, uint32_t seed, uint64_t n, float bmin,
                            float bmax, unsigned long long* bad, uint32_t* first) {
  Out* d = start();
  if (!d) return -1;
  hipLaunchKernelGGL(k_div_pair, dim3(8192), dim3(256), 0, 0, b, lo, hi, seed, n, bmin, bmax,
                     &d->bad, &d->first);
  return finish(d, bad, first);
}

int tsdf_selfcheck_convert(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
  Out* d = start();
  if (!d) return -1;
  hipLaunchKernelGGL(k_convert, dim3(8192), dim3(256), 0, 0, lo, hi, &d->bad, &d->first);
  return finish(d, bad, first);
}

// digest of the semantic-update function `kind` over the input bit patterns [lo, hi) (k_sem_digest)
int tsdf_selfcheck_sem_digest(int kind, uint64_t lo, uint64_t hi, unsigned long long* digest) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(*d)) != hipSuccess || hipMemset(d, 0, sizeof(*d)) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_sem_digest, dim3(4096), dim3(256), 0, 0, kind, lo, hi, d);
  hipError_t err = hipGetLastError();
  if (err == hipSuccess) err = hipMemcpy(digest, d, sizeof(*d), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (err != hipSuccess) {
    std::fprintf(stderr, "tsdf_selfcheck: %s\n", hipGetErrorString(err));
    return -2;
  }
  return 0;
}

}  // extern "C"
