// tsdf_block.h -- wave / workgroup building blocks shared by the engine kernels (wave64).
#pragma once

#include "tsdf_device.h"

namespace tsdf {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
// wave-wide minimum as a wave-uniform value (every lane of the wave active): DPP row reductions --
// quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror -- then the four rows' minima read as
// scalars. No permute addresses: __shfl_xor's ds_bpermute lane addresses are loop-invariant VGPRs
// that the update loops keep live and spill to scratch.
__device__ __forceinline__ float wave_min_u(float v) {
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
  const int x = __float_as_int(v);
  return fminf(fminf(__int_as_float(__builtin_amdgcn_readlane(x, 0)), __int_as_float(__builtin_amdgcn_readlane(x, 16))),
               fminf(__int_as_float(__builtin_amdgcn_readlane(x, 32)), __int_as_float(__builtin_amdgcn_readlane(x, 48))));
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int n = __shfl_up(v, o, 64);
    if (l >= o) v += n;
  }
  return v;
}
// exclusive workgroup scan; every thread of the block must call it. scratch: blockDim/64 ints.
// NW: the workgroup's waves when known at compile time (the loop over the wave totals is then
// unrolled; the run-time bound gets a 16-wide vectorised loop that costs ~30 VGPRs)
template <int NW = 0>
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int* total) {
  const int w = threadIdx.x >> 6, nw = NW ? NW : blockDim.x >> 6;
  const int incl = wave_incl_scan(v);
  if (lane_id() == 63) scratch[w] = incl;
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < nw; ++i) {
    const int s = scratch[i];
    if (i < w) before += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return before + incl - v;
}
// workgroup barrier for LDS hand-offs only: global stores stay in flight (HIP's __syncthreads is a
// release of all memory -- s_waitcnt vmcnt(0) -- and would drain every outstanding pool store)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// ---------------------------------------------------------------------------------------------
// Single-workgroup ordered streaming of an unsorted list whose sort keys are unique integers in
// [0, range): a histogram over <= kMaxWin windows of width <= 1024 groups the list into batches
// of <= kBatch elements in key order (a window holds at most `width` distinct keys), each batch
// is gathered into LDS and bitonic-sorted. Used by both resolvers to replay the reference's
// sequential order without a global sort.
// ---------------------------------------------------------------------------------------------
constexpr int kBatch = 2048;
constexpr int kMaxWin = 8192;
constexpr int kClaimSlots = 4096;

constexpr int kRankSortMax = 512;  // single-batch sizes sorted by rank (<= blockDim, <= kMaxWin / 2)
constexpr int kLockSlots = 8192;   // buckets locked by one single-batch allocation launch (<= 2 per key)

struct ResolveLds {
  uint32_t hist[kMaxWin];             // window counts -> exclusive prefix
  unsigned long long batch[kBatch];   // (sort key << 32) | list index
  uint32_t ckey[kClaimSlots];         // claim table: bucket + 1 (0 = empty)
  uint32_t cval[kClaimSlots];         // claim table: smallest claiming rank
  int scan[16];
  int count;
  int first_dirty;
  int sfree;
  int nfresh;
  int base;
  int nalloc;
  uint32_t epoch;
  int bcnt[16];                       // new blocks per visible-list band this round (frame mode)
  int bbase[16];                      // their base in the band list
  // single-batch allocation resolves (n <= kBatch): the new keys, their key-set slots and the
  // free-stack top, loaded once by the prologue instead of re-read from HBM every round
  unsigned long long skey[kBatch];
  int32_t sslot[kBatch];
  int32_t heap_top[kBatch];           // heap_top[i] = heap[free - 1 - i]
  // single-batch allocation resolves: the bucket locks this launch has taken (bucket + 1; 0 =
  // empty), instead of the epoch-tagged lock words in HBM -- a lock only matters within its launch
  uint32_t lkey[kLockSlots];
};

__device__ __forceinline__ void lds_bitonic_sort(unsigned long long* a, int m) {
  int P = 1;
  while (P < m) P <<= 1;
  for (int i = m + (int)threadIdx.x; i < P; i += blockDim.x) a[i] = ~0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// VoxelHashTable's bucket lock within one launch: true if this call took it (it was free)
__device__ __forceinline__ bool lock_take(ResolveLds& L, uint32_t bucket) {
  uint32_t h = mix32(bucket ^ 0x9E3779B9u) & (kLockSlots - 1);
  const uint32_t k = bucket + 1u;
  for (int p = 0; p < kLockSlots; ++p) {
    const uint32_t prev = atomicCAS(&L.lkey[h], 0u, k);
    if (prev == 0u) return true;
    if (prev == k) return false;
    h = (h + 1) & (kLockSlots - 1);
  }
  return false;
}
// claim table: each key claims buckets; the smallest rank per bucket wins
__device__ __forceinline__ void claims_clear(ResolveLds& L) {
  for (int i = threadIdx.x; i < kClaimSlots; i += blockDim.x) {
    L.ckey[i] = 0u;
    L.cval[i] = 0xFFFFFFFFu;
  }
}
__device__ __forceinline__ void claim(ResolveLds& L, uint32_t bucket, uint32_t rank) {
  uint32_t h = mix32(bucket) & (kClaimSlots - 1);
  const uint32_t k = bucket + 1u;
  for (int p = 0; p < kClaimSlots; ++p) {
    const uint32_t prev = atomicCAS(&L.ckey[h], 0u, k);
    if (prev == 0u || prev == k) {
      atomicMin(&L.cval[h], rank);
      return;
    }
    h = (h + 1) & (kClaimSlots - 1);
  }
}
__device__ __forceinline__ uint32_t claim_winner(const ResolveLds& L, uint32_t bucket) {
  uint32_t h = mix32(bucket) & (kClaimSlots - 1);
  const uint32_t k = bucket + 1u;
  for (int p = 0; p < kClaimSlots; ++p) {
    if (L.ckey[h] == k) return L.cval[h];
    h = (h + 1) & (kClaimSlots - 1);
  }
  return 0xFFFFFFFFu;
}

// Prepare ordered streaming of `n` elements with keys(i) in [0, range); returns the window width.
// After it, L.hist[w] holds the exclusive prefix count of window w.
template <typename KeyFn>
__device__ int stream_prepare(ResolveLds& L, int n, uint32_t range, KeyFn keyf) {
  uint32_t width = (range + kMaxWin - 1) / kMaxWin;
  if (width < 1) width = 1;
  const int nwin = (int)((range + width - 1) / width);
  if (n <= kBatch) return (int)width;  // single batch: no histogram needed
  for (int i = threadIdx.x; i < nwin; i += blockDim.x) L.hist[i] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&L.hist[keyf(i) / width], 1u);
  __syncthreads();
  // exclusive scan of hist[0..nwin) (kMaxWin / blockDim windows per thread)
  const int per = (nwin + blockDim.x - 1) / blockDim.x;
  const int w0 = threadIdx.x * per;
  int local = 0;
  for (int k = 0; k < per; ++k)
    if (w0 + k < nwin) local += (int)L.hist[w0 + k];
  int tot;
  int run = block_excl_scan(local, L.scan, &tot);
  for (int k = 0; k < per; ++k)
    if (w0 + k < nwin) {
      const int c = (int)L.hist[w0 + k];
      L.hist[w0 + k] = (uint32_t)run;
      run += c;
    }
  __syncthreads();
  return (int)width;
}

__device__ __forceinline__ void batch_sort(ResolveLds& L, int m, bool single);
// Gather batch `j` (elements whose window prefix >> 10 == j, or all when n <= kBatch) into
// L.batch sorted ascending by key; returns its size.
template <typename KeyFn>
__device__ int stream_batch(ResolveLds& L, int n, int width, int j, KeyFn keyf) {
  if (threadIdx.x == 0) L.count = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t k = keyf(i);
    if (n <= kBatch || (int)(L.hist[k / (uint32_t)width] >> 10) == j) {
      const int pos = atomicAdd(&L.count, 1);
      if (pos < kBatch) L.batch[pos] = ((unsigned long long)k << 32) | (uint32_t)i;
    }
  }
  __syncthreads();
  const int m = L.count < kBatch ? L.count : kBatch;  // bounded by construction (width <= 1024)
  batch_sort(L, m, n <= kBatch);
  return m;
}

// Sort L.batch[0..m) ascending (unique keys); single: the list is one batch, so L.hist is free
// as the rank sort's scratch.
__device__ __forceinline__ void batch_sort(ResolveLds& L, int m, bool single) {
  if (single && m <= kRankSortMax) {
    // single batch (hist unused): rank sort -- every element counts the smaller ones with
    // broadcast LDS reads, one barrier instead of bitonic's log^2 stages (keys are unique)
    unsigned long long* tmp = reinterpret_cast<unsigned long long*>(L.hist);
    unsigned long long x = 0ull;
    int rank = 0;
    if ((int)threadIdx.x < m) {
      x = L.batch[threadIdx.x];
      for (int j = 0; j < m; ++j) rank += L.batch[j] < x;
      tmp[rank] = x;
    }
    __syncthreads();
    if ((int)threadIdx.x < m) L.batch[threadIdx.x] = tmp[threadIdx.x];
    __syncthreads();
  } else {
    lds_bitonic_sort(L.batch, m);
  }
}

}  // namespace tsdf

// ---------------------------------------------------------------------------------------------
// Diagnostic build only (make DIAG=1): per-workgroup s_memrealtime stamps (100 MHz) at phase
// boundaries, written by thread 0 to D.dbg[((kernel * kDiagMaxWg) + wg) * kDiagStamps + k].
// ---------------------------------------------------------------------------------------------
#ifdef TSDF_DIAG_STAMPS
#define TSDF_STAMP(D, kern, k)                                                                 \
  do {                                                                                         \
    if (threadIdx.x == 0 && (D).dbg) {                                                         \
      const unsigned wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                \
      if (wg_ < (unsigned)::tsdf::kDiagMaxWg)                                                  \
        (D).dbg[((kern) * ::tsdf::kDiagMaxWg + wg_) * ::tsdf::kDiagStamps + (k)] =             \
            __builtin_amdgcn_s_memrealtime();                                                  \
    }                                                                                          \
  } while (0)
// explicit workgroup slot (kernel 5)
#define TSDF_STAMP_WG(D, kern, wg, k)                                                                    \
  do {                                                                                                   \
    if (threadIdx.x == 0 && (D).dbg && (unsigned)(wg) < (unsigned)::tsdf::kDiagMaxWg)                    \
      (D).dbg[((kern) * ::tsdf::kDiagMaxWg + (unsigned)(wg)) * ::tsdf::kDiagStamps + (k)] =              \
          __builtin_amdgcn_s_memrealtime();                                                              \
  } while (0)
#else
#define TSDF_STAMP(D, kern, k) \
  do {                         \
  } while (0)
#define TSDF_STAMP_WG(D, kern, wg, k) \
  do {                                \
  } while (0)
#endif
