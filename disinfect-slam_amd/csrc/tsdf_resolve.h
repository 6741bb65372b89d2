// tsdf_resolve.h -- the ordered allocation and carving resolvers as ONE-WORKGROUP device functions
// (256 threads, <= 25 KiB of LDS).
//
// They run in two places:
//  * fused into the frame kernels: the workgroup that arrives last at the end of k_ingest_dda runs
//    the allocation resolver, the one that arrives last at the end of k_integrate runs the carving
//    resolver -- so one frame is two launches (two kernel boundaries) instead of four;
//  * as their own single-workgroup kernels (k_resolve_alloc / k_resolve_delete) where an exchange
//    sits between the phases (sharded frames) and for the hash-level test path.
//
// Semantics (the canonical linearisation of the reference's racy launches):
//  * allocation: VoxelHashTable::Allocate (voxel_hash.cu:58-120) of every new key in candidate
//    order, <= 1 structural change per bucket per launch (losers dropped), AquireBlock pops
//    heap[free - 1] in commit order (voxel_mem.cu:37-52);
//  * carving: VoxelHashTable::Delete (voxel_hash.cu:122-171) of every candidate in hash-entry order;
//    slot-0 deletes are lock free, list-head / element deletes lock the bucket.
// Keys are processed in batches of <= kRB in order (a histogram threshold search over the global
// scratch picks each batch when a launch has more); within a batch, rounds of 256 keys are
// evaluated speculatively against the table, every key claims the buckets it would lock in an LDS
// claim table (smallest rank wins), and the longest prefix of keys that won all their claims
// commits (the first key always does).
//
// Cross-workgroup data of a fused launch (the new-key list, carve candidates) is published with
// agent-scope atomic stores (global_store ... sc1) and read back with agent-scope atomic loads
// (global_load ... sc1): the workgroup that arrives last has no kernel boundary between it and the
// producers.
#pragma once

#include "tsdf_block.h"
#include "tsdf_kernels.h"

namespace tsdf {

constexpr int kRT = 256;        // resolver workgroup size (= the ingest / integrate workgroup)
constexpr int kRB = 2 * kRT;    // keys / candidates per ordered batch
constexpr int kRHist = 1024;    // threshold-search bins (launches with more than kRB inputs)
constexpr int kRClaim = 1024;   // claim slots, packed (bucket + 1) << 9 | rank (<= 512 per round)
constexpr int kRLockA = 2048;   // LDS lock set of an allocation launch with <= kRLockKeysA keys
constexpr int kRLockKeysA = 768;
constexpr int kRLockD = 1024;   // LDS lock set of a carving launch with <= kRLockKeysD candidates
constexpr int kRLockKeysD = 768;
static_assert(kRT == 256, "resolver geometry");

// cross-workgroup publish / consume inside one launch (agent scope, relaxed)
template <class T>
__device__ __forceinline__ T ld_co(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_co(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a 16-B record written through / read at agent scope (two 8-byte halves)
template <class R>
__device__ __forceinline__ void st_rec_co(R* dst, const R& v) {
  static_assert(sizeof(R) == 16, "16-B record");
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(&v);
  unsigned long long* d = reinterpret_cast<unsigned long long*>(dst);
  st_co(&d[0], q[0]);
  st_co(&d[1], q[1]);
}
template <class R>
__device__ __forceinline__ R ld_rec_co(const R* src) {
  static_assert(sizeof(R) == 16, "16-B record");
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(src);
  unsigned long long a[2] = {ld_co(&q[0]), ld_co(&q[1])};
  R v;
  __builtin_memcpy(&v, a, 16);
  return v;
}

// Table stores of the carving resolver, written through at agent scope (32-bit sc1 stores; the
// 16-bit offset by read-modify-write of its dword -- nothing else writes the table meanwhile): a
// pipelined frame's chained sweep and probes on other XCDs read the carved table right after the
// carving is published, with no L2 write-back in between (tsdf_fuse.hip k_frame).
__device__ __forceinline__ void store_ent_co(int4* table, uint32_t e, int16_t x, int16_t y, int16_t z, int16_t off,
                                             int32_t idx) {
  uint32_t* p = reinterpret_cast<uint32_t*>(&table[e]);
  st_co(&p[0], (uint32_t)(uint16_t)x | ((uint32_t)(uint16_t)y << 16));
  st_co(&p[1], (uint32_t)(uint16_t)z | ((uint32_t)(uint16_t)off << 16));
  st_co(&p[2], (uint32_t)idx);
}
__device__ __forceinline__ void store_off_co(int4* table, uint32_t e, int16_t off) {
  uint32_t* p = reinterpret_cast<uint32_t*>(&table[e]) + 1;
  st_co(p, (ld_co(p) & 0xFFFFu) | ((uint32_t)(uint16_t)off << 16));
}
__device__ __forceinline__ void store_off_idx_co(int4* table, uint32_t e, int16_t off, int32_t idx) {
  store_off_co(table, e, off);
  st_co(reinterpret_cast<uint32_t*>(&table[e]) + 2, (uint32_t)idx);
}

// Entries the carving changed, by occupancy word (bit (e >> 6) & 63 of D.swdirty[e >> 12]): a
// pipelined frame's chained sweep tests visibility before the carving is published and re-tests
// only the words marked here (tsdf_ingest.h vis_sweep_chained). Conservative: a mark left by a
// carving no chained sweep followed only costs a re-test.
__device__ __forceinline__ void mark_swept_dirty(const EngineDev& D, uint32_t e) {
  atomicOr(&D.swdirty[e >> 12], 1ull << ((e >> 6) & 63));
}

// ---------------------------------------------------------------------------------------------
// per-frame new-key set: open addressing on 64-bit packed keys, min candidate order per key
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void keyset_insert(unsigned long long* keys, uint32_t* orders, NkEnt* list,
                              int32_t* count, uint32_t* status, uint64_t key, uint32_t order) {
  uint32_t h = (uint32_t)mix64(key) & (kNewKeyCap - 1);
  for (int p = 0; p < 256; ++p) {
    // the CAS itself reads the slot (measured equal to a plain read first)
    const unsigned long long cur = atomicCAS(&keys[h], 0ull, (unsigned long long)key);
    if (cur == 0ull) {
      const int s = atomicAdd(count, 1);
      // the list entry carries the key (the resolver's prologue needs no second load for it),
      // published for the workgroup that resolves at the end of this launch
      st_co(&list[s].key, (unsigned long long)key);
      st_co(&list[s].slot, (unsigned long long)h);
      atomicMin(&orders[h], order);
      return;
    }
    if (cur == key) {
      atomicMin(&orders[h], order);
      return;
    }
    h = (h + 1) & (kNewKeyCap - 1);
  }
  atomicOr(status, 2u);  // TSDF_STATUS_NEWKEY_OVERFLOW
}
__device__ __forceinline__ void nk_insert(const EngineDev& D, uint64_t key, uint32_t order) {
  keyset_insert(D.nk_key, D.nk_order, D.nk_list, &D.ctr->nk_count, &D.ctr->status, key, order);
}

// ---------------------------------------------------------------------------------------------
// Last-arriver detection: every workgroup of the launch arrives once at its end; the function
// returns true (in all threads) in the workgroup that arrives last. Arrivals go to 8 counters by
// blockIdx % 8 (one per XCD under round-robin placement: no single hot word), each counter's last
// arriver to a top counter. The high 24 bits of a counter count arrivals, the low 40 accumulate
// `payload` (k_integrate: its updated-voxel count). Each thread drains its own memory operations
// first, so everything it published (st_co) is complete before its workgroup arrives.
// Memory-model note: the ordering rests on the raw s_waitcnt vmcnt(0) + barrier before
// the relaxed arrival, with the publications as agent-scope (sc1) stores, which gfx950 counts in
// vmcnt -- not on an agent-scope release, whose gfx950 lowering (buffer_wbl2 sc1: a write-back of
// the L2) in every workgroup would cost the frame. tests/test_isa.py pins that codegen in the built
// library (every arrival after a drained barrier, no store sunk past it; sc1 publications).
// ---------------------------------------------------------------------------------------------
constexpr int kArrLine = 16;  // u64 per 128-B line
// drain: this wave published data (wave-uniform); other waves' outstanding stores stay in flight
// nwg: the arriving workgroups, blocks [0, nwg) of the launch (0: the whole grid)
// idx: the arriving workgroup's index among the nwg (default blockIdx.x)
__device__ __forceinline__ bool arrive_last(unsigned long long* words, unsigned long long payload,
                                            int* s_flag, bool drain = true, uint32_t nwg = 0u,
                                            uint32_t idx = 0xFFFFFFFFu) {
  if (drain) __builtin_amdgcn_s_waitcnt(0);
  lds_barrier();
  if (threadIdx.x == 0) {
    constexpr uint32_t NG = (uint32_t)kArrGroups;
    const uint32_t nw = nwg ? nwg : gridDim.x;
    const uint32_t g = (idx == 0xFFFFFFFFu ? blockIdx.x : idx) % NG, ngrp = nw < NG ? nw : NG;
    const uint32_t expect = (nw - g + NG - 1u) / NG;
    const unsigned long long old = __hip_atomic_fetch_add(&words[g * kArrLine], (1ull << 40) | payload,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = 0;
    if ((uint32_t)(old >> 40) + 1u == expect) {
      const unsigned long long top = __hip_atomic_fetch_add(&words[NG * kArrLine], 1ull, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
      last = (uint32_t)top + 1u == ngrp;
    }
    *s_flag = last;
  }
  lds_barrier();
  return *s_flag != 0;
}
// the last arriver, thread 0: the counters zeroed for the next launch (stores only)
__device__ __forceinline__ void arrive_reset(unsigned long long* words) {
  for (int g = 0; g <= kArrGroups; ++g) st_co(&words[g * kArrLine], 0ull);
}
// the last arriver, thread 0: the sum of the payloads; the counters are zeroed for the next launch
__device__ __forceinline__ unsigned long long arrive_collect(unsigned long long* words) {
  unsigned long long sum = 0ull;
  for (int g = 0; g < kArrGroups; ++g) sum += ld_co(&words[g * kArrLine]) & ((1ull << 40) - 1ull);
  for (int g = 0; g <= kArrGroups; ++g) st_co(&words[g * kArrLine], 0ull);
  return sum;
}

// ---------------------------------------------------------------------------------------------
// LDS helpers
// ---------------------------------------------------------------------------------------------
// claim table: slot = (bucket + 1) << 9 | rank; the smallest rank per bucket wins
template <int NC = kRClaim>
__device__ __forceinline__ void claim2(uint32_t* C, uint32_t bucket, uint32_t rank) {
  uint32_t h = mix32(bucket) & (NC - 1);
  const uint32_t k = ((bucket + 1u) << 9) | rank;
  for (int p = 0; p < NC; ++p) {
    const uint32_t prev = atomicCAS(&C[h], 0u, k);
    if (prev == 0u) return;
    if ((prev >> 9) == bucket + 1u) {
      atomicMin(&C[h], k);
      return;
    }
    h = (h + 1) & (NC - 1);
  }
}
template <int NC = kRClaim>
__device__ __forceinline__ uint32_t claim2_winner(const uint32_t* C, uint32_t bucket) {
  uint32_t h = mix32(bucket) & (NC - 1);
  for (int p = 0; p < NC; ++p) {
    const uint32_t v = C[h];
    if ((v >> 9) == bucket + 1u) return v & 511u;
    if (v == 0u) break;
    h = (h + 1) & (NC - 1);
  }
  return 0xFFFFFFFFu;
}
// VoxelHashTable's bucket lock within one launch, LDS form: true if this call took it
template <int N>
__device__ __forceinline__ bool lock_take2(uint32_t* S, uint32_t bucket) {
  uint32_t h = mix32(bucket ^ 0x9E3779B9u) & (N - 1);
  const uint32_t k = bucket + 1u;
  for (int p = 0; p < N; ++p) {
    const uint32_t prev = atomicCAS(&S[h], 0u, k);
    if (prev == 0u) return true;
    if (prev == k) return false;
    h = (h + 1) & (N - 1);
  }
  return false;
}
template <int N>
__device__ __forceinline__ bool lock_held(const uint32_t* S, uint32_t bucket) {
  uint32_t h = mix32(bucket ^ 0x9E3779B9u) & (N - 1);
  const uint32_t k = bucket + 1u;
  for (int p = 0; p < N; ++p) {
    const uint32_t v = S[h];
    if (v == k) return true;
    if (v == 0u) return false;
    h = (h + 1) & (N - 1);
  }
  return false;
}
// HBM form (launches with more keys than the LDS set holds): "locked" == this launch's epoch
__device__ __forceinline__ bool lock_take_hbm(uint32_t* tags, uint32_t bucket, uint32_t epoch) {
  if (tags[bucket] == epoch) return false;
  tags[bucket] = epoch;
  return true;
}

// exclusive scan over the 256-thread workgroup; scratch >= 4 ints
__device__ __forceinline__ int wg_excl_scan(int v, int* scratch, int* total) {
  const int w = threadIdx.x >> 6;
  const int incl = wave_incl_scan(v);
  if (lane_id() == 63) scratch[w] = incl;
  lds_barrier();
  const int s0 = scratch[0], s1 = scratch[1], s2 = scratch[2], s3 = scratch[3];
  lds_barrier();
  *total = s0 + s1 + s2 + s3;
  const int before = (w > 0 ? s0 : 0) + (w > 1 ? s1 : 0) + (w > 2 ? s2 : 0);
  return before + incl - v;
}

// ascending sort of a[0..m) (m <= RB, unique values) by rank counting: each thread ranks its one
// (RB = kRT) or two (RB = 2 kRT) elements against all m with broadcast LDS reads
template <int RB = kRB>
__device__ __forceinline__ void rank_sort(unsigned long long* a, unsigned long long* tmp, int m) {
  static_assert(RB == kRT || RB == 2 * kRT, "rank_sort geometry");
  const int t = threadIdx.x;
  const unsigned long long x0 = t < m ? a[t] : ~0ull;
  const unsigned long long x1 = RB > kRT && t + kRT < m ? a[t + kRT] : ~0ull;
  // the sort keys' high words are unique: compare those, two elements per 16-B broadcast read
  const uint32_t h0 = (uint32_t)(x0 >> 32), h1 = (uint32_t)(x1 >> 32);
  if (t == 0 && (m & 1)) a[m] = ~0ull;  // pad to pairs (a has RB + 2 entries)
  lds_barrier();
  const uint4* a4 = reinterpret_cast<const uint4*>(a);
  int r0 = 0, r1 = 0;
  const int np = (m + 1) >> 1;
  int j = 0;
  for (; j + 8 <= np; j += 8) {  // 8 reads in flight per step (a dependent LDS read is ~50 cycles)
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = a4[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      r0 += (v[u].y < h0) + (v[u].w < h0);
      r1 += (v[u].y < h1) + (v[u].w < h1);
    }
  }
  for (; j < np; ++j) {
    const uint4 v = a4[j];
    r0 += (v.y < h0) + (v.w < h0);
    r1 += (v.y < h1) + (v.w < h1);
  }
  if (t < m) tmp[r0] = x0;
  if (RB > kRT && t + kRT < m) tmp[r1] = x1;
  lds_barrier();
  if (t < m) a[t] = tmp[t];
  if (RB > kRT && t + kRT < m) a[t + kRT] = tmp[t + kRT];
  lds_barrier();
}

// Threshold search for multi-batch launches: keys[i] >> 32 (unique in [lo, range)) for i < n in
// global scratch; returns thr > lo with count(lo <= key < thr) in [1, RB] (some key remains).
template <int RB = kRB>
__device__ __forceinline__ uint32_t batch_threshold(const unsigned long long* __restrict__ keys, int n, uint32_t lo,
                                    uint32_t range, uint32_t* hist, int* scratch) {
  uint32_t hi = range;
  for (;;) {
    const uint32_t w = (hi - lo + kRHist - 1) / kRHist;
    for (int i = threadIdx.x; i < kRHist; i += kRT) hist[i] = 0u;
    lds_barrier();
    for (int i = threadIdx.x; i < n; i += kRT) {
      const uint32_t o = (uint32_t)(keys[i] >> 32);
      if (o >= lo && o < hi) atomicAdd(&hist[(o - lo) / w], 1u);
    }
    lds_barrier();
    // inclusive prefix of the 1024 bins, 4 per thread
    uint32_t c[4];
    int local = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c[k] = hist[threadIdx.x * 4 + k];
      local += (int)c[k];
    }
    int tot;
    int run = wg_excl_scan(local, scratch, &tot);
    // largest bin j whose inclusive prefix <= RB
    int best = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      run += (int)c[k];
      if (run <= RB) best = threadIdx.x * 4 + k;
    }
    lds_barrier();
    if (threadIdx.x == 0) scratch[4] = -1;
    lds_barrier();
    if (best >= 0) atomicMax(&scratch[4], best);
    lds_barrier();
    const int j = scratch[4];
    lds_barrier();
    if (j >= 0) {
      const unsigned long long thr = (unsigned long long)lo + (unsigned long long)(j + 1) * w;
      return thr > hi ? hi : (uint32_t)thr;
    }
    hi = lo + w;  // the first bin alone holds more than RB: narrow to it (w shrinks each time)
  }
}

// ---------------------------------------------------------------------------------------------
// Allocation resolver
// ---------------------------------------------------------------------------------------------
// RB keys per round: kRB (the frame kernels' tails, the standalone kernel) or kRT (the deferred
// resolve inside k_integrate, whose LDS budget is the update's: ~14 KiB instead of ~24).
template <int RB>
struct AllocLdsT {
  static constexpr int kClaim = 2 * RB, kLock = 4 * RB, kLockKeys = 3 * RB / 2;
  alignas(16) unsigned long long batch[RB + 2];  // (order << 32) | hint << 9 | p, ascending (+ pad)
  unsigned long long bkey[RB];   // packed key at position p
  int32_t bslot[RB];             // its new-key-set slot
  int32_t heap_top[RB];          // heap_top[i] = heap[free0 - 1 - i]
  union {
    uint32_t claim[kClaim];
    uint32_t hist[kRHist];
    unsigned long long tmp[RB];
  } u;
  uint32_t lock[kLock];
  int scan[8];
  int first_dirty, base, sfree, nfresh, nalloc, changed, m;
};
using AllocLds = AllocLdsT<kRB>;
static_assert(AllocLds::kClaim == kRClaim && AllocLds::kLock == kRLockA && AllocLds::kLockKeys == kRLockKeysA,
              "resolver geometry");
// batch low word: p (9 bits) | hint: bit 9 slot 0 empty, bit 10 slot 1 empty, bit 11 hint valid,
// bits 16..31 slot 1's list offset -- the key's bucket as the prologue loaded it (the table as the
// launch found it: valid until the first commit)
constexpr uint32_t kHintS0 = 1u << 9, kHintS1 = 1u << 10, kHintValid = 1u << 11;

// one key of an allocation round (registers)
struct AKey {
  bool have;
  int kind, slot, p;  // kind 1: SLOT(B, slot); 2: APPEND(tail T, empty slot-0 entry E)
  uint32_t B, T, E;
  int16_t x, y, z;
};

// ---------------------------------------------------------------------------------------------
// One-wave fast path of the allocation resolver for launches with <= 64 new keys (the steady state
// of a frame stream: ~50-80 new keys per 640x480 frame). The same rounds as resolve_alloc_wg --
// candidate order, speculative evaluation against the table, the longest prefix whose buckets are
// pairwise distinct commits -- with one key per lane and wave-level operations instead of LDS
// tables and workgroup barriers: the rank of each key by readlane comparisons and a ds_permute
// into rank order, the first conflicting rank by readlane comparisons of the claimed buckets, pool
// pops by the lane-mask prefix count of the committing owned keys. Only the launch's bucket locks
// live in LDS (a 256-slot set; <= 2 locks per key).
// ---------------------------------------------------------------------------------------------
constexpr int kWaveKeys = 64;
constexpr int kWaveLockSlots = 256;
// Measured (r3, same box, interleaved): 7.25 us per frame against the workgroup resolver's 6.75 --
// the readlane rank / conflict loops cost more VALU latency than the barriers they replace. Kept for
// A/B builds (-DTSDF_WAVE_RESOLVE); off by default.
#ifdef TSDF_WAVE_RESOLVE
__device__ constexpr bool resolve_wave_off() { return false; }
#else
__device__ constexpr bool resolve_wave_off() { return true; }
#endif

__device__ __forceinline__ unsigned long long lanemask_lt() {
  return (1ull << lane_id()) - 1ull;
}
// lane `rank` receives v (ranks distinct in [0, 64))
__device__ __forceinline__ uint32_t push_to(uint32_t v, int rank) {
  return (uint32_t)__builtin_amdgcn_ds_permute(rank << 2, (int)v);
}

__device__ __forceinline__ void resolve_alloc_wave(const EngineDev& D, const FrameParams& P, int frame_mode, int n, int free0,
                                   unsigned long long key_in, int32_t slot_in, uint32_t* lockset,
                                   unsigned long long tick0) {
  const int l = lane_id();
  // ---- round trip 2: candidate orders, the keys' buckets, the free-stack top ----
  uint32_t ord = 0xFFFFFFFFu, hint = 0u;
  if (l < n) {
    int16_t x, y, z;
    unpack_key(key_in, x, y, z);
    const uint32_t B = hash_block(x, y, z);
    ord = ld_co(&D.nk_order[slot_in]);
    const Ent s0 = load_ent(D.table, 2 * B), s1 = load_ent(D.table, 2 * B + 1);
    hint = (s0.idx < 0 ? 1u : 0u) | (s1.idx < 0 ? 2u : 0u) | ((uint32_t)(uint16_t)s1.off << 16);
  }
  const int32_t htop = l < min(n, max(free0, 0)) ? D.heap[free0 - 1 - l] : 0;  // heap[free0 - 1 - l]
  for (int i = l; i < kWaveLockSlots; i += 64) lockset[i] = 0u;
  // ---- keys into candidate order: lane r <- the key of rank r (orders are unique per key) ----
  int rank = 0;
#pragma unroll 16
  for (int j = 0; j < 64; ++j) {
    const uint32_t oj = __builtin_amdgcn_readlane(ord, j);
    rank += (oj < ord) || (oj == ord && j < l);
  }
  const unsigned long long key =
      ((unsigned long long)push_to((uint32_t)(key_in >> 32), rank) << 32) | push_to((uint32_t)key_in, rank);
  const int32_t slot = (int32_t)push_to((uint32_t)slot_in, rank);
  const uint32_t hint0 = push_to(hint, rank);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");  // (the lock set cleared above)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  const bool have = l < n;
  int16_t x = 0, y = 0, z = 0;
  uint32_t B = 0;
  if (have) {
    unpack_key(key, x, y, z);
    B = hash_block(x, y, z);
  }
  const bool owned = have && (P.shard_count <= 1 ||
                              brick_owner(x, y, z, (uint32_t)P.shard_count) == (uint32_t)P.shard_index);
  int base = 0, sfree = free0, nfresh = 0;
  bool first_round = true;
  while (base < n) {  // wave-uniform
    const bool act = have && l >= base;
    int kind = 0;
    uint32_t b1 = 0xFFFFFFFFu, b2 = 0xFFFFFFFFu, T = 0, E = 0;
    int sl = 0;
    if (act) {
      // the prologue's view of the bucket holds unless a commit of this launch wrote into it, and
      // every such commit locked it
      bool e0, e1;
      int16_t off1;
      if (first_round || !lock_held<kWaveLockSlots>(lockset, B)) {
        e0 = (hint0 & 1u) != 0;
        e1 = (hint0 & 2u) != 0;
        off1 = (int16_t)(hint0 >> 16);
      } else {
        const Ent s0 = load_ent(D.table, 2 * B), s1 = load_ent(D.table, 2 * B + 1);
        e0 = s0.idx < 0;
        e1 = s1.idx < 0;
        off1 = s1.off;
      }
      if (e0 || e1) {  // SLOT (voxel_hash.cu:79-91)
        kind = 1;
        sl = e0 ? 0 : 1;
        b1 = b2 = B;
      } else {  // APPEND (:93-119): tail T of the list from slot 1, first empty slot-0 entry E after it
        kind = 2;
        uint32_t last = 2 * B + 1;
        int16_t off = off1;
        while (off) {
          last = (uint32_t)(last + (int32_t)off) & kEntryMask;
          off = load_ent(D.table, last).off;
        }
        T = last;
        uint32_t nx = last;
        for (uint32_t q = 0; q < kNumEntry; ++q) {
          nx = (nx + 1) & kEntryMask;
          if ((nx & 1u) == 0u && load_ent(D.table, nx).idx < 0) break;
        }
        E = nx;
        b1 = T >> 1;
        b2 = E >> 1;
      }
    }
    // first rank (>= base) whose buckets meet an earlier key's of this round: the keys before it
    // take pairwise distinct buckets, so their locks and commits do not interact
    bool dirty = false;
    for (int j = base; j < n; ++j) {  // wave-uniform bounds
      const uint32_t c1 = __builtin_amdgcn_readlane(b1, j), c2 = __builtin_amdgcn_readlane(b2, j);
      dirty |= j < l && (c1 == b1 || c1 == b2 || c2 == b1 || c2 == b2);
    }
    const unsigned long long dm = __ballot(act && dirty);
    const int fd = dm ? __ffsll((long long)dm) - 1 : 64;
    const bool proc = act && l < fd;
    // atomicExch(&bucket_locks_[b], LOCKED) == FREE within the launch (locks of earlier rounds hold)
    bool ok = false;
    if (proc) {
      if (kind == 1)
        ok = lock_take2<kWaveLockSlots>(lockset, B);
      else if (lock_take2<kWaveLockSlots>(lockset, b1))
        ok = lock_take2<kWaveLockSlots>(lockset, b2);
    }
    // pool pops in key order among the committing keys this engine holds
    const bool mine = ok && owned;
    const unsigned long long mm = __ballot(mine);
    const int prank = __popcll(mm & lanemask_lt());
    const int nmine = __popcll(mm);
    const int hi = sfree - 1 - prank;
    const int top = free0 - 1 - hi;  // pops so far this launch + rank (< n <= 64)
    const int32_t popped = __shfl(htop, top & 63, 64);
    if (ok) {
      int32_t idx = kForeignIdx;
      bool insert = true;
      if (mine) {
        if (hi < 0) {
          atomicOr(&D.ctr->status, 1u);  // TSDF_STATUS_POOL_EXHAUSTED
          insert = P.shard_count > 1;    // (see resolve_alloc_wg)
        } else {
          idx = popped;
        }
      }
      if (insert) {
        uint32_t e;
        if (kind == 1) {
          e = 2 * B + (uint32_t)sl;
        } else {
          const uint32_t wrap = E > T ? 0u : kNumEntry;
          store_off_co(D.table, T, (int16_t)(E + wrap - T));
          e = E;
        }
        store_ent_co(D.table, e, x, y, z, 0, idx);
        mark_swept_dirty(D, e);
        if (mine && idx == kForeignIdx) {  // voxel-less owned entry: carved this frame
          const int pk = atomicAdd(&D.ctr->n_pend, 1);
          if (pk < (int)kNewKeyCap) {
            VisRec pr;
            pr.x = x;
            pr.y = y;
            pr.z = z;
            pr.pad = 0;
            pr.idx = kForeignIdx;
            pr.entry = (int32_t)e;
            st_rec_co(&D.pend[pk], pr);
          }
        }
        if (local_idx(idx)) {
          atomicOr(&D.occ[e >> 6], 1ull << (e & 63));
          if (frame_mode) {  // fresh and visible this frame (see resolve_alloc_wg)
            VisRec vr;
            vr.x = x;
            vr.y = y;
            vr.z = z;
            vr.pad = 1;
            vr.idx = idx;
            vr.entry = (int32_t)e;
            st_rec_co(&D.fresh_vis[nfresh + prank], vr);
          } else {
            D.fresh[nfresh + prank] = idx;
          }
        }
      }
    }
    if (proc) {  // processed: the key-set slot is empty for the next frame
      st_co(&D.nk_key[slot], 0ull);
      st_co(&D.nk_order[slot], 0xFFFFFFFFu);
    }
    const int used = nmine < sfree ? nmine : (sfree > 0 ? sfree : 0);
    sfree -= used;
    nfresh += used;
    base = min(fd, n);
    first_round = false;
    if (base < n) {  // the next round reloads buckets this one wrote
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
  }
  if (l == 0) {
    D.ctr->resolve_alloc_ticks += __builtin_amdgcn_s_memrealtime() - tick0;
    D.ctr->free_count = sfree;
    st_co(&D.ctr->n_fresh, nfresh);
    st_co(&D.ctr->nk_count, 0);
    if (frame_mode) {
      D.ctr->last_alloc = nfresh;
      D.ctr->last_new_keys = n;
      D.ctr->total_alloc += (unsigned long long)nfresh;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Commit-all fast path of the allocation resolver (a frame stream's steady state: tens of new keys
// per frame in a table ~1 % full). When every key's bucket has an empty slot (the SLOT case of
// voxel_hash.cu:79-91), no two keys share a bucket and the pool holds a block for every key this
// engine owns, the canonical linearisation commits every key: each locks only its own bucket, so
// no lock is lost and no key writes another key's bucket, and AquireBlock's pops go to the owned
// keys in candidate order. Then there is no round, no sort and no claim table: one key per thread,
// the distinct-bucket test in the LDS lock set, each key's pop rank by a broadcast scan of the
// candidate orders. Any other launch returns false before anything global is written, and the
// ordered resolver below handles it. Results are identical either way (the oracle decides:
// tests/test_gpu_*.py run both paths).
// ---------------------------------------------------------------------------------------------
#ifdef TSDF_NO_FAST_RESOLVE
__device__ constexpr bool resolve_fast_off() { return true; }
#else
__device__ constexpr bool resolve_fast_off() { return false; }
#endif
constexpr int kFastLockSlots = 1024;

#ifdef TSDF_FAST_NOINLINE
#define FAST_INLINE __attribute__((noinline))
#else
#define FAST_INLINE
#endif
template <int RB>
__device__ FAST_INLINE bool resolve_alloc_fast(const EngineDev& D, const FrameParams& P, int frame_mode, int n, int free0,
                                   uint32_t epoch, unsigned long long key, int32_t slot, AllocLdsT<RB>& L,
                                   unsigned long long tick0) {
  static_assert(AllocLdsT<RB>::kLock >= kFastLockSlots && 2 * (RB + 2) >= kRT && RB >= kRT, "fast-path LDS");
  const int t = threadIdx.x, wave = t >> 6;
  const bool have = t < n;
  for (int i = t; i < kFastLockSlots; i += kRT) L.lock[i] = 0u;
  int16_t x = 0, y = 0, z = 0;
  uint32_t B = 0, ord = 0xFFFFFFFFu;
  bool e0 = false, e1 = false;
  if (have) {
    unpack_key(key, x, y, z);
    B = hash_block(x, y, z);
    ord = ld_co(&D.nk_order[slot]);
    const Ent s0 = load_ent(D.table, 2 * B), s1 = load_ent(D.table, 2 * B + 1);
    e0 = s0.idx < 0;
    e1 = s1.idx < 0;
  }
  const int32_t htop = t < min(n, max(free0, 0)) ? D.heap[free0 - 1 - t] : 0;
  const bool owned = have && (P.shard_count <= 1 ||
                              brick_owner(x, y, z, (uint32_t)P.shard_count) == (uint32_t)P.shard_index);
  lds_barrier();  // the lock set is zero
  // a key whose bucket an earlier key of the launch already holds would be dropped: not this path
  const bool bad = have && (!(e0 || e1) || !lock_take2<kFastLockSlots>(L.lock, B));
  uint32_t* ordv = reinterpret_cast<uint32_t*>(L.batch);
  ordv[t] = owned ? ord : 0xFFFFFFFFu;  // (threads >= n pad the scan with "never smaller")
  L.heap_top[t] = htop;
  const unsigned long long bo = __ballot(owned), bb = __ballot(bad);
  TSDF_STAMP(D, 1, 3);  // (diag) the keys' orders, buckets and heap top loaded
  if (lane_id() == 0) {
    L.scan[wave] = __popcll(bo);
    L.scan[4 + wave] = __popcll(bb);
  }
  lds_barrier();
  TSDF_STAMP(D, 1, 4);
  const int nowned = L.scan[0] + L.scan[1] + L.scan[2] + L.scan[3];
  if (L.scan[4] + L.scan[5] + L.scan[6] + L.scan[7] != 0 || nowned > free0) return false;
  if (have) {
    // pop rank: owned keys earlier in candidate order (orders are unique per key)
    int prank = 0;
    if (owned) {
      const uint4* v4 = reinterpret_cast<const uint4*>(ordv);
      const int nq = (n + 3) >> 2;
#pragma unroll 2
      for (int j = 0; j < nq; ++j) {
        const uint4 v = v4[j];
        prank += (v.x < ord) + (v.y < ord) + (v.z < ord) + (v.w < ord);
      }
    }
    const int32_t idx = owned ? L.heap_top[prank] : kForeignIdx;
    const uint32_t e = 2 * B + (e0 ? 0u : 1u);
    store_ent_co(D.table, e, x, y, z, 0, idx);
        mark_swept_dirty(D, e);
    if (owned) {
      atomicOr(&D.occ[e >> 6], 1ull << (e & 63));
      if (frame_mode) {
        VisRec vr;
        vr.x = x;
        vr.y = y;
        vr.z = z;
        vr.pad = 1;
        vr.idx = idx;
        vr.entry = (int32_t)e;
        st_rec_co(&D.fresh_vis[prank], vr);
      } else {
        D.fresh[prank] = idx;
      }
    }
    st_co(&D.nk_key[slot], 0ull);
    st_co(&D.nk_order[slot], 0xFFFFFFFFu);
  }
  TSDF_STAMP(D, 1, 5);  // (diag) the commits issued
  if (t == 0) {
    D.ctr->lock_epoch = epoch;
    D.ctr->resolve_alloc_ticks += __builtin_amdgcn_s_memrealtime() - tick0;
    D.ctr->free_count = free0 - nowned;
    st_co(&D.ctr->n_fresh, nowned);
    st_co(&D.ctr->nk_count, 0);
    if (frame_mode) {
      D.ctr->last_alloc = nowned;
      D.ctr->last_new_keys = n;
      D.ctr->total_alloc += (unsigned long long)nowned;
    }
  }
  return true;
}

// frame_mode 1: new blocks this engine holds are listed in D.fresh_vis (flagged fresh, visible this
// frame); 0 (hash-level test path): their pool indices in D.fresh for k_fresh_init.
template <int RB>
__device__ __forceinline__ void resolve_alloc_wg(const EngineDev& D, const FrameParams& P, uint32_t range, int frame_mode,
                                 AllocLdsT<RB>& L) {
  constexpr int NR = RB / kRT;  // keys per thread and round
  constexpr int NC = AllocLdsT<RB>::kClaim, NL = AllocLdsT<RB>::kLock;
  const int t = threadIdx.x;
  TSDF_STAMP(D, 1, 0);
  const unsigned long long tick0 = __builtin_amdgcn_s_memrealtime();
  // ---- prologue, round trip 1: counters and (speculatively) the first RB list entries ----
  const int n = ld_co(&D.ctr->nk_count);
  const int free0 = D.ctr->free_count;
  const uint32_t epoch0 = D.ctr->lock_epoch;
  unsigned long long k0 = ld_co(&D.nk_list[t].key), k1 = NR > 1 ? ld_co(&D.nk_list[t + kRT].key) : 0ull;
  int32_t h0 = (int32_t)ld_co(&D.nk_list[t].slot), h1 = NR > 1 ? (int32_t)ld_co(&D.nk_list[t + kRT].slot) : 0;
  const bool single = n <= RB;
  const bool lds_locks = n <= AllocLdsT<RB>::kLockKeys;
  TSDF_STAMP(D, 1, 7);  // (diag) counters and key list loaded
  const uint32_t epoch = epoch0 + 1u;
  if (n <= kRT && !resolve_fast_off()) {
    if (resolve_alloc_fast<RB>(D, P, frame_mode, n, free0, epoch, k0, h0, L, tick0)) return;
    lds_barrier();  // fallback: the ordered rounds below reuse the LDS the fast path used
  }
  if (n <= kWaveKeys && !resolve_wave_off()) {  // one-wave fast path; the other waves are done
    static_assert(AllocLdsT<RB>::kLock >= kWaveLockSlots, "lock set");
    if (t == 0) D.ctr->lock_epoch = epoch;
    if (t < 64) resolve_alloc_wave(D, P, frame_mode, n, free0, k0, h0, L.lock, tick0);
    return;
  }
  if (lds_locks)
    for (int i = t; i < NL; i += kRT) L.lock[i] = 0u;
  if (t == 0) {
    D.ctr->lock_epoch = epoch;
    L.sfree = free0;
    L.nfresh = 0;
    L.nalloc = 0;
    L.changed = 0;
  }
  // ---- round trip 2: candidate orders, the keys' buckets, the free-stack top ----
  {
    const int npre = min(min(n, RB), max(free0, 0));
    for (int i = t; i < npre; i += kRT) L.heap_top[i] = D.heap[free0 - 1 - i];
  }
  if (single) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int p = t + r * kRT;
      if (p < n) {
        const unsigned long long key = r ? k1 : k0;
        const int32_t h = r ? h1 : h0;
        int16_t x, y, z;
        unpack_key(key, x, y, z);
        const uint32_t B = hash_block(x, y, z);
        const uint32_t ord = ld_co(&D.nk_order[h]);
        const Ent s0 = load_ent(D.table, 2 * B), s1 = load_ent(D.table, 2 * B + 1);
        const uint32_t hint = (s0.idx < 0 ? kHintS0 : 0u) | (s1.idx < 0 ? kHintS1 : 0u) | kHintValid |
                              ((uint32_t)(uint16_t)s1.off << 16);
        L.bkey[p] = key;
        L.bslot[p] = h;
        L.batch[p] = ((unsigned long long)ord << 32) | hint | (uint32_t)p;
      }
    }
  } else {
    // scratch of every key: (order << 32) | list index, for the batch threshold search
    for (int i = t; i < n; i += kRT) {
      const int32_t h = (int32_t)ld_co(&D.nk_list[i].slot);
      D.pairs[i] = ((unsigned long long)ld_co(&D.nk_order[h]) << 32) | (uint32_t)i;
    }
  }
  if (single) lds_barrier(); else __syncthreads();  // (D.pairs: global)
  TSDF_STAMP(D, 1, 1);
  uint32_t lo = 0u;
  int done = 0;
  while (done < n) {
    int m;
    uint32_t thr = 0xFFFFFFFFu;
    if (single) {
      m = n;
    } else {
      if (n - done > RB) thr = batch_threshold<RB>(D.pairs, n, lo, range, L.u.hist, L.scan);
      // gather the batch [lo, thr) into LDS (list order; the sort below orders it)
      if (t == 0) L.m = 0;
      lds_barrier();
      for (int i = t; i < n; i += kRT) {
        const unsigned long long pr = D.pairs[i];
        const uint32_t o = (uint32_t)(pr >> 32);
        if (o >= lo && o < thr) {
          const int p = atomicAdd(&L.m, 1);
          const int li = (int)(pr & 0xFFFFFFFFu);
          L.bkey[p] = ld_co(&D.nk_list[li].key);
          L.bslot[p] = (int32_t)ld_co(&D.nk_list[li].slot);
          L.batch[p] = (pr & 0xFFFFFFFF00000000ull) | (uint32_t)p;  // no hint: load the bucket
        }
      }
      lds_barrier();
      m = L.m;
    }
    rank_sort<RB>(L.batch, L.u.tmp, m);
    TSDF_STAMP(D, 1, 2);
#if defined(TSDF_EXP) && (TSDF_EXP & 16)  // experiment: the same sort again, instruction cache warm
    rank_sort<RB>(L.batch, L.u.tmp, m);
    TSDF_STAMP(D, 1, 7);
#endif
    if (t == 0) L.base = 0;
    lds_barrier();
    while (L.base < m) {
      // one round: the next min(RB, m - base) keys in order, NR per thread (ranks t, t + kRT)
      const int base = L.base;
      const int span = min(RB, m - base);
      for (int i = t; i < NC; i += kRT) L.u.claim[i] = 0u;
      if (t == 0) L.first_dirty = RB;
      lds_barrier();
      AKey k[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        k[r] = AKey{};
        const int rank = t + r * kRT;
        if (rank < span) {
          k[r].have = true;
          const uint32_t lw = (uint32_t)L.batch[base + rank];
          k[r].p = (int)(lw & 511u);
          unpack_key(L.bkey[k[r].p], k[r].x, k[r].y, k[r].z);
          const uint32_t B = hash_block(k[r].x, k[r].y, k[r].z);
          k[r].B = B;
          // the prologue's view of the bucket holds unless a commit of this launch wrote into it,
          // and every such commit locked it
          const bool fresh = (lw & kHintValid) && (lds_locks ? !lock_held<NL>(L.lock, B) : !L.changed);
          bool e0, e1;
          int16_t off1;
          if (fresh) {
            e0 = (lw & kHintS0) != 0;
            e1 = (lw & kHintS1) != 0;
            off1 = (int16_t)(lw >> 16);
          } else {
            const Ent s0 = load_ent(D.table, 2 * B), s1 = load_ent(D.table, 2 * B + 1);
            e0 = s0.idx < 0;
            e1 = s1.idx < 0;
            off1 = s1.off;
          }
          if (e0 || e1) {
            k[r].kind = 1;
            k[r].slot = e0 ? 0 : 1;
            claim2<NC>(L.u.claim, B, (uint32_t)rank);
          } else {  // APPEND: tail T of the list from slot 1, first empty slot-0 entry E after it
            k[r].kind = 2;
            uint32_t last = 2 * B + 1;
            int16_t off = off1;
            while (off) {
              last = (uint32_t)(last + (int32_t)off) & kEntryMask;
              off = load_ent(D.table, last).off;
            }
            k[r].T = last;
            uint32_t nx = last;
            for (uint32_t q = 0; q < kNumEntry; ++q) {
              nx = (nx + 1) & kEntryMask;
              if ((nx & 1u) == 0u && load_ent(D.table, nx).idx < 0) break;
            }
            k[r].E = nx;
            claim2<NC>(L.u.claim, last >> 1, (uint32_t)rank);
            claim2<NC>(L.u.claim, nx >> 1, (uint32_t)rank);
          }
        }
      }
      lds_barrier();
      TSDF_STAMP(D, 1, 3);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (!k[r].have) continue;
        const uint32_t rank = (uint32_t)(t + r * kRT);
        const bool clean = k[r].kind == 1 ? claim2_winner<NC>(L.u.claim, k[r].B) == rank
                                          : (claim2_winner<NC>(L.u.claim, k[r].T >> 1) == rank &&
                                             claim2_winner<NC>(L.u.claim, k[r].E >> 1) == rank);
        if (!clean) atomicMin(&L.first_dirty, (int)rank);
      }
      lds_barrier();
      TSDF_STAMP(D, 1, 4);
      const int first_dirty = L.first_dirty;
      bool ok[2] = {false, false}, mine[2] = {false, false};
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (!k[r].have || t + r * kRT >= first_dirty) continue;
        // atomicExch(&bucket_locks_[b], LOCKED) == FREE, per launch; the keys committing together
        // won all their claims, so they take distinct buckets
        if (k[r].kind == 1) {
          ok[r] = lds_locks ? lock_take2<NL>(L.lock, k[r].B) : lock_take_hbm(D.lock_tag, k[r].B, epoch);
        } else {
          const uint32_t Lb = k[r].T >> 1, C = k[r].E >> 1;
          if (lds_locks ? lock_take2<NL>(L.lock, Lb) : lock_take_hbm(D.lock_tag, Lb, epoch))
            ok[r] = lds_locks ? lock_take2<NL>(L.lock, C) : lock_take_hbm(D.lock_tag, C, epoch);
        }
        // Sharded volume: every shard commits every key's table change (the replicated index), and
        // only the key's owner pops a pool block; the others store kForeignIdx.
        mine[r] = ok[r] && (P.shard_count <= 1 || brick_owner(k[r].x, k[r].y, k[r].z, (uint32_t)P.shard_count) ==
                                                      (uint32_t)P.shard_index);
      }
      // pool pops in key order: rank among this round's owned commits (first half, then second)
      int tot;
      const int ex = wg_excl_scan((mine[0] ? 1 : 0) | (mine[1] ? 1 << 16 : 0), L.scan, &tot);
      const int prank[2] = {ex & 0xFFFF, (tot & 0xFFFF) + (ex >> 16)};
      const int nmine = (tot & 0xFFFF) + (tot >> 16);
      const int free_now = L.sfree;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (!k[r].have) continue;
        if (ok[r]) {
          int32_t idx = kForeignIdx;
          bool insert = true;
          if (mine[r]) {
            const int hi = free_now - 1 - prank[r];
            if (hi < 0) {
              atomicOr(&D.ctr->status, 1u);  // TSDF_STATUS_POOL_EXHAUSTED
              // one volume drops the insert; a shard keeps a voxel-less entry so that every
              // shard's index stays the same
              insert = P.shard_count > 1;
            } else {
              const int top = free0 - 1 - hi;  // pops so far this launch + rank
              idx = top < RB ? L.heap_top[top] : D.heap[hi];
            }
          }
          if (insert) {
            uint32_t e;
            if (k[r].kind == 1) {
              e = 2 * k[r].B + (uint32_t)k[r].slot;
            } else {
              const uint32_t T = k[r].T, E = k[r].E;
              const uint32_t wrap = E > T ? 0u : kNumEntry;
              store_off_co(D.table, T, (int16_t)(E + wrap - T));
              e = E;
            }
            store_ent_co(D.table, e, k[r].x, k[r].y, k[r].z, 0, idx);
            mark_swept_dirty(D, e);
            if (mine[r] && idx == kForeignIdx) {
              // a shard's owned entry without voxels (its pool is exhausted): listed for this
              // frame's carving, so no voxel-less owned entry outlives the frame and the key is
              // retried once the DDA meets it again (one volume drops the insert instead)
              const int pk = atomicAdd(&D.ctr->n_pend, 1);
              if (pk < (int)kNewKeyCap) {
                VisRec pr;
                pr.x = k[r].x;
                pr.y = k[r].y;
                pr.z = k[r].z;
                pr.pad = 0;
                pr.idx = kForeignIdx;
                pr.entry = (int32_t)e;
                st_rec_co(&D.pend[pk], pr);
              }
            }
            L.changed = 1;  // (a benign race: every writer stores 1)
            if (local_idx(idx)) {  // the occupancy bitmap lists the blocks this engine holds
              atomicOr(&D.occ[e >> 6], 1ull << (e & 63));
              if (frame_mode) {
                // a new block has all 8 corners in view, so it is visible this frame: listed for
                // k_integrate after the blocks the visibility sweep listed, flagged fresh so it
                // starts from AquireBlock's state
                VisRec vr;
                vr.x = k[r].x;
                vr.y = k[r].y;
                vr.z = k[r].z;
                vr.pad = 1;
                vr.idx = idx;
                vr.entry = (int32_t)e;
                st_rec_co(&D.fresh_vis[L.nfresh + prank[r]], vr);
              } else {
                D.fresh[L.nfresh + prank[r]] = idx;
              }
            }
          }
        }
        if (t + r * kRT < first_dirty) {  // processed: the key-set slot is empty for the next frame
          st_co(&D.nk_key[L.bslot[k[r].p]], 0ull);
          st_co(&D.nk_order[L.bslot[k[r].p]], 0xFFFFFFFFu);
        }
      }
      // the table writes must be visible to the next round's loads; after the launch's last round
      // nothing here reads them (the next kernel does, after the boundary)
      if (first_dirty < span || base + span < m || done + m < n) __syncthreads(); else lds_barrier();
      TSDF_STAMP(D, 1, 5);
      if (t == 0) {
        const int used = nmine < free_now ? nmine : (free_now > 0 ? free_now : 0);
        L.sfree = free_now - used;
        L.nfresh += used;
        L.nalloc += used;
        L.base = base + (first_dirty < span ? first_dirty : span);
      }
      lds_barrier();
    }
    done += m;
    lo = thr;
  }
  TSDF_STAMP(D, 1, 6);
  if (t == 0) {
    D.ctr->resolve_alloc_ticks += __builtin_amdgcn_s_memrealtime() - tick0;
    D.ctr->free_count = L.sfree;
    st_co(&D.ctr->n_fresh, L.nfresh);
    st_co(&D.ctr->nk_count, 0);
    if (frame_mode) {
      D.ctr->last_alloc = L.nalloc;
      D.ctr->last_new_keys = n;
      D.ctr->total_alloc += (unsigned long long)L.nalloc;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Carving resolver
// ---------------------------------------------------------------------------------------------
struct DeleteLds {
  alignas(16) unsigned long long batch[kRB + 2];  // (entry << 32) | hint << 9 | p, ascending (+ pad)
  unsigned long long bkey[kRB];   // packed key at position p
  int32_t bidx0[kRB];             // slot 0's pool index when the hint says slot 0 holds the key
  union {
    uint32_t claim[kRClaim];
    uint32_t hist[kRHist];
    unsigned long long tmp[kRB];
  } u;
  uint32_t lock[kRLockD];
  int scan[8];
  int sfree, ndel, changed, m;
};
constexpr uint32_t kHintSlot0 = 1u << 9;  // (with kHintValid) slot 0 holds the key

// Commit-all fast path of the carving resolver: when every candidate sits in slot 0 of its own
// bucket (voxel_hash.cu:126-135: the lock-free delete) or is its bucket's list head with no list
// behind it (:137-152 with offset 0: the head "moves onto itself", i.e. is cleared; it locks the
// bucket, and a bucket has one head), the deletes touch distinct entries, win every lock and read
// nothing another delete writes, so the entry-ordered linearisation commits them all; only
// ReleaseBlock's pushes are ordered (by hash entry). Any other launch returns false before anything
// global is written and the ordered rounds below handle it.
// Pipelined frames. rel_fid != 0: ReleaseBlock also tags the released pool block rtag = rel_fid (the
// update workgroups that deferred it drop it). fo_fid != 0: a deleted key that frame fo_fid's DDA
// found in the table -- at entry e, where the key sat when it was deleted (one structural change per
// bucket per launch: its entry cannot have moved in between) -- goes back into the new-key set with
// that frame's smallest candidate order (D.fo, tsdf_ingest.h): its key is missing again.
__device__ __forceinline__ void carved_key(const EngineDev& D, uint32_t e, int16_t x, int16_t y, int16_t z,
                                           uint32_t fo_fid) {
  if (!fo_fid) return;
  const unsigned long long w = D.fo[e];
  if ((uint32_t)(w >> 32) == ~fo_fid) nk_insert(D, pack_key(x, y, z), (uint32_t)w);
}
__device__ __forceinline__ bool resolve_delete_fast(const EngineDev& D, int n, int free0, uint32_t epoch, int direct,
                                    const unsigned long long (&a)[2], DeleteLds& L, unsigned long long tick0,
                                    uint32_t rel_fid, uint32_t fo_fid) {
  const int t = threadIdx.x, wave = t >> 6;
  int16_t x[2] = {0, 0}, y[2] = {0, 0}, z[2] = {0, 0};
  uint32_t A[2] = {0u, 0u}, entry[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
  int32_t idx[2] = {-1, -1};
  bool bad = false, rel[2] = {false, false};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (t + r * kRT >= n) continue;
    x[r] = (int16_t)(a[r] & 0xFFFF);
    y[r] = (int16_t)((a[r] >> 16) & 0xFFFF);
    z[r] = (int16_t)((a[r] >> 32) & 0xFFFF);
    A[r] = hash_block(x[r], y[r], z[r]);
    const Ent s0 = load_ent(D.table, 2 * A[r]), s1 = load_ent(D.table, 2 * A[r] + 1);
    const bool in0 = s0.x == x[r] && s0.y == y[r] && s0.z == z[r] && s0.idx >= 0;
    const bool head = !in0 && s1.x == x[r] && s1.y == y[r] && s1.z == z[r] && s1.idx >= 0 && s1.off == 0;
    bad |= !(in0 || head);
    // the entry as the table holds it now (a pipelined frame's record may predate an earlier carving)
    entry[r] = 2 * A[r] + (head ? 1u : 0u);
    if (head) A[r] |= 0x80000000u;  // (the entry is 2 A + 1)
    idx[r] = in0 ? s0.idx : s1.idx;
    rel[r] = (in0 || head) && local_idx(idx[r]);
  }
  uint32_t* ev = reinterpret_cast<uint32_t*>(L.batch);  // entries of the released candidates
  ev[t] = rel[0] ? entry[0] : 0xFFFFFFFFu;
  ev[t + kRT] = rel[1] ? entry[1] : 0xFFFFFFFFu;
  const unsigned long long bb = __ballot(bad);
  const unsigned long long br = __ballot(rel[0]), br1 = __ballot(rel[1]);
  if (lane_id() == 0) {
    L.scan[wave] = __popcll(bb);
    L.scan[4 + wave] = __popcll(br) + __popcll(br1);
  }
  TSDF_STAMP(D, 4, 3);  // (diag) the candidates' buckets loaded
  lds_barrier();
  if (L.scan[0] + L.scan[1] + L.scan[2] + L.scan[3] != 0) return false;
  const int nrel = L.scan[4] + L.scan[5] + L.scan[6] + L.scan[7];
  const int nq = (min(n, kRB) + 3) >> 2;
  const uint4* v4 = reinterpret_cast<const uint4*>(ev);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (t + r * kRT >= n) continue;
    const uint32_t cur = 2 * (A[r] & 0x7FFFFFFFu) + (A[r] >> 31);
    store_off_idx_co(D.table, cur, 0, -1);
    atomicAnd(&D.occ[cur >> 6], ~(1ull << (cur & 63)));
    mark_swept_dirty(D, cur);
    if (rel[r]) {  // ReleaseBlock in entry order among the released blocks (entries are unique)
      int rank = 0;
#pragma unroll 2
      for (int j = 0; j < nq; ++j) {
        const uint4 v = v4[j];
        rank += (v.x < entry[r]) + (v.y < entry[r]) + (v.z < entry[r]) + (v.w < entry[r]);
      }
      D.heap[free0 + rank] = idx[r];
      if (rel_fid) st_co(&D.rtag[idx[r]], rel_fid);
    }
    carved_key(D, cur, x[r], y[r], z[r], fo_fid);
  }
  TSDF_STAMP(D, 4, 4);  // (diag) the deletes issued
  if (t == 0) {
    D.ctr->lock_epoch = epoch;
    D.ctr->free_count = free0 + nrel;
    D.ctr->resolve_delete_ticks += __builtin_amdgcn_s_memrealtime() - tick0;
    if (!direct) {
      D.ctr->last_deleted = nrel;
      D.ctr->total_deleted += (unsigned long long)nrel;
    }
  }
  return true;
}

// Carve candidates recs[0..*count) (VisRec: key and hash entry; any order). direct: the hash-level
// test path -- the candidates in list order, one per round (VoxelHashTable::Delete's launch of
// voxel_hash_test.cu).
// rel_fid / fo_fid: pipelined frames (released_block above). The deletes are ordered by the entry each
// candidate holds in the table NOW (its record's entry may predate an earlier carving that moved a list
// element into its bucket's head).
__device__ __forceinline__ void resolve_delete_wg(const EngineDev& D, const VisRec* __restrict__ recs,
                                  const int32_t* __restrict__ count, int direct, DeleteLds& L,
                                  uint32_t rel_fid = 0u, uint32_t fo_fid = 0u) {
  const int t = threadIdx.x;
  TSDF_STAMP(D, 4, 0);
  const unsigned long long tick0 = __builtin_amdgcn_s_memrealtime();
  const int n = ld_co(count);
  const int free0 = D.ctr->free_count;
  const uint32_t epoch = D.ctr->lock_epoch + 1u;
  const bool single = n <= kRB && !direct;
  const bool lds_locks = n <= kRLockKeysD;
  const unsigned long long* rq = reinterpret_cast<const unsigned long long*>(recs);
  unsigned long long a0 = 0, b0 = 0, a1 = 0, b1 = 0;  // records t, t + kRT (speculative)
  if (single) {
    a0 = ld_co(&rq[2 * t]);
    b0 = ld_co(&rq[2 * t + 1]);
    a1 = ld_co(&rq[2 * (t + kRT)]);
    b1 = ld_co(&rq[2 * (t + kRT) + 1]);
    if (!resolve_fast_off()) {
      const unsigned long long a[2] = {a0, a1};
      if (resolve_delete_fast(D, n, free0, epoch, direct, a, L, tick0, rel_fid, fo_fid)) return;
      lds_barrier();  // fallback: the ordered rounds below reuse the LDS the fast path used
    }
  }
  if (lds_locks)
    for (int i = t; i < kRLockD; i += kRT) L.lock[i] = 0u;
  if (t == 0) {
    D.ctr->lock_epoch = epoch;
    L.sfree = free0;
    L.ndel = 0;
    L.changed = 0;
  }
  if (single) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = t + r * kRT;
      if (p < n) {
        const unsigned long long a = r ? a1 : a0, b = r ? b1 : b0;
        const int16_t x = (int16_t)(a & 0xFFFF), y = (int16_t)((a >> 16) & 0xFFFF),
                      z = (int16_t)((a >> 32) & 0xFFFF);
        const Ent s0 = load_ent(D.table, 2 * hash_block(x, y, z));
        const bool in0 = s0.x == x && s0.y == y && s0.z == z && s0.idx >= 0;
        int32_t ce = in0 ? (int32_t)(2 * hash_block(x, y, z)) : find_entry(D.table, x, y, z);
        const uint32_t entry = ce >= 0 ? (uint32_t)ce : (uint32_t)(b >> 32);
        L.bkey[p] = pack_key(x, y, z);
        L.bidx0[p] = s0.idx;
        L.batch[p] = ((unsigned long long)entry << 32) | (in0 ? kHintSlot0 : 0u) | kHintValid | (uint32_t)p;
      }
    }
  } else if (!direct) {
    for (int i = t; i < n; i += kRT) {
      const unsigned long long a = ld_co(&rq[2 * i]);
      const int32_t ce = find_entry(D.table, (int16_t)(a & 0xFFFF), (int16_t)((a >> 16) & 0xFFFF),
                                    (int16_t)((a >> 32) & 0xFFFF));
      const uint32_t entry = ce >= 0 ? (uint32_t)ce : (uint32_t)ld_co(&recs[i].entry);
      D.pairs[i] = ((unsigned long long)entry << 32) | (uint32_t)i;
    }
  }
  if (single || direct) lds_barrier(); else __syncthreads();  // (D.pairs: global)
  TSDF_STAMP(D, 4, 1);
  uint32_t lo = 0u;
  int done = 0;
  while (done < n) {
    int m;
    uint32_t thr = 0xFFFFFFFFu;
    if (single) {
      m = n;
      rank_sort(L.batch, L.u.tmp, m);
    } else if (direct) {  // one candidate (list order) per round
      if (t == 0) {
        const VisRec r = recs[done];
        L.bkey[0] = pack_key(r.x, r.y, r.z);
        L.batch[0] = 0ull;
      }
      lds_barrier();
      m = 1;
    } else {
      if (n - done > kRB) thr = batch_threshold(D.pairs, n, lo, kNumEntry, L.u.hist, L.scan);
      if (t == 0) L.m = 0;
      lds_barrier();
      for (int i = t; i < n; i += kRT) {
        const unsigned long long pr = D.pairs[i];
        const uint32_t o = (uint32_t)(pr >> 32);
        if (o >= lo && o < thr) {
          const int p = atomicAdd(&L.m, 1);
          const int li = (int)(pr & 0xFFFFFFFFu);
          const unsigned long long a = ld_co(&rq[2 * li]);
          L.bkey[p] = pack_key((int16_t)(a & 0xFFFF), (int16_t)((a >> 16) & 0xFFFF), (int16_t)((a >> 32) & 0xFFFF));
          L.batch[p] = (pr & 0xFFFFFFFF00000000ull) | (uint32_t)p;
        }
      }
      lds_barrier();
      m = L.m;
      rank_sort(L.batch, L.u.tmp, m);
    }
    // rounds of 256 candidates in entry order; the deletes of a round touch disjoint entries (slot-0
    // deletes their own, list deletes one per bucket), so a whole round commits at once
    for (int base = 0; base < m; base += kRT) {
      for (int i = t; i < kRClaim; i += kRT) L.u.claim[i] = 0u;
      lds_barrier();
      const bool have = base + t < m;
      int kind = 0;  // 1 slot 0, 2 list head, 3 list element
      uint32_t A = 0, prev = 0, cur = 0;
      Ent ecur = {}, eprev = {};
      int16_t x = 0, y = 0, z = 0;
      if (have) {
        const unsigned long long v = L.batch[base + t];
        const uint32_t lw = (uint32_t)v;
        const int p = (int)(lw & 511u);
        unpack_key(L.bkey[p], x, y, z);
        A = hash_block(x, y, z);
        if ((lw & kHintValid) && (lw & kHintSlot0) && !L.changed) {  // slot 0 as loaded
          kind = 1;
          cur = 2 * A;
          ecur.idx = L.bidx0[p];
        } else {
          const Ent s0 = load_ent(D.table, 2 * A);
          if (s0.x == x && s0.y == y && s0.z == z && s0.idx >= 0) {
            kind = 1;
            cur = 2 * A;
            ecur = s0;
          } else {
            const Ent hd = load_ent(D.table, 2 * A + 1);
            if (hd.x == x && hd.y == y && hd.z == z && hd.idx >= 0) {
              kind = 2;
              prev = 2 * A + 1;
              eprev = hd;
              cur = (uint32_t)(prev + (int32_t)hd.off) & kEntryMask;  // element moved into the head
              ecur = load_ent(D.table, cur);
            } else {
              uint32_t last = 2 * A + 1;
              Ent bl = hd;
              while (bl.off) {
                const uint32_t c = (uint32_t)(last + (int32_t)bl.off) & kEntryMask;
                const Ent bc = load_ent(D.table, c);
                if (bc.x == x && bc.y == y && bc.z == z && bc.idx >= 0) {
                  kind = 3;
                  prev = last;
                  eprev = bl;
                  cur = c;
                  ecur = bc;
                  break;
                }
                last = c;
                bl = bc;
              }
            }
          }
        }
        if (kind >= 2) claim2(L.u.claim, A, (uint32_t)t);
      }
      lds_barrier();
      bool ok = false;
      int32_t released = -1;
      if (kind == 1) {
        ok = true;
      } else if (kind >= 2 && claim2_winner(L.u.claim, A) == (uint32_t)t) {
        ok = lds_locks ? lock_take2<kRLockD>(L.lock, A) : lock_take_hbm(D.lock_tag, A, epoch);
      }
      if (ok) {
        if (kind == 1) {  // voxel_hash.cu:126-135
          released = ecur.idx;
          store_off_idx_co(D.table, cur, 0, -1);
        } else if (kind == 2) {  // :137-152 (cur aliases the head when the list is empty)
          released = eprev.idx;
          const int16_t noff = ecur.off ? (int16_t)(eprev.off + ecur.off) : (int16_t)0;
          store_ent_co(D.table, prev, ecur.x, ecur.y, ecur.z, noff, ecur.idx);
          store_off_idx_co(D.table, cur, 0, -1);
          // the next list element moved into the head entry: its occupancy bit moves with it
          // (a shard lists only its own blocks; one volume's head bit simply stays set)
          if (prev != cur) {
            if (local_idx(ecur.idx))
              atomicOr(&D.occ[prev >> 6], 1ull << (prev & 63));
            else
              atomicAnd(&D.occ[prev >> 6], ~(1ull << (prev & 63)));
          }
        } else {  // :154-170
          released = ecur.idx;
          const int16_t noff = ecur.off ? (int16_t)(eprev.off + ecur.off) : (int16_t)0;
          store_off_co(D.table, prev, noff);
          store_off_idx_co(D.table, cur, 0, -1);
        }
        atomicAnd(&D.occ[cur >> 6], ~(1ull << (cur & 63)));
        mark_swept_dirty(D, cur);
        if (kind == 2) mark_swept_dirty(D, prev);  // (the next element's content moved into prev)
        L.changed = 1;
      }
      // ReleaseBlock (voxel_mem.cu:54-59) of the blocks this engine holds (a shard deletes every
      // shard's candidates from its index, and releases only its own pool blocks)
      const bool rel = ok && local_idx(released);
      int nrel;
      const int rank = wg_excl_scan(rel ? 1 : 0, L.scan, &nrel);
      if (rel) {
        D.heap[L.sfree + rank] = released;
        if (rel_fid) st_co(&D.rtag[released], rel_fid);
      }
      if (ok) carved_key(D, kind == 2 ? prev : cur, x, y, z, fo_fid);  // (a list head's key lived at prev)
      if (base + kRT < m || done + m < n) __syncthreads(); else lds_barrier();
      if (t == 0) {
        L.sfree += nrel;
        L.ndel += nrel;
      }
      lds_barrier();
    }
    done += m;
    lo = thr;
  }
  TSDF_STAMP(D, 4, 2);
  if (t == 0) {
    D.ctr->free_count = L.sfree;
    D.ctr->resolve_delete_ticks += __builtin_amdgcn_s_memrealtime() - tick0;
  }
  if (t == 0 && !direct) {
    D.ctr->last_deleted = L.ndel;
    D.ctr->total_deleted += (unsigned long long)L.ndel;
  }
}

}  // namespace tsdf
