// tsdf_ingest.h -- the per-pixel-tile part of a frame's ingest: pixel records, the block-allocation
// DDA (block_allocate_kernel, utils/tsdf/voxel_tsdf.cu:104-147) into a per-tile LDS key set, the
// all-corners visibility of its keys and their table probe / new-key-set insert. Shared by
// k_ingest_dda (tsdf_alloc.hip) and the pipelined frame's k_frame (tsdf_fuse.hip), which runs the next
// frame's tiles while the current frame's blocks are updated.
#pragma once

#include "tsdf_block.h"
#include "tsdf_kernels.h"
#include "tsdf_resolve.h"

namespace tsdf {

// ---------------------------------------------------------------------------------------------
// k_ingest_dda: 16x16 pixel tile per workgroup.
//  1. pack the frame into per-pixel records the integrate kernel gathers (one 16-B gather per voxel):
//       pixA = {depth, +-range (range = |K^-1 [x y 1]|; negative: the pixel takes the semantic update's
//       exact path, sem_pixel_fast), logf(ht), logf(lt)} (sem_logf), pixC = rgb
//     (exactly the values tsdf_integrate_kernel recomputes per voxel, voxel_tsdf.cu:174-201; the
//     update computes w_new = (1 - d / max_depth) * 4 from the depth with the same operations)
//  2. DDA of [p - trunc dir, p + trunc dir] (voxel_tsdf.cu:116-146); block keys deduplicated in
//     an LDS hash set with their smallest candidate order (y*W + x)*maxs + i
//  3. each unique key once: all-8-corners visibility (is_block_visible<true>), table probe;
//     missing keys go to the global new-key set.
// The launch covers tiles [P.tile_lo, P.tile_hi): every tile of the frame, or a sharded frame's
// pixel slice. Step 1 runs only when P.pack_pixels (one volume); a shard's k_integrate gathers the
// raw frame, so a shard runs the DDA of its slice and nothing else per pixel. A shard probes its
// copy of the whole hash index, so its keys are exactly the ones one volume's DDA finds in those
// tiles, whichever shard owns them.
// ---------------------------------------------------------------------------------------------
// LDS key-set slots per 16x16 tile: TS > 256 pixels x maxs. 1024 for maxs <= 3 (the reference's
// 6x truncation / voxel ratio: 2-3 samples per pixel) keeps the workgroup at 16.5 KiB of LDS, so 9
// workgroups fit a CU and the whole 640x480 grid is resident at once; 2048 up to maxs = 6.
constexpr int kVisChunk = 1024;   // visibility sweep: 16 occupancy words x 64 entries per wave
static_assert(kBands == 16, "ResolveLds band arrays");

// LDS key-set slot of a block key: multiplicative hash of the two key words, top log2(TS) bits
// (a few VALU per DDA sample instead of a 64-bit mixer; placement only, the set is exact)
template <int TS>
__device__ __forceinline__ uint32_t tile_slot(uint64_t key) {
  const uint32_t h = (uint32_t)key * 0x9E3779B1u + (uint32_t)(key >> 32) * 0x85EBCA77u;
  return h >> (32 - __builtin_ctz(TS));
}

// The allocation resolver runs in rounds of kIngestRB keys: kRT, one key per thread (the frame's
// ~50-80 new keys fit one round either way). Measured against 2 kRT: the resolver 6.65 vs 7.15 us per
// frame (fewer registers and LDS reads per thread), 19.25k vs 19.09k frames/s; its LDS falls under the
// sweep's, so the union is 16.5 KiB instead of 24.6. (Forcing 7 or 8 resident workgroups per CU with
// that LDS, by capping the registers at 72 / 64, measured equal / slower: the ingest is not
// dispatch-bound.)
#ifndef TSDF_INGEST_RB
#define TSDF_INGEST_RB 256
#endif
constexpr int kIngestRB = TSDF_INGEST_RB;

// the two roles of k_ingest_dda share one LDS allocation
template <int TS>
struct IngestLds {
  union {
    struct {
      unsigned long long key[TS];
      uint32_t ord[TS];
      uint16_t vis[4][TS / 4];
    } tile;
    struct {
      uint32_t list[4][kVisChunk];
      int cnt[kBands], base[kBands];
      int npass;
      unsigned long long dm[4];  // (vis_sweep_chained) the carving's marks of each wave's 64 words
    } sweep;
    AllocLdsT<kIngestRB> res;  // the last-arriving workgroup's allocation resolve
  } u;
  int last;
};

// the workgroup waits until *flag == tag (thread 0 polls; bounded: a flag that never comes sets
// TSDF_STATUS_PIPELINE_TIMEOUT and the frame goes on, wrong but without a hung GPU)
#ifndef TSDF_PIPE_SLEEP
#define TSDF_PIPE_SLEEP 16
#endif
__device__ __forceinline__ void wait_tag(const unsigned long long* flag, uint32_t tag, uint32_t* status) {
  if (threadIdx.x == 0) {
    uint32_t n = 0;
    // polled with an atomic (performed past the L2): a plain or agent-scope load can keep hitting
    // this XCD's L2 copy of the line from the first poll, long after the tail wrote the tag
    while ((uint32_t)__hip_atomic_fetch_or(const_cast<unsigned long long*>(flag), 0ull, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) != tag) {
      __builtin_amdgcn_s_sleep(TSDF_PIPE_SLEEP);
      if (++n > (1u << 22)) {
        atomicOr(status, 64u);  // TSDF_STATUS_PIPELINE_TIMEOUT
        break;
      }
    }
  }
  __syncthreads();
}

// hash entry read at agent scope (two 8-byte atomic loads: the table is not being written while a
// chained tile or sweep reads it, so the halves are consistent)
__device__ __forceinline__ Ent load_ent_co(const int4* table, uint32_t e) {
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(table + e);
  const unsigned long long a = ld_co(q), b = ld_co(q + 1);
  Ent r;
  r.x = (int16_t)(a & 0xFFFF);
  r.y = (int16_t)((a >> 16) & 0xFFFF);
  r.z = (int16_t)((a >> 32) & 0xFFFF);
  r.off = (int16_t)((a >> 48) & 0xFFFF);
  r.idx = (int32_t)(uint32_t)b;
  return r;
}
template <bool Co>
__device__ __forceinline__ Ent load_ent_t(const int4* table, uint32_t e) {
  return Co ? load_ent_co(table, e) : load_ent(table, e);
}
// find_entry (tsdf_device.h) with the entry loads of load_ent_t<Co>
// (*idx: the entry's pool index when found)
template <bool Co>
__device__ __forceinline__ int32_t find_entry_t(const int4* __restrict__ table, int16_t x, int16_t y, int16_t z,
                                                int32_t* idx = nullptr) {
  const uint32_t e0 = hash_block(x, y, z) << 1;
  // (loading slot 1 beside slot 0 measured neutral: 24.1k either way; the probes are off the critical path)
  const Ent a = load_ent_t<Co>(table, e0);
  if (a.x == x && a.y == y && a.z == z && a.idx >= 0) {
    if (idx) *idx = a.idx;
    return (int32_t)e0;
  }
  Ent b = load_ent_t<Co>(table, e0 + 1);
  uint32_t last = e0 + 1;
  for (;;) {
    if (b.x == x && b.y == y && b.z == z && b.idx >= 0) {
      if (idx) *idx = b.idx;
      return (int32_t)last;
    }
    if (!b.off) return -1;
    last = (uint32_t)(last + (int32_t)b.off) & kEntryMask;
    b = load_ent_t<Co>(table, last);
  }
}

// ---------------------------------------------------------------------------------------------
// Visibility sweep (check_visibility_kernel + GatherVisible, voxel_tsdf.cu:82-93,388-397) over
// the 512 KiB occupancy bitmap instead of the 48 MiB table: every allocated block with any corner
// in view (no depth test) is appended to the list of the image band its centre projects into
// (LDS counts, one global atomic per band per pass). Workgroup `wg` covers occupancy words
// [256 wg, 256 wg + 256), 64 per wave, one per lane; each wave compacts the live entries of its
// words into LDS so the corner tests run 8 lanes per block on dense work, in passes of at most
// kVisChunk entries (one pass at the bench's ~1 % table occupancy; each pass costs three dependent
// global round trips). It runs inside k_ingest_dda, before allocation: it sees the
// blocks that existed after the previous frame's carving, and k_resolve_alloc appends the
// blocks it creates. Order within a list is irrelevant to the update; the carving resolver
// restores the reference's entry order for the deletes.
// ---------------------------------------------------------------------------------------------
// Co: the sweep of a pipelined frame after its wait (the chained sweep's fallback): the occupancy
// words and entries are read at agent scope
template <int TS, bool Co = false>
__device__ __forceinline__ void vis_sweep(const EngineDev& D, const FrameParams& P, int wg, IngestLds<TS>& S) {
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t* L = S.u.sweep.list[wave];
  int* s_cnt = S.u.sweep.cnt;
  int* s_base = S.u.sweep.base;
  const int grp = lane >> 3, corner = lane & 7;
  const int w = wg * 256 + wave * 64 + lane;
  const unsigned long long occ_all = Co ? ld_co(&D.occ[w]) : D.occ[w];
  const int cw = __popcll(occ_all);
  const int incl = wave_incl_scan(cw);
  const int excl = incl - cw;
  const int wave_total = __shfl(incl, 63, 64);
  if (threadIdx.x == 0) S.u.sweep.npass = 0;
  __syncthreads();
  if (lane == 0) atomicMax(&S.u.sweep.npass, (wave_total + kVisChunk - 1) / kVisChunk);
  __syncthreads();
  const int npass = S.u.sweep.npass;
  for (int pass = 0; pass < npass; ++pass) {
    if (threadIdx.x < kBands) s_cnt[threadIdx.x] = 0;
    // this pass lists the wave's live entries of rank [lo, lo + kVisChunk)
    const int lo = pass * kVisChunk;
    const int total = min(max(wave_total - lo, 0), kVisChunk);
    if (excl < lo + kVisChunk && incl > lo) {
      unsigned long long occ = occ_all;
      for (int r = excl; occ; ++r) {
        const int b = __ffsll((long long)occ) - 1;
        occ &= occ - 1;
        if (r >= lo && r < lo + kVisChunk) L[r - lo] = (uint32_t)(w * 64 + b);
      }
    }
    __syncthreads();
    // any-corner visibility (is_block_visible<false>), 8 lanes per block, one corner each; the
    // visible ones are packed in place as entry | band << 24
    int nvis = 0;
    for (int base = 0; base < total; base += 8) {
      const int i = base + grp;
      bool v = false;
      uint32_t e = 0;
      Ent en{};
      if (i < total) {
        e = L[i];
        en = load_ent_t<Co>(D.table, e);
        v = voxel_visible(P, (int16_t)((int16_t)(en.x << kBlockLenBits) + ((corner >> 0) & 1) * (kBlockLen - 1)),
                          (int16_t)((int16_t)(en.y << kBlockLenBits) + ((corner >> 1) & 1) * (kBlockLen - 1)),
                          (int16_t)((int16_t)(en.z << kBlockLenBits) + ((corner >> 2) & 1) * (kBlockLen - 1)));
      }
      const unsigned long long bal = __ballot(v);
      const bool lead = corner == 0 && i < total && ((bal >> (lane & ~7)) & 0xFFull) != 0;
      const unsigned long long leads = __ballot(lead);
      if (lead) {  // rank among this round's visible blocks; slots < base + 8 were all read above
        const int band = block_band(P, en.x, en.y, en.z);
        L[nvis + __popcll(leads & ((1ull << lane) - 1ull))] = e | ((uint32_t)band << 24);
        atomicAdd(&s_cnt[band], 1);
      }
      nvis += __popcll(leads);
    }
    __syncthreads();
    if (threadIdx.x < kBands) {  // one global atomic per non-empty band per pass
      const int cnt = s_cnt[threadIdx.x];
      s_base[threadIdx.x] = cnt ? atomicAdd(&D.band[threadIdx.x * kBandStride], cnt) : 0;
      s_cnt[threadIdx.x] = 0;
    }
    __syncthreads();
    for (int k = lane; k < nvis; k += 64) {
      const uint32_t pk = L[k];
      const uint32_t e = pk & 0xFFFFFFu;
      const int band = (int)(pk >> 24);
      const int pos = s_base[band] + atomicAdd(&s_cnt[band], 1);
      const Ent en = load_ent_t<Co>(D.table, e);
      VisRec r;
      r.x = en.x;
      r.y = en.y;
      r.z = en.z;
      r.pad = 0;  // existed before this frame (not fresh)
      r.idx = en.idx;
      r.entry = (int32_t)e;
      D.vis[(size_t)band * D.nblocks + pos] = r;
    }
    __syncthreads();  // L and the band counts are reused by the next pass
  }
}

// The chained sweep of a pipelined frame (k_frame: frame c's sweep inside the launch that carves
// frame c - 2 and allocates frame c - 1; "the carving" below is that launch's carving and allocation,
// both of which mark the words they change). Frame n's carving only clears entries and moves a list element into its head entry, and it
// marks every occupancy word it changes (D.swdirty, tsdf_resolve.h mark_swept_dirty); nothing else
// writes the table in the launch. So the listing and the visibility tests run BEFORE the carving is
// published (possibly while it runs), keeping each wave's visible blocks in LDS (entry | band << 24 in
// list[0, kPreMax), the record's x, y, z, idx in the 3 words per block after it); after the wait the
// workgroup takes its marks (and clears them), drops the blocks of marked words, re-lists and re-tests
// those words, and appends their visible blocks to the band lists directly. The result is the lists
// vis_sweep<TS, true> would build after the wait (order within a list is irrelevant). Every read of
// the occupancy and the table here is an atomic (performed past the L2 and not kept in it): a plain
// or agent-scope load would leave this XCD's L2 a pre-carving copy of the line, which the chained
// tiles' agent-scope probes after the wait would then read. A wave with more than kPreMax live
// entries (far above the bench's ~1 % occupancy) makes the workgroup wait and run the agent-scope
// sweep instead.
#ifndef TSDF_PRE_MAX  // (a test build lowers it to run the fallback)
#define TSDF_PRE_MAX 256
#endif
constexpr int kPreMax = TSDF_PRE_MAX;
__device__ __forceinline__ Ent load_ent_rmw(int4* table, uint32_t e) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(table + e);
  const unsigned long long a = __hip_atomic_fetch_or(q, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b = __hip_atomic_fetch_or(q + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Ent r;
  r.x = (int16_t)(a & 0xFFFF);
  r.y = (int16_t)((a >> 16) & 0xFFFF);
  r.z = (int16_t)((a >> 32) & 0xFFFF);
  r.off = (int16_t)((a >> 48) & 0xFFFF);
  r.idx = (int32_t)(uint32_t)b;
  return r;
}
template <int TS>
__device__ __forceinline__ void vis_sweep_chained(const EngineDev& D, const FrameParams& P, int wg, IngestLds<TS>& S,
                                  const unsigned long long* flag, uint32_t tag) {
  static_assert(kVisChunk >= 4 * kPreMax && kPreMax <= 256, "list + records of kPreMax blocks per wave");
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t* L = S.u.sweep.list[wave];
  uint32_t* R = L + kPreMax;
  int* s_cnt = S.u.sweep.cnt;
  int* s_base = S.u.sweep.base;
  const int grp = lane >> 3, corner = lane & 7;
  const int w = wg * 256 + wave * 64 + lane;
  const unsigned long long occ_all = __hip_atomic_fetch_or(&D.occ[w], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int cw = __popcll(occ_all);
  const int incl = wave_incl_scan(cw);
  const int excl = incl - cw;
  const int total = __shfl(incl, 63, 64);
  if (threadIdx.x == 0) S.u.sweep.npass = 0;
  __syncthreads();
  if (lane == 0) atomicMax(&S.u.sweep.npass, total);
  __syncthreads();
  if (S.u.sweep.npass > kPreMax) {  // (uniform) before any table read of this workgroup
    wait_tag(flag, tag, &D.ctr->status);
    if (threadIdx.x < 4)
      __hip_atomic_store(&D.swdirty[wg * 4 + threadIdx.x], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    vis_sweep<TS, true>(D, P, wg, S);
    return;
  }
  {
    unsigned long long occ = occ_all;
    for (int r = excl; occ; ++r) {
      const int b = __ffsll((long long)occ) - 1;
      occ &= occ - 1;
      L[r] = (uint32_t)(w * 64 + b);
    }
  }
  if (threadIdx.x < kBands) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  int nvis = 0;
  for (int base = 0; base < total; base += 8) {  // vis_sweep's any-corner test, 8 lanes per block
    const int i = base + grp;
    bool v = false;
    uint32_t e = 0;
    Ent en{};
    unsigned long long qa = 0ull, qb = 0ull;
    if (i < total) {
      e = L[i];
      if (corner == 0) {  // one lane of the 8 reads the entry (two 8-byte atomics), then broadcasts
        unsigned long long* q = reinterpret_cast<unsigned long long*>(D.table + e);
        qa = __hip_atomic_fetch_or(q, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        qb = __hip_atomic_fetch_or(q + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const int src = lane & ~7;
    const uint32_t a0 = __shfl((uint32_t)qa, src, 64), a1 = __shfl((uint32_t)(qa >> 32), src, 64);
    const uint32_t b0 = __shfl((uint32_t)qb, src, 64);
    if (i < total) {
      en.x = (int16_t)(a0 & 0xFFFFu);
      en.y = (int16_t)(a0 >> 16);
      en.z = (int16_t)(a1 & 0xFFFFu);
      en.idx = (int32_t)b0;
      v = voxel_visible(P, (int16_t)((int16_t)(en.x << kBlockLenBits) + ((corner >> 0) & 1) * (kBlockLen - 1)),
                        (int16_t)((int16_t)(en.y << kBlockLenBits) + ((corner >> 1) & 1) * (kBlockLen - 1)),
                        (int16_t)((int16_t)(en.z << kBlockLenBits) + ((corner >> 2) & 1) * (kBlockLen - 1)));
    }
    const unsigned long long bal = __ballot(v);
    const bool lead = corner == 0 && i < total && ((bal >> (lane & ~7)) & 0xFFull) != 0;
    const unsigned long long leads = __ballot(lead);
    if (lead) {  // slots < base + 8 were all read above
      const int k = nvis + __popcll(leads & ((1ull << lane) - 1ull));
      L[k] = e | ((uint32_t)block_band(P, en.x, en.y, en.z) << 24);
      R[3 * k] = (uint32_t)(uint16_t)en.x | ((uint32_t)(uint16_t)en.y << 16);
      R[3 * k + 1] = (uint32_t)(uint16_t)en.z;
      R[3 * k + 2] = (uint32_t)en.idx;
    }
    nvis += __popcll(leads);
  }
  // ---- frame n's carving published ----
  TSDF_STAMP_WG(D, 5, (int)blockIdx.x - D.integrate_grid_pre, 1);
  wait_tag(flag, tag, &D.ctr->status);
  TSDF_STAMP_WG(D, 5, (int)blockIdx.x - D.integrate_grid_pre, 2);
  if (threadIdx.x < 4)
    S.u.sweep.dm[threadIdx.x] = __hip_atomic_fetch_and(&D.swdirty[wg * 4 + threadIdx.x], 0ull, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned long long dm = S.u.sweep.dm[wave];  // bit j: word wg * 256 + wave * 64 + j
  if (dm) {  // (wave-uniform) drop the blocks of marked words, in place
    int keep = 0;
    for (int b0 = 0; b0 < nvis; b0 += 64) {
      const int k = b0 + lane;
      uint32_t pk = 0, r0 = 0, r1 = 0, r2 = 0;
      bool kp = false;
      if (k < nvis) {
        pk = L[k];
        r0 = R[3 * k];
        r1 = R[3 * k + 1];
        r2 = R[3 * k + 2];
        kp = !((dm >> (((pk & 0xFFFFFFu) >> 6) & 63)) & 1ull);
      }
      const unsigned long long kb = __ballot(kp);  // (every lane has read its slot)
      if (kp) {
        const int d = keep + __popcll(kb & ((1ull << lane) - 1ull));
        L[d] = pk;
        R[3 * d] = r0;
        R[3 * d + 1] = r1;
        R[3 * d + 2] = r2;
      }
      keep += __popcll(kb);
    }
    nvis = keep;
  }
  for (int k = lane; k < nvis; k += 64) atomicAdd(&s_cnt[L[k] >> 24], 1);
  __syncthreads();
  int gbase = 0;
  if (threadIdx.x < kBands) {  // one global atomic per non-empty band (its result waited for below)
    const int cnt = s_cnt[threadIdx.x];
    gbase = cnt ? atomicAdd(&D.band[threadIdx.x * kBandStride], cnt) : 0;
  }
  if ((dm >> lane) & 1ull) {  // this lane's word was changed: re-list and re-test it (any corner)
    unsigned long long occ = __hip_atomic_fetch_or(&D.occ[w], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (occ) {
      const int b = __ffsll((long long)occ) - 1;
      occ &= occ - 1;
      const uint32_t e = (uint32_t)(w * 64 + b);
      const Ent en = load_ent_rmw(D.table, e);
      bool v = false;
      for (int c = 0; c < 8; ++c)
        v |= voxel_visible(P, (int16_t)((int16_t)(en.x << kBlockLenBits) + ((c >> 0) & 1) * (kBlockLen - 1)),
                           (int16_t)((int16_t)(en.y << kBlockLenBits) + ((c >> 1) & 1) * (kBlockLen - 1)),
                           (int16_t)((int16_t)(en.z << kBlockLenBits) + ((c >> 2) & 1) * (kBlockLen - 1)));
      if (v) {
        const int band = block_band(P, en.x, en.y, en.z);
        const int pos = atomicAdd(&D.band[band * kBandStride], 1);
        VisRec r;
        r.x = en.x;
        r.y = en.y;
        r.z = en.z;
        r.pad = 0;
        r.idx = en.idx;
        r.entry = (int32_t)e;
        D.vis[(size_t)band * D.nblocks + pos] = r;
      }
    }
  }
  if (threadIdx.x < kBands) {
    s_base[threadIdx.x] = gbase;
    s_cnt[threadIdx.x] = 0;
  }
  __syncthreads();
  for (int k = lane; k < nvis; k += 64) {
    const uint32_t pk = L[k];
    const int band = (int)(pk >> 24);
    const int pos = s_base[band] + atomicAdd(&s_cnt[band], 1);
    VisRec r;
    r.x = (int16_t)(R[3 * k] & 0xFFFFu);
    r.y = (int16_t)(R[3 * k] >> 16);
    r.z = (int16_t)(R[3 * k + 1] & 0xFFFFu);
    r.pad = 0;  // existed before this frame (not fresh)
    r.idx = (int32_t)R[3 * k + 2];
    r.entry = (int32_t)(pk & 0xFFFFFFu);
    D.vis[(size_t)band * D.nblocks + pos] = r;
  }
}

// One 16x16 pixel tile. kTileFull: k_ingest_dda's tile -- pixel records, the DDA, the LDS key dedupe,
// the all-corners test, then the table probe and the new-key insert. kTileChained: the same tile of
// frame c inside a pipelined launch (k_frame): everything that reads only the frame and its camera runs
// while frame c - 1's blocks are updated; the probe and insert wait until frame c - 1's allocation has
// been published (*flag == tag) and read the table coherently (the allocation ran on another XCD). Frame
// c - 2's carving has not run yet (it runs in the next launch), so a key found now may be missing after
// it: a found key records its smallest candidate order in D.fo at its hash entry, tagged ~fid, and the
// carving re-inserts the keys it deletes (tsdf_resolve.h carved_key). Missing keys stay missing (a
// carving only deletes), so they go to the new-key set now.
constexpr int kTileFull = 0, kTileChained = 1;
#ifdef TSDF_CHAIN_PLAIN
constexpr bool kChainCoherentLoads = false;
#else
constexpr bool kChainCoherentLoads = true;
#endif

template <int TS, int Mode = kTileFull>
__device__ __forceinline__ void ingest_tile(const EngineDev& D, const FrameParams& P,
                                            const float* __restrict__ depth,
                                            const uint8_t* __restrict__ rgb,
                                            const float* __restrict__ ht,
                                            const float* __restrict__ lt, int tiles_x, int tile,
                                            IngestLds<TS>& S, const unsigned long long* flag = nullptr,
                                            uint32_t tag = 0u, uint32_t fid = 0u) {
  unsigned long long* s_key = S.u.tile.key;
  uint32_t* s_ord = S.u.tile.ord;
  TSDF_STAMP(D, 0, 0);
  for (int i = threadIdx.x; i < TS; i += 256) {
    s_key[i] = 0ull;
    s_ord[i] = 0xFFFFFFFFu;
  }
  __syncthreads();
  TSDF_STAMP(D, 0, 1);
  const int x = (tile % tiles_x) * 16 + (threadIdx.x & 15);
  const int y = (tile / tiles_x) * 16 + (threadIdx.x >> 4);
  // DDA state of this lane's ray (valid: a pixel of this slice with 0 < d <= max_depth)
  bool ray = false;
  int nsamp = 0;
  f3 pos{}, st{};
  uint32_t order0 = 0;
  if (x < P.W && y < P.H) {
    const int i = y * P.W + x;
    const float d = depth[i];
    const f3 pc = pixel_ray(P, x, y);
    const float range = sqrtf(dot3(pc, pc));  // img_depth_to_range (voxel_tsdf.cu:120)
    if (P.pack_pixels) {  // (a shard's k_integrate reads the raw frame instead)
      const uint32_t c = (uint32_t)rgb[3 * i] | ((uint32_t)rgb[3 * i + 1] << 8) |
                         ((uint32_t)rgb[3 * i + 2] << 16);
      const float h = ht ? ht[i] : 1.0f;
      const float l = lt ? lt[i] : 1.0f;
      // the range's sign carries sem_pixel_fast (range >= 1): negative = the update's exact path
      D.pixA[P.pix_off + i] = make_float4(d, sem_pixel_fast(h, l, d, P.max_depth) ? range : -range,
                                          sem_logf(h), sem_logf(l));
      D.pixC[P.pix_off + i] = c;
    }
    TSDF_STAMP(D, 0, 2);
    if (!(d == 0 || d > P.max_depth)) {
      const f3 pcd = {pc.x * d, pc.y * d, pc.z * d};
      const f3 pw = se3_apply(P.wq, P.wt, pcd);
      // pc / range (IEEE quotients; pc.z = 1): the Newton-refined pair division, exact in range
      const float rr = __builtin_amdgcn_rcpf(range);
      const v2f dxy = div_pair(v2(pc.x, pc.y), v2(range, range), v2(rr, rr), true, true);
      const v2f dz1 = div_pair(v2(pc.z, pc.z), v2(range, range), v2(rr, rr), true, false);
      const f3 dc = {dxy.x, dxy.y, dz1.x};
      const f3 dw = qrot(P.wq, dc);
      const f3 sw = {pw.x - dw.x * P.trunc, pw.y - dw.y * P.trunc, pw.z - dw.z * P.trunc};
      const f3 dg = {quot_const(dw.x, P.voxel, P.inv_voxel), quot_const(dw.y, P.voxel, P.inv_voxel),
                     quot_const(dw.z, P.voxel, P.inv_voxel)};
      const f3 sg = {quot_const(sw.x, P.voxel, P.inv_voxel), quot_const(sw.y, P.voxel, P.inv_voxel),
                     quot_const(sw.z, P.voxel, P.inv_voxel)};
      const float two_trunc = 2 * P.trunc;
      const f3 rg = {two_trunc * dg.x, two_trunc * dg.y, two_trunc * dg.z};
      const int step_grid =
          f2i(ceilf(fmaxf(fmaxf(fabsf(rg.x), fabsf(rg.y)), fabsf(rg.z)) / kBlockLen));
      const float div = fmaxf((float)step_grid, 1.0f);
      // ray / max(step_grid, 1): step_grid is 1 or 2 at the reference's 6x truncation / voxel
      // ratio, where the quotient is exact as a product; larger counts take the IEEE divide
      if (__builtin_expect(div <= 2.0f, 1)) {
        const float m = div == 2.0f ? 0.5f : 1.0f;
        st = {rg.x * m, rg.y * m, rg.z * m};
      } else {
        st = {rg.x / div, rg.y / div, rg.z / div};
      }
      pos = sg;
      ray = true;
      nsamp = step_grid + 1;
      if (nsamp > P.maxs) {
        atomicOr(&D.ctr->status, 4u);  // TSDF_STATUS_DDA_OVERFLOW
        nsamp = P.maxs;
      }
      order0 = (uint32_t)i * (uint32_t)P.maxs;
    }
  }
  // Samples s = 0 .. step_grid of every ray (voxel_tsdf.cu:141-146) into the tile's LDS key set
  // with their smallest candidate order. Neighbouring pixels mostly hit the same blocks, so a sample
  // whose key equals the key of the same step at the pixel to its left or above (a lane 1 or 16
  // lower: the wave's 16x4 pixels are in raster order), or of the previous step at this pixel, is
  // left out -- that sample has a smaller candidate order, and by induction some sample with the
  // key and an order no larger is inserted. That removes most same-key LDS atomics (the serialised
  // bank conflicts of r2's profile: 1.3 conflict cycles per LDS instruction cycle).
  unsigned long long prev_key = 0ull;
  for (int s = 0; s < P.maxs; ++s) {
    const bool on = ray && s < nsamp;  // (uniform loop; the shuffles need every lane)
    unsigned long long key = 0ull;
    if (on) {
      const int16_t kx = (int16_t)(round_s16(pos.x) >> kBlockLenBits);
      const int16_t ky = (int16_t)(round_s16(pos.y) >> kBlockLenBits);
      const int16_t kz = (int16_t)(round_s16(pos.z) >> kBlockLenBits);
      pos.x += st.x;
      pos.y += st.y;
      pos.z += st.z;
      key = pack_key(kx, ky, kz);
    }
    const int lane = lane_id();
    const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
    const uint32_t llo = __shfl_up(lo, 1, 64), lhi = __shfl_up(hi, 1, 64);
    const uint32_t ulo = __shfl_up(lo, 16, 64), uhi = __shfl_up(hi, 16, 64);
    const unsigned long long left = (lane & 15) ? (((unsigned long long)lhi << 32) | llo) : 0ull;
    const unsigned long long up = lane >= 16 ? (((unsigned long long)uhi << 32) | ulo) : 0ull;
    if (on && key != left && key != up && key != prev_key) {
      const uint32_t order = order0 + (uint32_t)s;
      uint32_t hs = tile_slot<TS>(key);
      for (int p = 0; p < TS; ++p) {
        const unsigned long long prev = atomicCAS(&s_key[hs], 0ull, key);
        if (prev == 0ull || prev == key) {
          atomicMin(&s_ord[hs], order);
          break;
        }
        hs = (hs + 1) & (TS - 1);
      }
    }
    prev_key = key;
  }
  TSDF_STAMP(D, 0, 3);
  __syncthreads();
  TSDF_STAMP(D, 0, 4);
  // Each wave sweeps its 64-slot strips; the few occupied slots of a strip (ballot) are tested
  // 8 at a time with 8 lanes per key, one block corner per lane (is_block_visible<true>), and the
  // fully visible ones are listed in LDS. The table probes and new-key inserts then run one key
  // per lane over that list, so the wave pays their memory latency once, not once per 8 keys.
  uint16_t(*s_vis)[TS / 4] = S.u.tile.vis;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const int grp = lane >> 3, corner = lane & 7;
  int nv = 0;
  for (int strip = wave; strip < TS / 64; strip += 4) {
    const unsigned long long skey = s_key[strip * 64 + lane];
    const unsigned long long occ = __ballot(skey != 0ull);
    const int n = __popcll(occ);
    for (int base = 0; base < n; base += 8) {
      const int want = base + grp;  // rank of the occupied slot this 8-lane group handles
      int src = 0;                  // lane holding that slot: binary search on prefix popcounts
#pragma unroll
      for (int step = 32; step > 0; step >>= 1)
        if (src + step < 64 && __popcll(occ & ((1ull << (src + step)) - 1ull)) <= want) src += step;
      const unsigned long long key = __shfl(skey, src, 64);
      bool vis = false;
      if (want < n) {
        int16_t kx, ky, kz;
        unpack_key(key, kx, ky, kz);
        vis = voxel_visible(P, (int16_t)((int16_t)(kx << kBlockLenBits) + ((corner >> 0) & 1) * (kBlockLen - 1)),
                            (int16_t)((int16_t)(ky << kBlockLenBits) + ((corner >> 1) & 1) * (kBlockLen - 1)),
                            (int16_t)((int16_t)(kz << kBlockLenBits) + ((corner >> 2) & 1) * (kBlockLen - 1)));
      }
      const unsigned long long bal = __ballot(vis);
      const bool lead = want < n && corner == 0 && ((bal >> (lane & ~7)) & 0xFFull) == 0xFFull;
      const unsigned long long leads = __ballot(lead);
      if (lead) s_vis[wave][nv + __popcll(leads & ((1ull << lane) - 1ull))] = (uint16_t)(strip * 64 + src);
      nv += __popcll(leads);
    }
  }
  TSDF_STAMP(D, 0, 6);  // (diag) corner tests done
  if (Mode == kTileChained) wait_tag(flag, tag, &D.ctr->status);  // the previous frame's allocation is published
  TSDF_STAMP(D, 0, 7);  // (diag) the allocation flag seen
  for (int i = lane; i < nv; i += 64) {
    const int slot = s_vis[wave][i];
    const unsigned long long key = s_key[slot];
    int16_t kx, ky, kz;
    unpack_key(key, kx, ky, kz);
    const int32_t e = find_entry_t<Mode == kTileChained && kChainCoherentLoads>(D.table, kx, ky, kz);
    if (e >= 0) {
      if (Mode == kTileChained) atomicMin(&D.fo[e], ((unsigned long long)~fid << 32) | s_ord[slot]);
      continue;
    }
    nk_insert(D, key, s_ord[slot]);
  }
  TSDF_STAMP(D, 0, 5);
}

}  // namespace tsdf
