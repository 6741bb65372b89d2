// tsdf_alloc.hip -- block allocation: frame ingest + DDA, and the in-order allocation resolver.
//
// Reference: TSDFGrid::Allocate (utils/tsdf/voxel_tsdf.cu:377-386) launching block_allocate_kernel
// (:104-147), which calls VoxelHashTable::Allocate (voxel_hash.cu:58-120) from every pixel
// thread. That insert is racy by design (one structural change per bucket per launch, losers
// dropped); this engine replays the canonical sequential linearisation:
// candidates in pixel raster order then DDA step, with the exact bucket-lock semantics.
#include "tsdf_block.h"
#include "tsdf_kernels.h"

namespace tsdf {

// ---------------------------------------------------------------------------------------------
// per-frame new-key set: open addressing on 64-bit packed keys, min candidate order per key
// ---------------------------------------------------------------------------------------------
__device__ void keyset_insert(unsigned long long* keys, uint32_t* orders, int32_t* list,
                              int32_t* count, uint32_t* status, uint64_t key, uint32_t order) {
  uint32_t h = (uint32_t)mix64(key) & (kNewKeyCap - 1);
  for (int p = 0; p < 256; ++p) {
    // the CAS itself reads the slot (measured equal to a plain read first)
    const unsigned long long cur = atomicCAS(&keys[h], 0ull, (unsigned long long)key);
    if (cur == 0ull) {
      const int s = atomicAdd(count, 1);
      list[s] = (int32_t)h;
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
__device__ void nk_insert(const EngineDev& D, uint64_t key, uint32_t order) {
  keyset_insert(D.nk_key, D.nk_order, D.nk_list, &D.ctr->nk_count, &D.ctr->status, key, order);
}

// ---------------------------------------------------------------------------------------------
// k_ingest_dda: 16x16 pixel tile per workgroup.
//  1. pack the frame into per-pixel records the integrate kernel gathers:
//       pixA = {depth, range = |K^-1 [x y 1]|, w_new = (1 - d / max_depth) * 4, rgb}
//       pixB = log2 ht - log2 lt
//     (exactly the values tsdf_integrate_kernel recomputes per voxel, voxel_tsdf.cu:174-201)
//  2. DDA of [p - trunc dir, p + trunc dir] (voxel_tsdf.cu:116-146); block keys deduplicated in
//     an LDS hash set with their smallest candidate order (y*W + x)*maxs + i
//  3. each unique key once: all-8-corners visibility (is_block_visible<true>), table probe;
//     missing keys go to the global new-key set.
// Steps 2-3 run only for tiles in [P.tile_lo, P.tile_hi) (a sharded frame's pixel slice; every
// tile otherwise). A shard probes its copy of the whole hash index, so its keys are exactly the
// ones one volume's DDA finds in those tiles, whichever shard owns them.
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

// the two roles of k_ingest_dda share one LDS allocation
template <int TS>
union IngestLds {
  struct {
    unsigned long long key[TS];
    uint32_t ord[TS];
    uint16_t vis[4][TS / 4];
  } tile;
  struct {
    uint32_t list[4][kVisChunk];
    int cnt[kBands], base[kBands];
    int npass;
  } sweep;
};

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
template <int TS>
__device__ void vis_sweep(const EngineDev& D, const FrameParams& P, int wg, IngestLds<TS>& S) {
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t* L = S.sweep.list[wave];
  int* s_cnt = S.sweep.cnt;
  int* s_base = S.sweep.base;
  const int grp = lane >> 3, corner = lane & 7;
  const int w = wg * 256 + wave * 64 + lane;
  const unsigned long long occ_all = D.occ[w];
  const int cw = __popcll(occ_all);
  const int incl = wave_incl_scan(cw);
  const int excl = incl - cw;
  const int wave_total = __shfl(incl, 63, 64);
  if (threadIdx.x == 0) S.sweep.npass = 0;
  __syncthreads();
  if (lane == 0) atomicMax(&S.sweep.npass, (wave_total + kVisChunk - 1) / kVisChunk);
  __syncthreads();
  const int npass = S.sweep.npass;
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
        en = load_ent(D.table, e);
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
      const Ent en = load_ent(D.table, e);
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

// grid: kVisWorkgroups sweep workgroups first (dispatched first, they overlap the tiles), then
// one workgroup per 16x16 pixel tile (tiles_x per row, `tiles` in all)
template <int TS>
__device__ __forceinline__ void ingest_dda(EngineDev D, FrameParams P,
                                           const float* __restrict__ depth,
                                           const uint8_t* __restrict__ rgb,
                                           const float* __restrict__ ht,
                                           const float* __restrict__ lt, int tiles_x, int tiles) {
  __shared__ IngestLds<TS> S;
  if ((int)blockIdx.x < kVisWorkgroups) {
    TSDF_STAMP(D, 2, 0);
    vis_sweep(D, P, blockIdx.x, S);
    TSDF_STAMP(D, 2, 1);
    return;
  }
  const int tile = (int)blockIdx.x - kVisWorkgroups;
  if (tile >= tiles) return;
  unsigned long long* s_key = S.tile.key;
  uint32_t* s_ord = S.tile.ord;
  TSDF_STAMP(D, 0, 0);
  for (int i = threadIdx.x; i < TS; i += 256) {
    s_key[i] = 0ull;
    s_ord[i] = 0xFFFFFFFFu;
  }
  __syncthreads();
  TSDF_STAMP(D, 0, 1);
  const int x = (tile % tiles_x) * 16 + (threadIdx.x & 15);
  const int y = (tile / tiles_x) * 16 + (threadIdx.x >> 4);
  if (x < P.W && y < P.H) {
    const int i = y * P.W + x;
    const float d = depth[i];
    const uint32_t c = (uint32_t)rgb[3 * i] | ((uint32_t)rgb[3 * i + 1] << 8) |
                       ((uint32_t)rgb[3 * i + 2] << 16);
    const float h = ht ? ht[i] : 1.0f;
    const float l = lt ? lt[i] : 1.0f;
    const f3 pc = pixel_ray(P, x, y);
    const float range = sqrtf(dot3(pc, pc));  // img_depth_to_range (voxel_tsdf.cu:120)
    const float w_new = (1.0f - quot_const(d, P.max_depth, P.inv_max_depth)) * 4.0f;
    D.pixA[i] = make_float4(d, range, w_new, __uint_as_float(c));
    // base-2 log-odds of the pixel (k_integrate); the hardware log2 (1 ulp) is far inside the
    // 1e-4 prob tolerance and still gives exactly 0 when ht == lt
    D.pixB[i] = __log2f(h) - __log2f(l);
    TSDF_STAMP(D, 0, 2);
    if (tile >= P.tile_lo && tile < P.tile_hi && !(d == 0 || d > P.max_depth)) {
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
      f3 st;
      if (__builtin_expect(div <= 2.0f, 1)) {
        const float m = div == 2.0f ? 0.5f : 1.0f;
        st = {rg.x * m, rg.y * m, rg.z * m};
      } else {
        st = {rg.x / div, rg.y / div, rg.z / div};
      }
      f3 pos = sg;
      for (int s = 0; s <= step_grid; ++s) {
        if (s >= P.maxs) {
          atomicOr(&D.ctr->status, 4u);  // TSDF_STATUS_DDA_OVERFLOW
          break;
        }
        const int16_t kx = (int16_t)(f2s(roundf(pos.x)) >> kBlockLenBits);
        const int16_t ky = (int16_t)(f2s(roundf(pos.y)) >> kBlockLenBits);
        const int16_t kz = (int16_t)(f2s(roundf(pos.z)) >> kBlockLenBits);
        pos.x += st.x;
        pos.y += st.y;
        pos.z += st.z;
        const unsigned long long key = pack_key(kx, ky, kz);
        const uint32_t order = (uint32_t)i * (uint32_t)P.maxs + (uint32_t)s;
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
    }
  }
  TSDF_STAMP(D, 0, 3);
  __syncthreads();
  if (tile < P.tile_lo || tile >= P.tile_hi) return;  // pixel records only (workgroup-uniform)
  TSDF_STAMP(D, 0, 4);
  // Each wave sweeps its 64-slot strips; the few occupied slots of a strip (ballot) are tested
  // 8 at a time with 8 lanes per key, one block corner per lane (is_block_visible<true>), and the
  // fully visible ones are listed in LDS. The table probes and new-key inserts then run one key
  // per lane over that list, so the wave pays their memory latency once, not once per 8 keys.
  uint16_t(*s_vis)[TS / 4] = S.tile.vis;
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
  for (int i = lane; i < nv; i += 64) {
    const int slot = s_vis[wave][i];
    const unsigned long long key = s_key[slot];
    int16_t kx, ky, kz;
    unpack_key(key, kx, ky, kz);
    if (find_entry(D.table, kx, ky, kz) >= 0) continue;
    nk_insert(D, key, s_ord[slot]);
  }
  TSDF_STAMP(D, 0, 5);
}
template <int TS>
__global__ __launch_bounds__(256) void k_ingest_dda(EngineDev D, FrameParams P,
                                                    const float* __restrict__ depth,
                                                    const uint8_t* __restrict__ rgb,
                                                    const float* __restrict__ ht,
                                                    const float* __restrict__ lt, int tiles_x,
                                                    int tiles) {
  ingest_dda<TS>(D, P, depth, rgb, ht, lt, tiles_x, tiles);
}
template <int TS>
__global__ __launch_bounds__(256) void k_ingest_dda_g(EngineDev D, const FrameArgs* __restrict__ A) {
  const FrameParams P = A->P;
  ingest_dda<TS>(D, P, A->depth, A->rgb, A->ht, A->lt, A->tiles_x, A->tiles);
}
template __global__ void k_ingest_dda<1024>(EngineDev, FrameParams, const float*, const uint8_t*, const float*,
                                            const float*, int, int);
template __global__ void k_ingest_dda<2048>(EngineDev, FrameParams, const float*, const uint8_t*, const float*,
                                            const float*, int, int);
template __global__ void k_ingest_dda_g<1024>(EngineDev, const FrameArgs*);
template __global__ void k_ingest_dda_g<2048>(EngineDev, const FrameArgs*);

// ---------------------------------------------------------------------------------------------
// Sharded frames: the key exchange. k_key_pack drains this shard's new-key set
// (its DDA slice's keys) into its outbox slot; after the all-gather, k_key_merge inserts every
// shard's slot into the set with the smallest candidate order per key -- the set one volume's DDA
// over the whole frame builds -- so every shard's allocation resolver makes the same decisions.
// The senders probed the same index, so no probe is repeated here.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_key_pack(EngineDev D, ShardRec* __restrict__ out, int cap) {
  const int n = D.ctr->nk_count;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int h = D.nk_list[i];
    const unsigned long long key = D.nk_key[h];
    const uint32_t ord = D.nk_order[h];
    D.nk_key[h] = 0ull;  // the set is rebuilt from the exchanged slots
    D.nk_order[h] = 0xFFFFFFFFu;
    if (i < cap) {
      ShardRec r;
      unpack_key(key, r.x, r.y, r.z);
      r.pad = 0;
      r.val = ord;
      r.zero = 0u;
      out[1 + i] = r;
    }
  }
  __syncthreads();  // every wave has read nk_count before it is reset
  if (threadIdx.x == 0) {
    ShardRec h{};
    h.val = (uint32_t)min(n, cap);
    out[0] = h;
    if (n > cap) atomicOr(&D.ctr->status, 16u);  // TSDF_STATUS_SHARD_OVERFLOW
    D.ctr->nk_count = 0;
  }
}

// grid (ceil(cap / 256), nshard): workgroup row s merges the slot shard s wrote
__global__ __launch_bounds__(256) void k_key_merge(EngineDev D, const ShardRec* __restrict__ in, int cap) {
  const ShardRec* slot = in + (size_t)blockIdx.y * (cap + 1);
  const int n = min((int)slot[0].val, cap);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ShardRec r = slot[1 + i];
  nk_insert(D, pack_key(r.x, r.y, r.z), r.val);
}

// test path: keys[n] in list order (one VoxelHashTable::Allocate launch, voxel_hash_test.cu)
__global__ void k_keys_to_newset(EngineDev D, const int16_t* __restrict__ keys, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int16_t x = keys[3 * i], y = keys[3 * i + 1], z = keys[3 * i + 2];
    if (find_entry(D.table, x, y, z) >= 0) continue;
    nk_insert(D, pack_key(x, y, z), (uint32_t)i);
  }
}

// render replica import (tsdf_import_blocks): the records' block keys into the new-key set, in
// record order, for the resolver; keys already in the table are skipped
__global__ void k_import_keys(EngineDev D, const uint8_t* __restrict__ recs, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const short4 h = *reinterpret_cast<const short4*>(recs + (size_t)i * kBlockRecBytes);
    if (find_entry(D.table, h.x, h.y, h.z) >= 0) continue;
    nk_insert(D, pack_key(h.x, h.y, h.z), (uint32_t)i);
  }
}

// ---------------------------------------------------------------------------------------------
// k_resolve_alloc: one 1024-thread workgroup replays VoxelHashTable::Allocate in candidate order.
// Every unique missing key K is evaluated against the current table:
//   SLOT(B, s)   : an empty slot s of its bucket B                  -> takes lock B
//   APPEND(L, C) : bucket full -> tail T of B's list (bucket L = T/2), first empty slot-0 entry E
//                  after T (bucket C = E/2)                         -> takes lock L, then lock C
// A key's outcome depends on earlier keys only through the buckets it locks (every table write
// happens under those locks), so up to 1024 keys are evaluated speculatively, each claims its
// buckets in an LDS table (smallest rank wins), and the longest prefix whose keys won all their
// claims commits in parallel. The first key always wins, so each round commits >= 1 key.
// Pool blocks are popped in commit order by prefix sum (AquireBlock, voxel_mem.cu:37-52).
// frame_mode 1: append new blocks to this frame's visible-block lists flagged fresh (integrate
// initialises them), 0: list them in D.fresh for k_fresh_init.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void resolve_alloc(EngineDev D, FrameParams P, uint32_t range,
                                              int frame_mode) {
  __shared__ ResolveLds L;
  const int t = threadIdx.x;
  TSDF_STAMP(D, 1, 0);
  // the counters are loaded together (one memory round trip) before anything waits on them
  const int n = D.ctr->nk_count;
  const int free0 = D.ctr->free_count;  // every thread: the pops index the stack top by it
  uint32_t epoch0 = 0u;
  if (t == 0) epoch0 = D.ctr->lock_epoch;
  claims_clear(L);
  if (t == 0) {
    L.epoch = epoch0 + 1;
    D.ctr->lock_epoch = L.epoch;
    L.sfree = free0;
    L.nfresh = 0;
    L.nalloc = 0;
  }
  // One batch (the common case): (candidate order, list index) straight into the LDS batch, keys
  // and set slots into LDS, plus the free-stack top the pops will read -- all in one round trip.
  // Otherwise (order, slot) pairs go to a compact scratch array so every batch pass is one
  // coalesced read.
  const bool single = n <= kBatch;
  if (single) {
    for (int i = t; i < kLockSlots; i += kResolveThreads) L.lkey[i] = 0u;
    const int npre = min(n, free0);
    for (int i = t; i < npre; i += kResolveThreads) L.heap_top[i] = D.heap[free0 - 1 - i];
    for (int i = t; i < n; i += kResolveThreads) {
      const int h = D.nk_list[i];
      L.batch[i] = ((unsigned long long)D.nk_order[h] << 32) | (uint32_t)i;
      L.skey[i] = D.nk_key[h];
      L.sslot[i] = h;
    }
  } else {
    for (int i = t; i < n; i += kResolveThreads) {
      const int h = D.nk_list[i];
      D.pairs[i] = ((unsigned long long)D.nk_order[h] << 32) | (uint32_t)h;
      D.pkey[i] = D.nk_key[h];
    }
  }
  __syncthreads();
  auto keyf = [&](int i) -> uint32_t { return (uint32_t)(D.pairs[i] >> 32); };
  const int width = single ? 1 : stream_prepare(L, n, range, keyf);
  const int nbatch = single ? (n > 0 ? 1 : 0) : ((n - 1) >> 10) + 1;
  int rounds = 0;
  TSDF_STAMP(D, 1, 1);
  for (int j = 0; j < nbatch; ++j) {
    int m;
    if (single) {
      m = n;
      batch_sort(L, m, true);
    } else {
      m = stream_batch(L, n, width, j, keyf);
    }
    TSDF_STAMP(D, 1, 2);
    if (t == 0) L.base = 0;
    __syncthreads();
    while (L.base < m) {
      if (++rounds > n + 8) {  // unreachable: the first key of a round always commits
        if (t == 0) atomicOr(&D.ctr->status, 8u);
        j = nbatch;
        break;
      }
      const int base = L.base;
      const bool have = base + t < m;
      int kind = 0, slot = 0, h = -1;
      uint32_t B = 0, Lb = 0, C = 0, T = 0, E = 0;
      int16_t kx = 0, ky = 0, kz = 0;
      if (have) {
        const int li = (int)(L.batch[base + t] & 0xFFFFFFFFu);
        if (single) {
          h = L.sslot[li];
          unpack_key(L.skey[li], kx, ky, kz);
        } else {
          h = (int)(D.pairs[li] & 0xFFFFFFFFu);
          unpack_key(D.pkey[li], kx, ky, kz);
        }
        B = hash_block(kx, ky, kz);
        const Ent s0 = load_ent(D.table, 2 * B);
        const Ent s1 = load_ent(D.table, 2 * B + 1);
        if (s0.idx < 0) {
          kind = 1;
          slot = 0;
        } else if (s1.idx < 0) {
          kind = 1;
          slot = 1;
        } else {
          kind = 2;
          uint32_t last = 2 * B + 1;
          Ent b = s1;
          while (b.off) {
            last = (uint32_t)(last + (int32_t)b.off) & kEntryMask;
            b = load_ent(D.table, last);
          }
          T = last;
          Lb = T >> 1;
          uint32_t nx = T;
          for (uint32_t p = 0; p < kNumEntry; ++p) {
            nx = (nx + 1) & kEntryMask;
            if ((nx & 1u) == 0u && load_ent(D.table, nx).idx < 0) break;
          }
          E = nx;
          C = E >> 1;
        }
        if (kind == 1) {
          claim(L, B, (uint32_t)t);
        } else {
          claim(L, Lb, (uint32_t)t);
          claim(L, C, (uint32_t)t);
        }
      }
      if (t == 0) L.first_dirty = kResolveThreads;
      __syncthreads();
      if (have) {
        const bool clean = kind == 1 ? claim_winner(L, B) == (uint32_t)t
                                     : (claim_winner(L, Lb) == (uint32_t)t &&
                                        claim_winner(L, C) == (uint32_t)t);
        if (!clean) atomicMin(&L.first_dirty, t);
      }
      __syncthreads();
      const int first_dirty = L.first_dirty;
      const bool commit = have && t < first_dirty;
      bool ok = false;
      if (commit && single) {  // the launch's locks in LDS (<= 2 x 2048 of the 8192 slots)
        if (kind == 1)
          ok = lock_take(L, B);
        else if (lock_take(L, Lb))
          ok = lock_take(L, C);
      } else if (commit) {
        const uint32_t ep = L.epoch;
        if (kind == 1) {
          if (D.lock_tag[B] != ep) {
            D.lock_tag[B] = ep;
            ok = true;
          }
        } else if (D.lock_tag[Lb] != ep) {
          D.lock_tag[Lb] = ep;
          if (D.lock_tag[C] != ep) {
            D.lock_tag[C] = ep;
            ok = true;
          }
        }
      }
      // Sharded volume: every shard commits every key's table change (the replicated index), and
      // only the key's owner pops a pool block; the others store kForeignIdx.
      const bool mine = ok && (P.shard_count <= 1 ||
                               brick_owner(kx, ky, kz, (uint32_t)P.shard_count) == (uint32_t)P.shard_index);
      int nok;
      const int rank = block_excl_scan(mine ? 1 : 0, L.scan, &nok);
      const int free_now = L.sfree;
      if (ok) {
        int32_t idx = kForeignIdx;
        bool insert = true;
        if (mine) {
          const int hi = free_now - 1 - rank;
          if (hi < 0) {
            atomicOr(&D.ctr->status, 1u);  // TSDF_STATUS_POOL_EXHAUSTED
            // one volume drops the insert; a shard keeps a voxel-less entry so that every
            // shard's index stays the same
            insert = P.shard_count > 1;
          } else {
            const int top = free0 - 1 - hi;  // pops so far this launch + rank
            idx = single ? L.heap_top[top] : D.heap[hi];
          }
        }
        if (insert) {
          uint32_t e;
          if (kind == 1) {
            e = 2 * B + (uint32_t)slot;
          } else {
            const uint32_t wrap = E > T ? 0u : kNumEntry;
            store_off(D.table, T, (int16_t)(E + wrap - T));
            e = E;
          }
          store_ent(D.table, e, kx, ky, kz, 0, idx);
          if (local_idx(idx)) {  // the occupancy bitmap lists the blocks this engine holds
            atomicOr(&D.occ[e >> 6], 1ull << (e & 63));
            if (frame_mode) {
              // a new block has all 8 corners in view, so it is visible this frame: listed for
              // the fresh-block integrate launch (the sweep in k_ingest_dda listed only the
              // blocks that existed before), flagged fresh so it starts from AquireBlock's state
              VisRec vr;
              vr.x = kx;
              vr.y = ky;
              vr.z = kz;
              vr.pad = 1;
              vr.idx = idx;
              vr.entry = (int32_t)e;
              D.fresh_vis[L.nfresh + rank] = vr;
            } else {
              D.fresh[L.nfresh + rank] = idx;
            }
          }
        }
      }
      if (commit) {
        D.nk_key[h] = 0ull;
        D.nk_order[h] = 0xFFFFFFFFu;
      }
      claims_clear(L);
      __syncthreads();
      if (t == 0) {
        const int used = nok < free_now ? nok : (free_now > 0 ? free_now : 0);
        L.sfree = free_now - used;
        L.nfresh += used;
        L.nalloc += used;
        const int span = m - base < kResolveThreads ? m - base : kResolveThreads;
        L.base = base + (first_dirty < span ? first_dirty : span);
      }
      __syncthreads();
    }
  }
  TSDF_STAMP(D, 1, 3);
  __syncthreads();  // every thread's table / list writes precede the release below
  if (t == 0) {
    D.ctr->free_count = L.sfree;
    D.ctr->n_fresh = L.nfresh;
    D.ctr->nk_count = 0;
    if (frame_mode) {
      D.ctr->last_alloc = L.nalloc;
      D.ctr->last_new_keys = n;
      D.ctr->total_alloc += (unsigned long long)L.nalloc;
    }
  }
}

__global__ __launch_bounds__(kResolveThreads) void k_resolve_alloc(EngineDev D, FrameParams P,
                                                                   uint32_t range, int frame_mode) {
  resolve_alloc(D, P, range, frame_mode);
}
__global__ __launch_bounds__(kResolveThreads) void k_resolve_alloc_g(EngineDev D,
                                                                     const FrameArgs* __restrict__ A) {
  const FrameParams P = A->P;
  resolve_alloc(D, P, A->range, 1);
}

// AquireBlock's initialisation (voxel_mem.cu:43-51) for the hash-level test path
__global__ __launch_bounds__(256) void k_fresh_init(EngineDev D) {
  const int n = D.ctr->n_fresh;
  const int quads = n * (kBlockVolume / 4);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += gridDim.x * blockDim.x) {
    const int b = q >> 7, v = (q & 127) * 4;
    uint8_t* blk = D.pool + (size_t)D.fresh[b] * kBlockBytes;
    *reinterpret_cast<float4*>(blk + v * 4) = make_float4(-1.f, -1.f, -1.f, -1.f);
    *reinterpret_cast<float4*>(blk + kProbOffset + v * 4) = make_float4(0.f, 0.f, 0.f, 0.f);  // p = 0.5
    // weight 0; the colour of a weight-0 voxel is defined as 0 (see k_integrate / the oracle)
    *reinterpret_cast<uint4*>(blk + kRgbwOffset + v * 4) = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace tsdf
