// tsdf_alloc.hip -- block allocation: frame ingest + DDA, and the in-order allocation resolver.
//
// Reference: TSDFGrid::Allocate (utils/tsdf/voxel_tsdf.cu:377-386) launching block_allocate_kernel
// (:104-147), which calls VoxelHashTable::Allocate (voxel_hash.cu:58-120) from every pixel
// thread. That insert is racy by design (one structural change per bucket per launch, losers
// dropped); this engine replays the canonical sequential linearisation:
// candidates in pixel raster order then DDA step, with the exact bucket-lock semantics.
#include "tsdf_block.h"
#include "tsdf_kernels.h"
#include "tsdf_resolve.h"
#include "tsdf_ingest.h"

namespace tsdf {

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
  uint32_t* L = S.u.sweep.list[wave];
  int* s_cnt = S.u.sweep.cnt;
  int* s_base = S.u.sweep.base;
  const int grp = lane >> 3, corner = lane & 7;
  const int w = wg * 256 + wave * 64 + lane;
  const unsigned long long occ_all = D.occ[w];
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

// a shard's split frame: the new-key set (this slice's keys) into the exchange slot, drained for
// the merge of every shard's slots (k_resolve_alloc after the all-gather)
__device__ void pack_keys_wg(const EngineDev& D, ShardRec* __restrict__ out, int cap) {
  const int n = ld_co(&D.ctr->nk_count);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int h = (int)ld_co(&D.nk_list[i].slot);
    const unsigned long long key = ld_co(&D.nk_list[i].key);
    const uint32_t ord = ld_co(&D.nk_order[h]);
    D.nk_key[h] = 0ull;
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
  __syncthreads();  // every thread has read nk_count before it is reset
  if (threadIdx.x == 0) {
    ShardRec h{};
    h.val = (uint32_t)min(n, cap);
    out[0] = h;
    if (n > cap) atomicOr(&D.ctr->status, 16u);  // TSDF_STATUS_SHARD_OVERFLOW
    D.ctr->nk_count = 0;
  }
}

// grid: kVisWorkgroups sweep workgroups first (dispatched first, they overlap the tiles), then one
// workgroup per 16x16 pixel tile (tiles_x per row, `tiles` in all). Every workgroup arrives at the
// end; the last one resolves the frame's allocation (kTailResolve) or packs a shard's keys for the
// exchange (kTailPack): block_allocate_kernel and VoxelHashTable::Allocate's launch in one.
template <int TS>
__device__ __forceinline__ void ingest_dda(EngineDev D, FrameParams P,
                                           const float* __restrict__ depth,
                                           const uint8_t* __restrict__ rgb,
                                           const float* __restrict__ ht,
                                           const float* __restrict__ lt, int tiles_x, int tiles) {
  __shared__ IngestLds<TS> S;
  // device-clock span of the ingest (WG 0 is dispatched first; the end is the last arrival)
  if (blockIdx.x == 0 && threadIdx.x == 0)
    st_co(&D.arrive[kArrStart + 8], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  if ((int)blockIdx.x < kVisWorkgroups) {
    TSDF_STAMP(D, 2, 0);
    vis_sweep(D, P, blockIdx.x, S);
    TSDF_STAMP(D, 2, 1);
  } else if ((int)blockIdx.x - kVisWorkgroups < tiles) {  // tiles [P.tile_lo, P.tile_lo + tiles)
    const int tile = P.tile_lo + (int)blockIdx.x - kVisWorkgroups;
    if (P.prepared)
      ingest_tile<TS, kTileProbe>(D, P, depth, rgb, ht, lt, tiles_x, tile, S);
    else
      ingest_tile<TS, kTileFull>(D, P, depth, rgb, ht, lt, tiles_x, tile, S);
  }
  if (!arrive_last(D.arrive + kArrIngest, 0ull, &S.last)) return;
  const unsigned long long tend = __builtin_amdgcn_s_memrealtime();
  TSDF_STAMP(D, 6, 0);
  if (threadIdx.x == 0) arrive_reset(D.arrive + kArrIngest);  // (no loads: the resolver starts at once)
  if (P.tail == kTailPack)
    pack_keys_wg(D, P.slot, P.slot_cap);
  else
    resolve_alloc_wg(D, P, (uint32_t)P.W * (uint32_t)P.H * (uint32_t)P.maxs, 1, S.u.res);
  // the ingest's device span (start -> last arrival), accounted after the resolver, off its path
  TSDF_STAMP(D, 6, 1);
  if (threadIdx.x == 0) D.ctr->ingest_ticks += tend - ld_co(&D.arrive[kArrStart + 8]);
  TSDF_STAMP(D, 6, 2);
}
// at least 6 waves per SIMD (<= 80 VGPRs): the whole 640x480 grid (1456 workgroups) resident at once;
// the resolver tail alone would raise the kernel to 81 VGPRs (5 waves: 1280 workgroups, +2 us span)
template <int TS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TS <= 1024 ? 6 : 5))) void k_ingest_dda(EngineDev D, FrameParams P,
                                                    const float* __restrict__ depth,
                                                    const uint8_t* __restrict__ rgb,
                                                    const float* __restrict__ ht,
                                                    const float* __restrict__ lt, int tiles_x,
                                                    int tiles) {
  ingest_dda<TS>(D, P, depth, rgb, ht, lt, tiles_x, tiles);
}
template <int TS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TS <= 1024 ? 6 : 5))) void k_ingest_dda_g(EngineDev D, const FrameArgs* __restrict__ A) {
  const FrameParams P = A->P;
  ingest_dda<TS>(D, P, A->depth, A->rgb, A->ht, A->lt, A->tiles_x, A->tiles);
}
template __global__ void k_ingest_dda<1024>(EngineDev, FrameParams, const float*, const uint8_t*, const float*,
                                            const float*, int, int);
template __global__ void k_ingest_dda<2048>(EngineDev, FrameParams, const float*, const uint8_t*, const float*,
                                            const float*, int, int);
template __global__ void k_ingest_dda_g<1024>(EngineDev, const FrameArgs*);
template __global__ void k_ingest_dda_g<2048>(EngineDev, const FrameArgs*);

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
// k_resolve_alloc: the allocation resolver (tsdf_resolve.h) as its own one-workgroup launch -- a
// shard's split frame after the key all-gather (keys_in: every shard's slot, merged into the
// new-key set first with the smallest candidate order per key, the set one volume's DDA over the
// whole frame builds; the senders probed the same index, so no probe is repeated), and the
// hash-level test / import path (frame_mode 0).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void resolve_alloc_merged(EngineDev D, const FrameParams& P, uint32_t range,
                                                     int frame_mode, const ShardRec* __restrict__ keys_in,
                                                     int cap, int nshard) {
  __shared__ AllocLdsT<kIngestRB> L;
  if (keys_in) {
    for (int s = 0; s < nshard; ++s) {
      const ShardRec* slot = keys_in + (size_t)s * (cap + 1);
      const int n = min((int)slot[0].val, cap);
      for (int i = threadIdx.x; i < n; i += kRT) {
        const ShardRec r = slot[1 + i];
        nk_insert(D, pack_key(r.x, r.y, r.z), r.val);
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  resolve_alloc_wg(D, P, range, frame_mode, L);
}
__global__ __launch_bounds__(kRT) void k_resolve_alloc(EngineDev D, FrameParams P, uint32_t range,
                                                       int frame_mode, const ShardRec* __restrict__ keys_in,
                                                       int cap, int nshard) {
  resolve_alloc_merged(D, P, range, frame_mode, keys_in, cap, nshard);
}
__global__ __launch_bounds__(kRT) void k_resolve_alloc_g(EngineDev D, const FrameArgs* __restrict__ A) {
  const FrameParams P = A->P;
  resolve_alloc_merged(D, P, A->range, 1, A->keys_in, A->key_cap, A->nshard);
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
