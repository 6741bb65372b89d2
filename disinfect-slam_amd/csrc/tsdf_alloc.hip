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
#include "tsdf_raycast.h"

namespace tsdf {

// a shard's split frame: the new-key set (this slice's keys) into the exchange slot, drained for
// the merge of every shard's slots (k_resolve_alloc after the all-gather)
__device__ __forceinline__ void pack_keys_wg(const EngineDev& D, ShardRec* __restrict__ out, int cap) {
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
// wg / nwg: this workgroup among the ingest's (its own launch: the block index and the grid; the
// fused render + ingest launch: past the raycast's workgroups)
template <int TS>
__device__ __forceinline__ void ingest_dda(EngineDev D, FrameParams P,
                                           const float* __restrict__ depth,
                                           const uint8_t* __restrict__ rgb,
                                           const float* __restrict__ ht,
                                           const float* __restrict__ lt, int tiles_x, int tiles,
                                           IngestLds<TS>& S, int wg, int nwg) {
  // device-clock span of the ingest (WG 0 is dispatched first; the end is the last arrival)
  if (wg == 0 && threadIdx.x == 0)
    st_co(&D.arrive[kArrStart + 8], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  if (wg < kVisWorkgroups) {
    TSDF_STAMP(D, 2, 0);
    vis_sweep(D, P, wg, S);
    TSDF_STAMP(D, 2, 1);
  } else if (wg - kVisWorkgroups < tiles) {  // tiles [P.tile_lo, P.tile_lo + tiles)
    ingest_tile<TS, kTileFull>(D, P, depth, rgb, ht, lt, tiles_x, P.tile_lo + wg - kVisWorkgroups, S);
  }
  if (!arrive_last(D.arrive + kArrIngest, 0ull, &S.last, true, (uint32_t)nwg, (uint32_t)wg)) return;
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
// k_ingest_dda at 8 waves per SIMD (<= 64 VGPRs): 2048 resident workgroups, so a 1280x720 frame's 3,856
// take 1.9 rounds instead of 2.5. Measured at C4 (300 frames, same box, interleaved): ingest span
// 24.6 -> 23.1 us, the tail's resolver 3.35 -> 4.45 us (a few spills), 16.85k -> 17.02k frames/s;
// 7 waves 16.91k. At 640x480 every tile is resident at 6 waves (1456 workgroups) already. The fused
// render + ingest launch keeps 6 (<= 80 VGPRs; its raycast part is register-hungry).
#ifndef TSDF_INGEST_MIN_WAVES
#define TSDF_INGEST_MIN_WAVES 8
#endif
#define INGEST_WAVES(TS) __attribute__((amdgpu_waves_per_eu(TS <= 1024 ? TSDF_INGEST_MIN_WAVES : 5)))
#ifndef TSDF_RENDER_INGEST_WAVES
#define TSDF_RENDER_INGEST_WAVES 6
#endif
#define RENDER_INGEST_WAVES __attribute__((amdgpu_waves_per_eu(TSDF_RENDER_INGEST_WAVES)))
template <int TS>
__global__ __launch_bounds__(256) INGEST_WAVES(TS) void k_ingest_dda(EngineDev D, FrameParams P,
                                                    const float* __restrict__ depth,
                                                    const uint8_t* __restrict__ rgb,
                                                    const float* __restrict__ ht,
                                                    const float* __restrict__ lt, int tiles_x,
                                                    int tiles) {
  __shared__ IngestLds<TS> S;
  ingest_dda<TS>(D, P, depth, rgb, ht, lt, tiles_x, tiles, S, (int)blockIdx.x, (int)gridDim.x);
}
template <int TS>
__global__ __launch_bounds__(256) INGEST_WAVES(TS) void k_ingest_dda_g(EngineDev D, const FrameArgs* __restrict__ A) {
  __shared__ IngestLds<TS> S;
  const FrameParams P = A->P;
  ingest_dda<TS>(D, P, A->depth, A->rgb, A->ht, A->lt, A->tiles_x, A->tiles, S, (int)blockIdx.x, (int)gridDim.x);
}

// ---------------------------------------------------------------------------------------------
// k_render_ingest: frame n's raycast (its view grid built before the launch) and frame n + 1's ingest
// (k_ingest_dda: pixel records, DDA, probes, visibility sweep, the allocation in its last arriver) in
// one launch. With a view grid the raycast reads only the grid, its bitmaps and the pool; the ingest
// writes none of them (it writes the table, the occupancy bitmap, the new-key set, the pixel records
// and frame n + 1's lists; the blocks it allocates are written by frame n + 1's update, a later
// launch). So the two are independent and the ingest's workgroups fill the slots the latency-bound
// raycast leaves (tsdf_raycast_deferred). The raycast's workgroups come first in the grid.
// ---------------------------------------------------------------------------------------------
union RenderIngestLds {
  IngestLds<1024> ing;
  uint32_t bits[kViewGraphBitmapWords];  // the raycast's staged bitmaps
};
__global__ __launch_bounds__(256) RENDER_INGEST_WAVES TSDF_RAY_PK void k_render_ingest(
    EngineDev D, FrameParams R, float step_size, ViewGrid V, uchar4* __restrict__ rgba, uchar4* __restrict__ normal,
    int rgx, int nray, FrameParams P, const float* __restrict__ depth, const uint8_t* __restrict__ rgb,
    const float* __restrict__ ht, const float* __restrict__ lt, int tiles_x, int tiles) {
  __shared__ RenderIngestLds U;
  const int b = (int)blockIdx.x;
  if (b < nray) {
    raycast(D, R, step_size, V, U.bits, rgba, normal, b, rgx, nray);
    return;
  }
  ingest_dda<1024>(D, P, depth, rgb, ht, lt, tiles_x, tiles, U.ing, b - nray, (int)gridDim.x - nray);
}
__global__ __launch_bounds__(256) RENDER_INGEST_WAVES TSDF_RAY_PK void k_render_ingest_g(EngineDev D,
                                                                            const FrameArgs* __restrict__ A,
                                                                            int rgx, int nray) {
  __shared__ RenderIngestLds U;
  const int b = (int)blockIdx.x;
  if (b < nray) {
    const FrameArgs* Q = A->prev;
    if (!Q) return;
    const FrameParams R = Q->R;
    const ViewGrid V = Q->V;
    raycast(D, R, Q->step_size, V, U.bits, Q->rgba, Q->normal, b, rgx, nray);
    return;
  }
  const FrameParams P = A->P;
  ingest_dda<1024>(D, P, A->depth, A->rgb, A->ht, A->lt, A->tiles_x, A->tiles, U.ing, b - nray,
                   (int)gridDim.x - nray);
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
    *reinterpret_cast<float4*>(blk + kProbOffset + v * 4) = make_float4(0.5f, 0.5f, 0.5f, 0.5f);  // p = 0.5
    // weight 0; the colour of a weight-0 voxel is defined as 0 (see k_integrate / the oracle)
    *reinterpret_cast<uint4*>(blk + kRgbwOffset + v * 4) = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace tsdf
