// tsdf_fuse.hip -- the fused integrate kernel and the space-carving resolver.
#include "tsdf_block.h"
#include "tsdf_kernels.h"
#include "tsdf_resolve.h"
#include "tsdf_ingest.h"

namespace tsdf {

// ---------------------------------------------------------------------------------------------
// k_integrate: tsdf_integrate_kernel (voxel_tsdf.cu:149-205) + the space_carving_kernel minimum
// (:207-230) fused. Two waves per visible 8^3 block, 4 voxels per lane: lane l of wave half h owns
// voxels v = 256h + 4l .. +3 (x = 4(l&1)+j, y = (l>>1)&7, z = l>>4 + 4h), so each of the three
// state arrays moves as one 16-B-per-lane, 1-KiB-per-wave access inside the block's contiguous
// 6-KiB record. Pixel data is two gathers per voxel (16 B + 4 B, L2 resident). Blocks allocated
// this frame (VisRec.pad, set by the allocation resolver) start from AquireBlock's state
// (voxel_mem.cu:43-51) in registers.
// Carve candidates (min |tsdf| >= 0.9) are appended with their hash-entry index.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float comp(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
__device__ __forceinline__ void setc(float4& v, int j, float f) {
  if (j == 0) v.x = f; else if (j == 1) v.y = f; else if (j == 2) v.z = f; else v.w = f;
}
__device__ __forceinline__ uint32_t compu(const uint4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
__device__ __forceinline__ void setu(uint4& v, int j, uint32_t f) {
  if (j == 0) v.x = f; else if (j == 1) v.y = f; else if (j == 2) v.z = f; else v.w = f;
}

// end of a frame's bookkeeping (after its carving): running totals, empty candidate / band lists
__device__ void frame_end(const EngineDev& D) {
  lds_barrier();
  if (threadIdx.x == 0) {
    D.ctr->total_visible += (unsigned long long)D.ctr->n_vis;
    D.ctr->total_updated += D.ctr->last_updated;
    D.ctr->frames += 1ull;
    D.ctr->n_cand = 0;  // the next frame's lists start empty (its sweep runs before allocation)
    D.ctr->n_pend = 0;
  }
  if (threadIdx.x < kBands) st_co(&D.band[threadIdx.x * kBandStride], 0);  // (written through: see k_integrate_pre)
}

// a shard's frame: its carve candidates into the exchange slot, then the owned entries its
// exhausted pool left without voxels this frame (D.pend, written by the allocation resolver before
// this launch)
__device__ void pack_cands_wg(const EngineDev& D, ShardRec* __restrict__ out, int cap) {
  const int nc = ld_co(&D.ctr->n_cand);
  const int np = min(D.ctr->n_pend, (int)kNewKeyCap);
  const int n = nc + np;
  const unsigned long long* rq = reinterpret_cast<const unsigned long long*>(D.cand);
  for (int i = threadIdx.x; i < min(n, cap); i += blockDim.x) {
    unsigned long long a, b;
    if (i < nc) {
      a = ld_co(&rq[2 * i]);
      b = ld_co(&rq[2 * i + 1]);
    } else {
      const unsigned long long* pq = reinterpret_cast<const unsigned long long*>(D.pend + (i - nc));
      a = pq[0];
      b = pq[1];
    }
    ShardRec r;
    r.x = (int16_t)(a & 0xFFFF);
    r.y = (int16_t)((a >> 16) & 0xFFFF);
    r.z = (int16_t)((a >> 32) & 0xFFFF);
    r.pad = 0;
    r.val = (uint32_t)(b >> 32);  // hash entry
    r.zero = 0u;
    out[1 + i] = r;
  }
  if (threadIdx.x == 0) {
    ShardRec h{};
    h.val = (uint32_t)min(n, cap);
    out[0] = h;
    if (n > cap) atomicOr(&D.ctr->status, 16u);  // TSDF_STATUS_SHARD_OVERFLOW
  }
}

// tsdf_integrate_shard_abort (one workgroup): the per-frame state of a sharded frame that will not
// complete back to "between frames" -- the new-key set (slots listed in the new-key list), the
// visible-band counts, candidate / fresh / pending counts and the arrival counters. Structural
// changes a phase already committed stay (TSDF_STATUS_SHARD_ABORTED tells the caller the shards may
// differ: restore a snapshot).
__global__ __launch_bounds__(256) void k_shard_abort(EngineDev D) {
  const int n = min(D.ctr->nk_count, (int)kNewKeyCap);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int h = (int)D.nk_list[i].slot;
    D.nk_key[h] = 0ull;
    D.nk_order[h] = 0xFFFFFFFFu;
  }
  if (threadIdx.x < kBands) D.band[threadIdx.x * kBandStride] = 0;
  for (int i = threadIdx.x; i < kArriveWords; i += blockDim.x) D.arrive[i] = 0ull;
  __syncthreads();
  if (threadIdx.x == 0) {
    D.ctr->nk_count = 0;
    D.ctr->n_cand = 0;
    D.ctr->n_fresh = 0;
    D.ctr->n_pend = 0;
    D.ctr->status |= 32u;  // TSDF_STATUS_SHARD_ABORTED
  }
}

// The last-arriving workgroup of k_integrate: the frame's statistics (updated voxels from the
// arrivals, the update's device-clock span, visible = listed by the sweep + created), then the
// space carving of the candidates (voxel_tsdf.cu:483-488, kTailResolve) or, in a shard's frame,
// the packing of its candidates for the exchange (kTailPack; k_resolve_delete follows it).
// The statistics (their loads) come after the carving, off its path.
// Pre (k_integrate_pre): only the carving and the band-count reset the next frame's chained sweep
// waits for; the statistics follow once the carving is published (integrate_stats), off the frame's
// path. The band counts are read before the carving (they are final since the previous launch).
__device__ __forceinline__ void integrate_stats(const EngineDev& D, DeleteLds& L) {
  const int t = threadIdx.x;
  lds_barrier();
  const int bc = t < kBands ? L.bcnt[t] : 0;
  int nband;
  (void)wg_excl_scan(bc, L.scan, &nband);
  if (t == 0) {
    const unsigned long long upd = arrive_collect(D.arrive + kArrIntegrate);
    const int nvis = nband + D.ctr->n_fresh;
    D.ctr->last_updated = upd;
    D.ctr->integrate_ticks += L.tend - ld_co(&D.arrive[kArrStart]);
    D.ctr->n_vis = nvis;
    D.ctr->total_visible += (unsigned long long)nvis;
    D.ctr->total_updated += upd;
    D.ctr->frames += 1ull;
  }
}

template <bool Pre = false>
__device__ __forceinline__ void integrate_tail(const EngineDev& D, const FrameParams& P, DeleteLds& L) {
  const int t = threadIdx.x;
  const unsigned long long tend = __builtin_amdgcn_s_memrealtime();  // the update's span ends here
  TSDF_STAMP(D, 7, 0);
  const int bc_pre = Pre && t < kBands ? D.band[t * kBandStride] : 0;
  if (P.tail == kTailPack)
    pack_cands_wg(D, P.slot, P.slot_cap);
  else
    resolve_delete_wg(D, D.cand, &D.ctr->n_cand, 0, L);
  TSDF_STAMP(D, 7, 1);
  if (Pre) {
    lds_barrier();
    if (t < kBands) {
      L.bcnt[t] = bc_pre;
      st_co(&D.band[t * kBandStride], 0);  // (written through: see k_integrate_pre)
    }
    if (t == 0) {  // (written through: the allocation resolver later in this launch adds to n_pend)
      L.tend = tend;
      st_co(&D.ctr->n_cand, 0);
      st_co(&D.ctr->n_pend, 0);
    }
    return;
  }
  lds_barrier();  // (L.scan is reused below)
  const int bc = t < kBands ? D.band[t * kBandStride] : 0;
  int nband;
  (void)wg_excl_scan(bc, L.scan, &nband);
  if (t == 0) {
    const unsigned long long upd = arrive_collect(D.arrive + kArrIntegrate);
    D.ctr->last_updated = upd;
    D.ctr->integrate_ticks += tend - ld_co(&D.arrive[kArrStart]);
    D.ctr->n_vis = nband + D.ctr->n_fresh;
  }
  if (P.tail != kTailPack) frame_end(D);
  TSDF_STAMP(D, 7, 2);
}

// 64 VGPRs: 8 waves per SIMD (65 without the bound: 7). Graph: the graph-captured form reads its
// camera from the FrameArgs block the graph's first node uploads.
// The visible blocks are the sweep's band lists (blocks that existed before the frame) followed by
// the blocks k_resolve_alloc created (D.fresh_vis, flagged fresh).
// Raw: a shard's frame -- the pixel terms come from the raw frame (depth, rgb, ht, lt gathers) and
// are computed per voxel with the ingest's operations (pixel_w_new, pixel_logodds, the range of
// pixel_ray), instead of from pixel records packed for the whole frame.
#ifndef TSDF_INTEGRATE_WAVES
#define TSDF_INTEGRATE_WAVES 7
#endif
// nint: the update's workgroups (blocks [0, nint) of the launch; k_integrate_pre appends the next
// frame's pixel-tile workgroups after them). L: the LDS of the last arriver's carving resolve.
// returns true in the workgroup that arrived last (and ran the carving tail)
template <bool Graph, bool Raw, bool Pre = false>
__device__ __forceinline__ bool integrate_body(const EngineDev& D, const FrameParams& Pv,
                                               const FrameArgs* __restrict__ A, int nint, DeleteLds& L) {
  FrameParams P = Graph ? A->P : Pv;
  if (Graph && A->cands_out) {  // a shard's graph frame: the tail packs the carve candidates
    P.tail = kTailPack;
    P.slot = A->cands_out;
    P.slot_cap = A->cand_cap;
  } else if (Graph) {
    P.tail = kTailResolve;
  }
  __shared__ float s_min[4];
  __shared__ int s_upd[4];
  __shared__ int s_last;
  __shared__ int s_ncand, s_ovf;
  __shared__ VisRec s_cand[kIntegrateCandBuf];  // this workgroup's carve candidates
  const int lane = lane_id();
  // wave-uniform (scalar) loop state: the band search, the list record and the fresh flag are
  // SALU / scalar loads instead of per-lane selects
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave >> 1, hf = wave & 1;
  // concatenated band lists: band i holds visible-block indices [bstart_i, bstart_i + count_i)
  int bstart[kBands];
  int nvis = 0;
#pragma unroll
  for (int i = 0; i < kBands; ++i) {
    bstart[i] = nvis;
    nvis += D.band[i * kBandStride];
  }
  const int nband = nvis;
  nvis += D.ctr->n_fresh;
  const int g = blockIdx.x & 7, ngrp = nint >> 3;
  const int rx0 = (lane & 1) * 4, ry = (lane >> 1) & 7, rz = (lane >> 4) + 4 * hf;
  const int off = (hf * 256 + lane * 4) * 4;
  const float neg_trunc = -P.trunc;
  int my_upd = 0;
  if (threadIdx.x == 0) {  // (ordered before their first use by the pair loop's barrier)
    s_ncand = 0;
    s_ovf = 0;
  }
  TSDF_STAMP(D, 3, 0);
  // device-clock duration of the update: start stamp by WG 0 (dispatched first), end = the last
  // workgroup's arrival (bench cross-check of the HIP-event timing)
  if (blockIdx.x == 0 && threadIdx.x == 0) st_co(&D.arrive[kArrStart], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  // XCD-aware split (workgroups b and b + 8 share an XCD): group g = blockIdx % 8 takes the g-th
  // contiguous eighth of the block pairs in band order, a compact image region whose pixel
  // records stay resident in that XCD's L2.
  const int npairs = (nvis + 1) >> 1;
  const int p_lo = (int)(((long long)npairs * g) >> 3), p_hi = (int)(((long long)npairs * (g + 1)) >> 3);
  for (int pp = p_lo + (blockIdx.x >> 3); pp < p_hi; pp += ngrp) {
    const int b = 2 * pp + pair;
    float mn = __builtin_inff();
    bool fresh = false;
    int32_t pidx = 0;
    VisRec r{};
    if (b < nvis) {
      if (b >= nband) {
        r = D.fresh_vis[b - nband];
      } else {
        int bd = 0, ofs = b;
#pragma unroll
        for (int i = 1; i < kBands; ++i)
          if (b >= bstart[i]) {
            bd = i;
            ofs = b - bstart[i];
          }
        r = D.vis[(size_t)bd * D.nblocks + __builtin_amdgcn_readfirstlane(ofs)];
      }
      pidx = r.idx;
      uint8_t* blk = D.pool + (size_t)pidx * kBlockBytes;
#if defined(TSDF_EXP) && (TSDF_EXP & 2)  // experiment build: no pool state loads
      float4 ts = make_float4(0.5f, 0.5f, 0.5f, 0.5f), pr = ts;
      uint4 cw = make_uint4(0x05808080u, 0x05808080u, 0x05808080u, 0x05808080u);
#else
      float4 ts, pr;
      uint4 cw;
      fresh = r.pad != 0;
      if (fresh) {  // wave-uniform: a block created this frame loads nothing
        ts = make_float4(-1.f, -1.f, -1.f, -1.f);
        pr = make_float4(0.f, 0.f, 0.f, 0.f);  // log-odds of AquireBlock's p = 0.5
        // weight 0; AquireBlock leaves rgb as it was (voxel_mem.cu:43-51): uninitialised memory
        // or a previous block's colour, i.e. unspecified, visible only on weight-0 voxels. It is
        // defined as 0 here and in the oracle (a sharded volume's pool indices differ).
        cw = make_uint4(0u, 0u, 0u, 0u);
      } else {
        ts = pool_ld(blk + off);
        pr = pool_ld(blk + kProbOffset + off);
        cw = pool_ldu(blk + kRgbwOffset + off);
      }
#endif
#if defined(TSDF_EXP) && (TSDF_EXP & 2)
      fresh = r.pad != 0;
#endif
      const int16_t ax0 = (int16_t)(r.x << kBlockLenBits), ay = (int16_t)((r.y << kBlockLenBits) + ry),
                    az = (int16_t)((r.z << kBlockLenBits) + rz);
      const float fy = (float)ay * P.voxel, fz = (float)az * P.voxel;
      int upd_mask = 0;
      // ---- pass 1: project the lane's 4 voxels (two packed pairs) and issue every pixel gather
      // before any is consumed (predicated, so all 8 stay in flight together).
      // cam_T_world * (x voxel, fy, fz) in QuaternionBase::_transformVector's exact order, with the
      // parts that do not depend on x computed once per lane (identical operations, so identical
      // results to se3_apply per voxel).
      const float qx = P.cq.x, qy = P.cq.y, qz = P.cq.z, qw = P.cq.w;
      const float qx_fz = qx * fz, qx_fy = qx * fy;
      float uvx = qy * fz - qz * fy;
      uvx += uvx;
      const float w_uvx = qw * uvx, qz_uvx = qz * uvx, qy_uvx = qy * uvx;
      v2f hzs[2];
      float4 px[4];
      float lg[4];
      bool inb[4];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const v2f wx = v2((float)(int16_t)(ax0 + rx0 + 2 * k), (float)(int16_t)(ax0 + rx0 + 2 * k + 1)) * P.voxel;
        v2f uvy = qz * wx - qx_fz;
        v2f uvz = qx_fy - qy * wx;
        uvy += uvy;
        uvz += uvz;
        const v2f cx = qy * uvz - qz * uvy;
        const v2f cy = qz_uvx - qx * uvz;
        const v2f cz = qx * uvy - qy_uvx;
        const v2f pcx = ((wx + w_uvx) + cx) + P.ct.x;
        const v2f pcy = ((fy + qw * uvy) + cy) + P.ct.y;
        const v2f pcz = ((fz + qw * uvz) + cz) + P.ct.z;
        const v2f hx = P.fx * pcx + P.cx * pcz;
        const v2f hy = P.fy * pcy + P.cy * pcz;
        const v2f rz = v2(__builtin_amdgcn_rcpf(pcz.x), __builtin_amdgcn_rcpf(pcz.y));
        int u0, u1, v0, v1;
        round_quot_i2(hx, pcz, rz, true, true, u0, u1);
        round_quot_i2(hy, pcz, rz, true, true, v0, v1);
        hzs[k] = pcz;
        const int uu[2] = {u0, u1}, vv[2] = {v0, v1};
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * k + e;
          inb[j] = uu[e] >= 0 && uu[e] < P.W && vv[e] >= 0 && vv[e] < P.H;
#if defined(TSDF_EXP) && (TSDF_EXP & 1)  // experiment build: no pixel gathers
          if (inb[j]) px[j] = make_float4(pcz[e] + 0.01f, 1.0f, 1.0f, __uint_as_float(0x00808080u));
#else
          // unconditional gathers at a clamped index (pixel 0 when out of the image): no exec-
          // masked region around the loads, so all 8 stay in flight until pass 2
          const int img = inb[j] ? vv[e] * P.W + uu[e] : 0;
          if (Raw) {  // x: depth, y: pixel x, z: pixel y, w: rgb (range / w_new computed in pass 2)
            const uint32_t c = (uint32_t)P.rgb[3 * img] | ((uint32_t)P.rgb[3 * img + 1] << 8) |
                               ((uint32_t)P.rgb[3 * img + 2] << 16);
            px[j] = make_float4(P.depth[img], __int_as_float(uu[e]), __int_as_float(vv[e]), __uint_as_float(c));
            lg[j] = P.ht ? pixel_logodds(P.ht[img], P.lt[img]) : 0.0f;
          } else {
            px[j] = D.pixA[P.pix_off + img];
            lg[j] = D.pixB[P.pix_off + img];
          }
#endif
        }
      }
      // ---- pass 2: tsdf_integrate_kernel's update (voxel_tsdf.cu:174-203), branch-free on
      // packed pairs; each voxel's result is kept only where it is updated (the reference's
      // conditions: in image, 0 < d <= max_depth, sdf > -trunc).
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j0 = 2 * k, j1 = 2 * k + 1;
        const v2f d = v2(px[j0].x, px[j1].x);
        v2f rng, w_new;
        if (Raw) {  // the ingest's per-pixel terms (identical operations)
          const f3 r0 = pixel_ray(P, __float_as_int(px[j0].y), __float_as_int(px[j0].z));
          const f3 r1 = pixel_ray(P, __float_as_int(px[j1].y), __float_as_int(px[j1].z));
          rng = v2(sqrtf(dot3(r0, r0)), sqrtf(dot3(r1, r1)));
          w_new = v2(pixel_w_new(P, d.x), pixel_w_new(P, d.y));
        } else {
          rng = v2(px[j0].y, px[j1].y);
          w_new = v2(px[j0].z, px[j1].z);
        }
        const uint32_t n0 = __float_as_uint(px[j0].w), n1 = __float_as_uint(px[j1].w);
        const v2f sdf = rng * (d - hzs[k]);
        const bool a0 = inb[j0] && !(d.x == 0 || d.x > P.max_depth) && sdf.x > neg_trunc;
        const bool a1 = inb[j1] && !(d.y == 0 || d.y > P.max_depth) && sdf.y > neg_trunc;
        if (a0 || a1) {
          v2f tn = quot_const2(sdf, P.trunc, P.inv_trunc, a0, a1);
          tn = v2(fminf(1.0f, tn.x), fminf(1.0f, tn.y));
          const uint32_t o0 = compu(cw, j0), o1 = compu(cw, j1);
          const v2f w_old = v2((float)(o0 >> 24), (float)(o1 >> 24));
          const v2f wc = w_old + w_new;  // >= 0: both weights are
          const v2f iwc = v2(__builtin_amdgcn_rcpf(wc.x), __builtin_amdgcn_rcpf(wc.y));
          uint32_t c0 = 0, c1 = 0;
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) {  // rgb running average, numerators >= 0
            const v2f num = v2((float)((o0 >> (8 * ch)) & 0xFF), (float)((o1 >> (8 * ch)) & 0xFF)) * w_old +
                            v2((float)((n0 >> (8 * ch)) & 0xFF), (float)((n1 >> (8 * ch)) & 0xFF)) * w_new;
            int32_t r0, r1;
            round_quot_pos2(num, wc, iwc, a0, a1, r0, r1);
            c0 |= (uint32_t)min(255, r0) << (8 * ch);
            c1 |= (uint32_t)min(255, r1) << (8 * ch);
          }
          const v2f tnum = v2(comp(ts, j0), comp(ts, j1)) * w_old + tn * w_new;
          const v2f tq = div_pair(tnum, wc, iwc, a0, a1);
          const v2f wr = wc + v2(0x1.fffffep-2f, 0x1.fffffep-2f);
          c0 |= weight_round_cap(wr.x, 40u) << 24;
          c1 |= weight_round_cap(wr.y, 40u) << 24;
          // semantic fusion (voxel_tsdf.cu:196-202): p' = P / (P + N) with
          //   P = exp((w_old ln p + w_new ln ht) / wc), N = exp((w_old ln(1 - p) + w_new ln lt) / wc)
          // is exactly the logistic of  L' = (w_old L + w_new log2(ht / lt)) / wc  in the base-2
          // log-odds L = log2(p / (1 - p)) the pool stores (pixB holds log2 ht - log2 lt), so the
          // update is two products and a sum; readers convert with prob_of_logodds (within 1e-4
          // of the reference's float chain, and L stays exactly 0 -- p 0.5 -- when ht == lt)
          const v2f pn = (w_old * v2(comp(pr, j0), comp(pr, j1)) + w_new * v2(lg[j0], lg[j1])) * iwc;
          if (a0) {
            setc(ts, j0, tq.x);
            setc(pr, j0, pn.x);
            setu(cw, j0, c0);
          }
          if (a1) {
            setc(ts, j1, tq.y);
            setc(pr, j1, pn.y);
            setu(cw, j1, c1);
          }
          upd_mask |= (a0 ? 1 << j0 : 0) | (a1 ? 1 << j1 : 0);
        }
        mn = fminf(mn, fminf(fabsf(comp(ts, j0)), fabsf(comp(ts, j1))));
      }
#if defined(TSDF_EXP) && (TSDF_EXP & 4)  // experiment build: no pool state stores
      if (upd_mask < 0) {
#else
      if (upd_mask == 0xF || fresh) {
#endif
        // all four voxels written (a fresh block's untouched voxels get AquireBlock's state)
        pool_st(blk + off, ts);
        pool_st(blk + kProbOffset + off, pr);
        pool_stu(blk + kRgbwOffset + off, cw);
      } else if (upd_mask) {  // only the updated voxels' words: writes stay N_upd x 12 B
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (upd_mask & (1 << j)) {
            reinterpret_cast<float*>(blk + off)[j] = comp(ts, j);
            reinterpret_cast<float*>(blk + kProbOffset + off)[j] = comp(pr, j);
            reinterpret_cast<uint32_t*>(blk + kRgbwOffset + off)[j] = compu(cw, j);
          }
      }
      my_upd += __popc(upd_mask);
    }
    mn = wave_min(mn);
    if (lane == 0) s_min[wave] = mn;
    lds_barrier();  // (LDS only: this pair's pool stores stay in flight)
    if (hf == 0 && lane == 0 && b < nvis) {
      const float m2 = fminf(s_min[wave], s_min[wave + 1]);
      if (m2 >= 0.9f) {  // space_carving_kernel threshold (voxel_tsdf.cu:227, :485)
        const int k = atomicAdd(&s_ncand, 1);
        if (k < kIntegrateCandBuf) {
          s_cand[k] = r;
        } else {  // buffer full (heavy carving): publish this one now
          const int kg = atomicAdd(&D.ctr->n_cand, 1);
          const unsigned long long* rv = reinterpret_cast<const unsigned long long*>(&r);
          unsigned long long* dst = reinterpret_cast<unsigned long long*>(&D.cand[kg]);
          st_co(&dst[0], rv[0]);
          st_co(&dst[1], rv[1]);
          s_ovf = 1;
        }
      }
    }
    lds_barrier();
  }
  // updated-voxel count: the workgroup's total rides on its arrival (summed by the last arriver)
  const int tot = wave_sum(my_upd);
  if (lane == 0) s_upd[wave] = tot;
  lds_barrier();
  const unsigned long long wg_upd = (unsigned long long)(s_upd[0] + s_upd[1] + s_upd[2] + s_upd[3]);
  // carve candidates: published (agent-scope stores) for the workgroup that resolves the carving at
  // the end of this launch; only wave 0 publishes, so only it drains its stores before arriving
  const int nc = min(s_ncand, kIntegrateCandBuf);
  if (wave == 0 && nc > 0) {
    int k0 = 0;
    if (lane == 0) k0 = atomicAdd(&D.ctr->n_cand, nc);
    k0 = __shfl(k0, 0, 64);
    if (lane < nc) {
      const unsigned long long* rv = reinterpret_cast<const unsigned long long*>(&s_cand[lane]);
      unsigned long long* dst = reinterpret_cast<unsigned long long*>(&D.cand[k0 + lane]);
      st_co(&dst[0], rv[0]);
      st_co(&dst[1], rv[1]);
    }
  }
  TSDF_STAMP(D, 3, 1);
#ifdef TSDF_DIAG_STAMPS
  if (threadIdx.x == 0 && D.dbg && blockIdx.x < (unsigned)kDiagMaxWg) {  // placement + work of the WG
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* q = D.dbg + ((size_t)3 * kDiagMaxWg + blockIdx.x) * kDiagStamps;
    q[4] = hw;
    q[5] = xcc;
    q[6] = (unsigned long long)((p_hi - (p_lo + (int)(blockIdx.x >> 3)) + ngrp - 1) / ngrp);  // pairs
  }
#endif
  // waves that published drain their stores before the workgroup arrives (wave 0: the buffer;
  // the even waves' lane 0: overflow records)
  const bool drain = (wave == 0 && nc > 0) || (s_ovf && (wave & 1) == 0);
  if (!arrive_last(D.arrive + kArrIntegrate, wg_upd, &s_last, drain, (uint32_t)nint)) return false;
  integrate_tail<Pre>(D, P, L);
  return true;
}

template <bool Graph, bool Raw>
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_INTEGRATE_WAVES, TSDF_INTEGRATE_WAVES))) void k_integrate_t(
    EngineDev D, FrameParams Pv, const FrameArgs* __restrict__ A) {
  __shared__ DeleteLds L;  // the last-arriving workgroup's carving resolve
  integrate_body<Graph, Raw>(D, Pv, A, (int)gridDim.x, L);
}

// A pipelined frame: ONE launch does frame n's update and carving and frame n + 1's ingest.
//  * workgroups [0, nint): frame n's update (D.integrate_grid_pre: one resident wave of them, all
//    dispatched before any of the workgroups below); the last to arrive carves frame n, publishes
//    the carving (write-through stores drained, then one flag per XCD = tag), waits until every
//    workgroup below has counted itself (per-XCD counters) and then runs frame n + 1's allocation
//    resolver -- k_ingest_dda's tail;
//  * kVisWorkgroups workgroups: frame n + 1's visibility sweep (vis_sweep_chained: listed and tested
//    while frame n is updated, the words the carving marks re-tested once it is published, then the
//    band lists appended);
//  * one workgroup per pixel tile of frame n + 1 (kTileChained): pixel records into the other record
//    buffer, the DDA, the key dedupe and the all-corners test while frame n is updated, then, once
//    the carving is published, the table probe and the new-key insert.
// The tail publishes the carving, then computes frame n's statistics (integrate_stats) while the
// chained workgroups run. The sweep and the probes see the table frame n's carving left and the allocation reads the keys
// they inserted: the same operations in the same order as the two-launch frame, so the same results.
// The waits cannot deadlock: the update's workgroups are all dispatched before the waiting ones and
// wait for nothing; the last of them waits only for workgroups that wait for nothing it has not
// already published. Every wait is bounded (TSDF_STATUS_PIPELINE_TIMEOUT).
#ifndef TSDF_PRE_WAVES
#define TSDF_PRE_WAVES TSDF_INTEGRATE_WAVES
#endif
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_PRE_WAVES, TSDF_PRE_WAVES))) void k_integrate_pre(
    EngineDev D, FrameParams P, FrameParams Pn, int tiles_x, int tiles, uint32_t tag) {
  __shared__ union {
    DeleteLds del;
    IngestLds<1024> ing;
  } U;
  const int nint = D.integrate_grid_pre;
  const int w = (int)blockIdx.x - nint;
  if (w >= 0) {
    TSDF_STAMP_WG(D, 5, w, 0);
    // the tiles first, then the sweep workgroups. Measured: with the sweep after the wait, sweep
    // first was faster (22.85k vs 22.3k frames/s); since the sweep tests before the carving is
    // published, tiles first ends the chained work 0.3-0.5 us earlier (23.77k / 23.95k vs 23.65k /
    // 23.82k, scripts/gpu_r3_last.sh): the tiles' DDA, dispatched as the update retires, is the
    // longer pre-carving part
#ifndef TSDF_PRE_SWEEP_FIRST
    if (w >= tiles) {
      vis_sweep_chained<1024>(D, Pn, w - tiles, U.ing, D.arrive + kArrCarved + (blockIdx.x % kCarvedFlags) * 16, tag);
    } else {
      ingest_tile<1024, kTileChained>(D, Pn, Pn.depth, Pn.rgb, Pn.ht, Pn.lt, tiles_x, w, U.ing, tag);
    }
#else
    if (w < kVisWorkgroups) {
#ifdef TSDF_SWEEP_AFTER_WAIT  // (experiment: the whole sweep after the carving)
      wait_tag(D.arrive + kArrCarved + (blockIdx.x % kCarvedFlags) * 16, tag, &D.ctr->status);
      vis_sweep<1024, true>(D, Pn, w, U.ing);
#else
      vis_sweep_chained<1024>(D, Pn, w, U.ing, D.arrive + kArrCarved + (blockIdx.x % kCarvedFlags) * 16, tag);
#endif
    } else {
      ingest_tile<1024, kTileChained>(D, Pn, Pn.depth, Pn.rgb, Pn.ht, Pn.lt, tiles_x, w - kVisWorkgroups, U.ing, tag);
    }
#endif
    // done: this workgroup's band counts / new keys are published (atomics that returned, sc1 list
    // stores drained), then it counts itself for the allocation
    __builtin_amdgcn_s_waitcnt(0);
    lds_barrier();
    TSDF_STAMP_WG(D, 5, w, 3);
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(D.arrive + kArrChained + (blockIdx.x % kChainCounters) * 16, 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (!integrate_body<false, false, true>(D, P, nullptr, nint, U.del)) return;
  const unsigned long long t_pub = __builtin_amdgcn_s_memrealtime();
  TSDF_STAMP_WG(D, 5, kDiagMaxWg - 1, 0);
  // the carving tail has run (it reset the band counts the sweep appends to); its table and
  // band stores were written through (sc1) and its occupancy updates are atomics: drained, they are
  // visible to agent-scope reads on every XCD, so publish (no L2 write-back of the update's lines)
  __builtin_amdgcn_s_waitcnt(0);
  lds_barrier();
  const int t = threadIdx.x;
  if (t < kCarvedFlags) st_co(D.arrive + kArrCarved + t * 16, (unsigned long long)tag);
  TSDF_STAMP_WG(D, 5, kDiagMaxWg - 1, 1);
  integrate_stats(D, U.del);  // frame n's statistics, while the chained workgroups run
  unsigned long long t_done = 0ull;
  if (t < 64) {  // wave 0 polls the completion counters, one per lane (spread: no hot word)
    const unsigned long long want = (unsigned long long)(kVisWorkgroups + tiles);
    unsigned long long* ctr = D.arrive + kArrChained + (t % kChainCounters) * 16;
    const bool mine = t < kChainCounters;
    uint32_t n = 0;
    for (;;) {
      unsigned long long done =
          mine ? __hip_atomic_fetch_add(ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) done += __shfl_xor(done, o, 64);
      if (done >= want) break;  // (wave-uniform)
      __builtin_amdgcn_s_sleep(2);
      if (++n > (1u << 23)) {
        if (t == 0) atomicOr(&D.ctr->status, 64u);  // TSDF_STATUS_PIPELINE_TIMEOUT
        break;
      }
    }
    if (mine) st_co(ctr, 0ull);  // (for the next launch)
    t_done = __builtin_amdgcn_s_memrealtime();
  }
  TSDF_STAMP_WG(D, 5, kDiagMaxWg - 1, 2);
  __syncthreads();
  // frame n + 1's allocation (k_ingest_dda's tail)
  resolve_alloc_wg(D, Pn, (uint32_t)Pn.W * (uint32_t)Pn.H * (uint32_t)Pn.maxs, 1, U.ing.u.res);
  TSDF_STAMP_WG(D, 5, kDiagMaxWg - 1, 3);
  // chained frames have no k_ingest_dda: its span counter holds carving published -> every chained
  // workgroup counted (the sweep and the probes after the carving)
  if (t == 0) D.ctr->ingest_ticks += t_done - t_pub;
}
template __global__ void k_integrate_t<false, false>(EngineDev, FrameParams, const FrameArgs*);
template __global__ void k_integrate_t<true, false>(EngineDev, FrameParams, const FrameArgs*);
template __global__ void k_integrate_t<false, true>(EngineDev, FrameParams, const FrameArgs*);
template __global__ void k_integrate_t<true, true>(EngineDev, FrameParams, const FrameArgs*);

// ---------------------------------------------------------------------------------------------
// k_resolve_delete: the carving resolver (tsdf_resolve.h) as its own one-workgroup launch -- a
// shard's frame after the candidate all-gather (cands_in: every shard's slot, listed as D.cand --
// the candidate set of one volume -- so every shard's index takes the same deletes), and the
// hash-level test path (direct: the keys in list order, one per round).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void resolve_delete_merged(EngineDev D, const VisRec* __restrict__ recs,
                                                      const int32_t* __restrict__ count, int direct,
                                                      const ShardRec* __restrict__ cands_in, int cap,
                                                      int nshard) {
  __shared__ DeleteLds L;
  __shared__ int s_base[kMaxShards + 1];
  if (cands_in) {
    if (threadIdx.x == 0) {
      // the union is listed in D.cand (cand_cap records; the resolver's D.pairs scratch holds at
      // least as many): more candidates than that is a shard overflow, the rest are dropped
      int run = 0;
      bool ovf = false;
      for (int s = 0; s < nshard; ++s) {
        s_base[s] = run;
        int n = min((int)cands_in[(size_t)s * (cap + 1)].val, cap);
        if (n > D.cand_cap - run) {
          n = D.cand_cap - run;
          ovf = true;
        }
        run += n;
      }
      s_base[nshard] = run;
      st_co(&D.ctr->n_cand, run);
      if (ovf) atomicOr(&D.ctr->status, 16u);  // TSDF_STATUS_SHARD_OVERFLOW
    }
    __syncthreads();
    unsigned long long* cq = reinterpret_cast<unsigned long long*>(D.cand);
    for (int s = 0; s < nshard; ++s) {
      const ShardRec* slot = cands_in + (size_t)s * (cap + 1) + 1;
      const int n = s_base[s + 1] - s_base[s];
      for (int i = threadIdx.x; i < n; i += kRT) {
        const ShardRec r = slot[i];
        VisRec c;
        c.x = r.x;
        c.y = r.y;
        c.z = r.z;
        c.pad = 0;
        c.idx = -1;
        c.entry = (int32_t)r.val;
        const unsigned long long* cv = reinterpret_cast<const unsigned long long*>(&c);
        st_co(&cq[2 * (s_base[s] + i)], cv[0]);
        st_co(&cq[2 * (s_base[s] + i) + 1], cv[1]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  resolve_delete_wg(D, recs, count, direct, L);
  if (!direct) frame_end(D);
}
__global__ __launch_bounds__(kRT) void k_resolve_delete(EngineDev D, const VisRec* __restrict__ recs,
                                                        const int32_t* __restrict__ count, int direct,
                                                        const ShardRec* __restrict__ cands_in, int cap,
                                                        int nshard) {
  resolve_delete_merged(D, recs, count, direct, cands_in, cap, nshard);
}
__global__ __launch_bounds__(kRT) void k_resolve_delete_g(EngineDev D, const FrameArgs* __restrict__ A) {
  resolve_delete_merged(D, D.cand, &D.ctr->n_cand, 0, A->cands_in, A->cand_cap, A->nshard);
}


}  // namespace tsdf
