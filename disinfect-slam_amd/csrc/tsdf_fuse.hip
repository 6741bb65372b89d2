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
__device__ __forceinline__ void frame_end(const EngineDev& D) {
  lds_barrier();
  if (threadIdx.x == 0) {
    D.ctr->total_visible += (unsigned long long)D.ctr->n_vis;
    D.ctr->total_updated += D.ctr->last_updated;
    D.ctr->frames += 1ull;
    *D.ncand = 0;  // the next frame's lists start empty (its sweep runs before allocation)
    D.ctr->n_pend = 0;
  }
  if (threadIdx.x < kBands) st_co(&D.band[threadIdx.x * kBandStride], 0);
}

// a shard's frame: its carve candidates into the exchange slot, then the owned entries its
// exhausted pool left without voxels this frame (D.pend, written by the allocation resolver before
// this launch)
// (cand / ncand: the frame's candidate list, D.cand / D.ncand of its view). dsts (a group's frame,
// tsdf_group_*): the slot is written into each of the ndst destinations instead -- this shard's slot in
// every shard's inbox, across GPUs by peer stores -- so no exchange runs between the launches.
__device__ __forceinline__ void pack_cands_wg(const EngineDev& D, const VisRec* cand, const int32_t* ncand, ShardRec* __restrict__ out,
                              int cap, ShardRec* const* dsts = nullptr, int ndst = 0) {
  const int nc = ld_co(ncand);
  const int np = min(ld_co(&D.ctr->n_pend), (int)kNewKeyCap);
  const int n = nc + np;
  const unsigned long long* rq = reinterpret_cast<const unsigned long long*>(cand);
  for (int i = threadIdx.x; i < min(n, cap); i += blockDim.x) {
    unsigned long long a, b;
    if (i < nc) {
      a = ld_co(&rq[2 * i]);
      b = ld_co(&rq[2 * i + 1]);
    } else {
      const unsigned long long* pq = reinterpret_cast<const unsigned long long*>(D.pend + (i - nc));
      a = ld_co(&pq[0]);
      b = ld_co(&pq[1]);
    }
    ShardRec r;
    r.x = (int16_t)(a & 0xFFFF);
    r.y = (int16_t)((a >> 16) & 0xFFFF);
    r.z = (int16_t)((a >> 32) & 0xFFFF);
    r.pad = 0;
    r.val = (uint32_t)(b >> 32);  // hash entry
    r.zero = 0u;
    if (dsts) {
      for (int d = 0; d < ndst; ++d) dsts[d][1 + i] = r;
    } else {
      out[1 + i] = r;
    }
  }
  if (threadIdx.x == 0) {
    ShardRec h{};
    h.val = (uint32_t)min(n, cap);
    if (dsts) {
      for (int d = 0; d < ndst; ++d) dsts[d][0] = h;
    } else {
      out[0] = h;
    }
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
  // every frame view's band counts and candidate count, and the pipelined frames' statistics (a
  // shard's pending pipelined frames are dropped as well; D is the base view)
  for (int i = threadIdx.x; i < 3 * kBands; i += blockDim.x) D.band[i * kBandStride] = 0;
  if (threadIdx.x < 2) D.pipe[kPipeNCand + 16 * threadIdx.x] = 0ull;
  for (int i = kPipeStats + threadIdx.x; i < kPipeWords; i += blockDim.x) D.pipe[i] = 0ull;
  for (int i = threadIdx.x; i < kArriveWords; i += blockDim.x) D.arrive[i] = 0ull;
  __syncthreads();
  if (threadIdx.x == 0) {
    D.ctr->nk_count = 0;
    *D.ncand = 0;
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
// The C5 loop's raycast view grid built inside the update launch (k_integrate_vg): the render camera,
// its grid and the launch's release tag (the carving tags the pool blocks it releases with it)
struct ViewFuse {
  FrameParams R;
  ViewGrid V;
  uint32_t vtag;
};
// the grid's cells of the blocks this launch's carving released read as missing again: the grid
// workgroups listed them before the carving (their cells are written through and drained before they
// arrive, so these stores, after every arrival, are the cells' last writes)
__device__ __forceinline__ void view_patch_carved(const EngineDev& D, const ViewFuse& F) {
  __builtin_amdgcn_s_waitcnt(0);  // (the carving's rtag stores of every wave)
  __syncthreads();
  const ViewGrid& V = F.V;
  const int n = min(ld_co(D.ncand), D.cand_cap);
  const int ox = view_origin(F.R.wt.x, F.R.voxel, V.half), oy = view_origin(F.R.wt.y, F.R.voxel, V.half),
            oz = view_origin(F.R.wt.z, F.R.voxel, V.half);
  const unsigned long long* rq = reinterpret_cast<const unsigned long long*>(D.cand);
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const unsigned long long a = ld_co(&rq[2 * k]), b = ld_co(&rq[2 * k + 1]);
    const int lx = (int16_t)(a & 0xFFFF) - ox, ly = (int16_t)((a >> 16) & 0xFFFF) - oy,
              lz = (int16_t)((a >> 32) & 0xFFFF) - oz;
    const int32_t idx = (int32_t)(uint32_t)b;
    if ((unsigned)lx >= (unsigned)V.n || (unsigned)ly >= (unsigned)V.n || (unsigned)lz >= (unsigned)V.n || idx < 0)
      continue;
    if (__hip_atomic_load(&D.rtag[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != F.vtag) continue;
    const int kb = ((lz >> 2) * V.nb + (ly >> 2)) * V.nb + (lx >> 2);
    __hip_atomic_store(&V.cell[view_cell(kb, lx, ly, lz)], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void integrate_tail(const EngineDev& D, const FrameParams& P, DeleteLds& L,
                                               const ViewFuse* F = nullptr) {
  const int t = threadIdx.x;
  const unsigned long long tend = __builtin_amdgcn_s_memrealtime();  // the update's span ends here
  TSDF_STAMP(D, 7, 0);
  if (P.tail == kTailPack)
    pack_cands_wg(D, D.cand, D.ncand, P.slot, P.slot_cap);
  else
    resolve_delete_wg(D, D.cand, D.ncand, 0, L, F ? F->vtag : 0u);
#ifndef TSDF_NO_VIEW_PATCH  // (a test build leaves the released blocks' cells: the C5 tests must fail)
  if (F) view_patch_carved(D, *F);
#endif
  TSDF_STAMP(D, 7, 1);
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

// One visible block's update (tsdf_integrate_kernel, voxel_tsdf.cu:149-205) by one wave of the two
// that share it (hf: which half of its 512 voxels; 4 voxels per lane). mn: the minimum |tsdf| of the
// lane's voxels after the update (the carving test), my_upd: + the lane's updated voxels.
// The block's loads (pool state: update_issue_pool; projection + pixel gathers: update_issue_pix) and
// the update itself (update_finish); update_block = all three. (Issuing the next record's loads before
// finishing this one -- all of them, or the pool state only -- measured 5-17 % slower at 4-6 waves per
// SIMD: the carried state spills at 5-6 waves, and 4 waves starve the launch's tiles;
// profiles/ab/r6_update_prefetch_ab.txt.)
struct UpdState {
  float4 ts, pr;
  uint4 cw;
  float4 px[4];
  uint32_t pc[4];
  v2f hzs[2];
  bool inb[4];
  bool fresh;
};

__device__ __forceinline__ void update_issue_pool(const EngineDev& D, const VisRec& r, int lane, int hf,
                                                  UpdState& S) {
  const int off = (hf * 256 + lane * 4) * 4;
  const int32_t pidx = r.idx;
  uint8_t* blk = D.pool + (size_t)pidx * kBlockBytes;
  float4& ts = S.ts;
  float4& pr = S.pr;
  uint4& cw = S.cw;
#if defined(TSDF_EXP) && (TSDF_EXP & 2)  // experiment build: no pool state loads
  bool fresh;
  ts = make_float4(0.5f, 0.5f, 0.5f, 0.5f), pr = ts;
  cw = make_uint4(0x05808080u, 0x05808080u, 0x05808080u, 0x05808080u);
#else
  const bool fresh = r.pad != 0;
  if (fresh) {  // wave-uniform: a block created this frame loads nothing
    ts = make_float4(-1.f, -1.f, -1.f, -1.f);
    pr = make_float4(0.5f, 0.5f, 0.5f, 0.5f);  // AquireBlock's p = 0.5
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
  S.fresh = fresh;
}
template <bool Raw>
__device__ __forceinline__ void update_issue_pix(const EngineDev& D, const FrameParams& P, const VisRec& r, int lane,
                                                 int hf, UpdState& S) {
  const int rx0 = (lane & 1) * 4, ry = (lane >> 1) & 7, rz = (lane >> 4) + 4 * hf;
  float4* px = S.px;
  uint32_t* pc = S.pc;
  v2f* hzs = S.hzs;
  bool* inb = S.inb;
  const int16_t ax0 = (int16_t)(r.x << kBlockLenBits), ay = (int16_t)((r.y << kBlockLenBits) + ry),
                az = (int16_t)((r.z << kBlockLenBits) + rz);
  const float fy = (float)ay * P.voxel, fz = (float)az * P.voxel;
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
      if (inb[j]) px[j] = make_float4(pcz[e] + 0.01f, 1.0f, 0.0f, 0.0f), pc[j] = 0x00808080u;
#else
      // unconditional gathers at a clamped index (pixel 0 when out of the image): no exec-
      // masked region around the loads, so all 8 stay in flight until pass 2
      const int img = inb[j] ? vv[e] * P.W + uu[e] : 0;
      if (Raw) {  // x: depth, y / z: ht / lt (their logs, range and w_new computed in pass 2)
        pc[j] = (uint32_t)P.rgb[3 * img] | ((uint32_t)P.rgb[3 * img + 1] << 8) |
                ((uint32_t)P.rgb[3 * img + 2] << 16);
        px[j] = make_float4(P.depth[img], P.ht ? P.ht[img] : 1.0f, P.lt ? P.lt[img] : 1.0f,
                            __int_as_float((uu[e] & 0xFFFF) | (vv[e] << 16)));  // w: the pixel (u, v)
      } else {  // x: depth, y: range, z: logf(ht), w: logf(lt) (w_new computed in pass 2)
        px[j] = D.pixA[P.pix_off + img];
        pc[j] = D.pixC[P.pix_off + img];
      }
#endif
    }
  }
}

template <bool Raw>
__device__ __forceinline__ void update_issue(const EngineDev& D, const FrameParams& P, const VisRec& r, int lane,
                                             int hf, UpdState& S) {
  update_issue_pool(D, r, lane, hf, S);
  update_issue_pix<Raw>(D, P, r, lane, hf, S);
}

template <bool Raw>
__device__ __forceinline__ void update_finish(const EngineDev& D, const FrameParams& P, const VisRec& r, int lane,
                                              int hf, UpdState& S, float& mn, int& my_upd) {
  const int off = (hf * 256 + lane * 4) * 4;
  const float neg_trunc = -P.trunc;
  uint8_t* blk = D.pool + (size_t)r.idx * kBlockBytes;
  float4 ts = S.ts, pr = S.pr;
  uint4 cw = S.cw;
  const float4* px = S.px;
  const uint32_t* pc = S.pc;
  const v2f* hzs = S.hzs;
  const bool* inb = S.inb;
  const bool fresh = S.fresh;
  int upd_mask = 0;
  // ---- pass 2: tsdf_integrate_kernel's update (voxel_tsdf.cu:174-203) of tsdf, colour and weight,
  // branch-free on packed pairs; each voxel's result is kept only where it is updated (the
  // reference's conditions: in image, 0 < d <= max_depth, sdf > -trunc). The semantic update
  // follows in pass 3, once the pixel records and the other state are dead (its chain of logs and
  // exponentials beside them spilled the loop out of 72 VGPRs).
  const uint32_t wold4 = (compu(cw, 0) >> 24) | ((compu(cw, 1) >> 24) << 8) | ((compu(cw, 2) >> 24) << 16) |
                         ((compu(cw, 3) >> 24) << 24);  // the old weights, one byte per voxel
  float wn[4] = {0.f, 0.f, 0.f, 0.f};
  int pfast = 0;  // sem_pixel_fast per voxel
  v2f lnh2[2], lnl2[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j0 = 2 * k, j1 = 2 * k + 1;
    const v2f d = v2(px[j0].x, px[j1].x);
    v2f rng, w_new = v2(0.f, 0.f), lnh, lnl;
    bool pf0, pf1;  // sem_pixel_fast
    if (Raw) {  // the ingest's per-pixel terms (identical operations)
      const int w0 = __float_as_int(px[j0].w), w1 = __float_as_int(px[j1].w);
      const f3 r0 = pixel_ray(P, w0 & 0xFFFF, w0 >> 16);
      const f3 r1 = pixel_ray(P, w1 & 0xFFFF, w1 >> 16);
      rng = v2(sqrtf(dot3(r0, r0)), sqrtf(dot3(r1, r1)));
      w_new = v2(pixel_w_new(P, d.x), pixel_w_new(P, d.y));
      lnh = sem_logf2(v2(px[j0].y, px[j1].y));
      lnl = sem_logf2(v2(px[j0].z, px[j1].z));
      pf0 = sem_pixel_fast(px[j0].y, px[j0].z, d.x, P.max_depth);
      pf1 = sem_pixel_fast(px[j1].y, px[j1].z, d.y, P.max_depth);
    } else {
      rng = v2(fabsf(px[j0].y), fabsf(px[j1].y));
      pf0 = px[j0].y > 0.0f;
      pf1 = px[j1].y > 0.0f;
      lnh = v2(px[j0].z, px[j1].z);
      lnl = v2(px[j0].w, px[j1].w);
    }
    const uint32_t n0 = pc[j0], n1 = pc[j1];
    const v2f sdf = rng * (d - hzs[k]);
    const bool a0 = inb[j0] && !(d.x == 0 || d.x > P.max_depth) && sdf.x > neg_trunc;
    const bool a1 = inb[j1] && !(d.y == 0 || d.y > P.max_depth) && sdf.y > neg_trunc;
    if (a0 || a1) {
      // w_new = (1 - d / max_depth) * 4 (pixel_w_new's operations, on the pair; the 16-B pixel record
      // has no room for it: one gather per voxel instead of two)
      if (!Raw) w_new = (v2(1.0f, 1.0f) - quot_const2(d, P.max_depth, P.inv_max_depth, a0, a1)) * v2(4.0f, 4.0f);
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
      wn[j0] = w_new.x;
      wn[j1] = w_new.y;
      if (a0) {
        setc(ts, j0, tq.x);
        setu(cw, j0, c0);
      }
      if (a1) {
        setc(ts, j1, tq.y);
        setu(cw, j1, c1);
      }
      upd_mask |= (a0 ? 1 << j0 : 0) | (a1 ? 1 << j1 : 0);
    }
    lnh2[k] = lnh;
    lnl2[k] = lnl;
    pfast |= (pf0 ? 1 << j0 : 0) | (pf1 ? 1 << j1 : 0);
    mn = fminf(mn, fminf(fabsf(comp(ts, j0)), fabsf(comp(ts, j1))));
  }
  __builtin_amdgcn_sched_barrier(0);
  // ---- pass 3: semantic fusion (voxel_tsdf.cu:196-202), the reference's float chain operation for
  // operation:
  //   P = expf((w_old logf(p) + w_new logf(ht)) / wc), N = expf((w_old logf(1 - p) + w_new logf(lt)) / wc),
  //   p' = P / (P + N)
  // (logf / expf: the oracle's fixed algorithms, sem_logf / sem_expf; the quotients IEEE-exact). The
  // fast path runs on both voxels of a pair; a voxel whose operands leave its range -- p 0 or 1, ht or
  // lt 0, extreme quotients -- is recomputed with every special case (sem_update_exact).
#if !(defined(TSDF_EXP) && (TSDF_EXP & 8))  // (experiment build: no semantic update, timing only)
  // both pairs' fast chains first, with no branch between them (the compiler interleaves the two
  // dependency chains: +0.3 % frames/s, the update span -1 us, same box), then the rare exact
  // recomputations
  {
    v2f pn2[2], pv2[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j0 = 2 * k, j1 = 2 * k + 1;
      const v2f w_old = v2((float)((wold4 >> (8 * j0)) & 0xFF), (float)((wold4 >> (8 * j1)) & 0xFF));
      const v2f w_new = v2(wn[j0], wn[j1]);
      const v2f wc = w_old + w_new;
      const v2f pv = v2(comp(pr, j0), comp(pr, j1));
      const v2f an = w_old * sem_log_fast2(pv) + w_new * lnh2[k];
      const v2f bn = w_old * sem_log_fast2(v2(1.0f, 1.0f) - pv) + w_new * lnl2[k];
      const v2f y1 = div_refine(wc, v2(__builtin_amdgcn_rcpf(wc.x), __builtin_amdgcn_rcpf(wc.y)));
      const v2f sp = sem_exp_fast2(div_expand(an, wc, y1));
      const v2f sn = sem_exp_fast2(div_expand(bn, wc, y1));
      const v2f ss = sp + sn;
      pn2[k] = div_expand(sp, ss, div_refine(ss, v2(__builtin_amdgcn_rcpf(ss.x), __builtin_amdgcn_rcpf(ss.y))));
      pv2[k] = pv;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!((upd_mask >> j) & 1)) continue;
      const float pv = pv2[j >> 1][j & 1];
      float pn = pn2[j >> 1][j & 1];
      if (__builtin_expect(!sem_voxel_fast((pfast >> j) & 1, pv), 0)) {
        const float w_old = (float)((wold4 >> (8 * j)) & 0xFF);
        pn = sem_update_exact(pv, w_old, wn[j], w_old + wn[j], lnh2[j >> 1][j & 1], lnl2[j >> 1][j & 1]);
      }
      setc(pr, j, pn);
    }
  }
#endif
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

template <bool Raw>
__device__ __forceinline__ void update_block(const EngineDev& D, const FrameParams& P, const VisRec& r, int lane,
                                             int hf, float& mn, int& my_upd) {
  UpdState S;
  update_issue<Raw>(D, P, r, lane, hf, S);
  update_finish<Raw>(D, P, r, lane, hf, S, mn, my_upd);
}

// The concatenated band lists: band i holds visible-block indices [start_i, start_i + count_i).
// Lane i < kBands keeps start_i (one VGPR; an indexed array of 16 starts is spilled to scratch in
// the big kernels), and the wave-uniform search for index b is a ballot: the starts are
// non-decreasing, so the lanes with start <= b are a prefix and the band is its last lane.
__device__ __forceinline__ int band_starts_p(const int32_t* band, int lane, int* total) {
  const int c = lane < kBands ? band[lane * kBandStride] : 0;
  int incl = c;
#pragma unroll
  for (int o = 1; o < kBands; o <<= 1) {
    const int n = __shfl_up(incl, o, 64);
    if (lane >= o) incl += n;
  }
  *total = __builtin_amdgcn_readlane(incl, kBands - 1);
  return incl - c;
}
__device__ __forceinline__ int band_starts(const EngineDev& D, int lane, int* total) {
  return band_starts_p(D.band, lane, total);
}
// (b wave-uniform, 0 <= b < total) -> the band's list record index: band * nblocks + offset
__device__ __forceinline__ size_t band_find_n(int nblocks, int bst, int lane, int b) {
  const unsigned long long m = __ballot(lane < kBands && b >= bst);
  const int bd = __popcll(m) - 1;
  const int ofs = b - __builtin_amdgcn_readlane(bst, bd);
  return (size_t)bd * nblocks + (size_t)__builtin_amdgcn_readfirstlane(ofs);
}
__device__ __forceinline__ size_t band_find(const EngineDev& D, int bst, int lane, int b) {
  return band_find_n(D.nblocks, bst, lane, b);
}

// 64 VGPRs: 8 waves per SIMD (65 without the bound: 7). Graph: the graph-captured form reads its
// camera from the FrameArgs block the graph's first node uploads.
// The visible blocks are the sweep's band lists (blocks that existed before the frame) followed by
// the blocks k_resolve_alloc created (D.fresh_vis, flagged fresh).
// Raw: a shard's frame -- the pixel terms come from the raw frame (depth, rgb, ht, lt gathers) and
// are computed per voxel with the ingest's operations (pixel_w_new, sem_logf of ht / lt, the range of
// pixel_ray), instead of from pixel records packed for the whole frame.
#ifndef TSDF_INTEGRATE_WAVES  // 6: the semantic update's chain (pass 3) spills the update loop at 7
#define TSDF_INTEGRATE_WAVES 6
#endif
// nint: the update's workgroups (the whole grid). L: the LDS of the last arriver's carving resolve.
// returns true in the workgroup that arrived last (and ran the carving tail)
template <bool Graph, bool Raw>
__device__ __forceinline__ bool integrate_body(const EngineDev& D, const FrameParams& Pv,
                                               const FrameArgs* __restrict__ A, int nint, DeleteLds& L,
                                               int narrive = 0, const ViewFuse* F = nullptr) {
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
  int nvis = 0;
  const int bst = band_starts(D, lane, &nvis);
  const int nband = nvis;
  nvis += D.ctr->n_fresh;
  const int g = blockIdx.x & 7, ngrp = nint >> 3;
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
  // (The chunked, barrier-free form of pipe_update measured slower here, 14.07-14.27k vs 14.8k frames/s
  // at C4 on one box: a k_integrate workgroup updates one or two pairs, so the collection's extra round
  // trip is not amortised.)
  for (int pp = p_lo + (blockIdx.x >> 3); pp < p_hi; pp += ngrp) {
    const int b = 2 * pp + pair;
    float mn = __builtin_inff();
    VisRec r{};
    if (b < nvis) {
      if (b >= nband) {
        r = D.fresh_vis[b - nband];
      } else {
        r = D.vis[band_find(D, bst, lane, b)];
      }
      update_block<Raw>(D, P, r, lane, hf, mn, my_upd);
    }
    mn = wave_min_u(mn);
    if (lane == 0) s_min[wave] = mn;
    lds_barrier();  // (LDS only: this pair's pool stores stay in flight)
    if (hf == 0 && lane == 0 && b < nvis) {
      const float m2 = fminf(s_min[wave], s_min[wave + 1]);
      if (m2 >= 0.9f) {  // space_carving_kernel threshold (voxel_tsdf.cu:227, :485)
        const int k = atomicAdd(&s_ncand, 1);
        if (k < kIntegrateCandBuf) {
          s_cand[k] = r;
        } else {  // buffer full (heavy carving): publish this one now
          const int kg = atomicAdd(D.ncand, 1);
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
    if (lane == 0) k0 = atomicAdd(D.ncand, nc);
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
  if (!arrive_last(D.arrive + kArrIntegrate, wg_upd, &s_last, drain, (uint32_t)(narrive ? narrive : nint)))
    return false;
  integrate_tail(D, P, L, F);
  return true;
}

template <bool Graph, bool Raw>
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_INTEGRATE_WAVES, TSDF_INTEGRATE_WAVES))) void k_integrate_t(
    EngineDev D, FrameParams Pv, const FrameArgs* __restrict__ A) {
  __shared__ DeleteLds L;  // the last-arriving workgroup's carving resolve
  integrate_body<Graph, Raw>(D, Pv, A, (int)gridDim.x, L);
}

// k_integrate with the C5 loop's view grid (tsdf_raycast_deferred after an unpipelined update):
// workgroups [0, nint) update, the rest build the render camera's view grid from the table as the
// update leaves it (nothing in the launch but the carving changes the table) -- its cells written
// through (sc1) -- and the carving's last arriver clears the cells of the blocks it released. The
// k_view_grid launch and its kernel boundary drop out of the frame.
template <bool Graph>
__device__ __forceinline__ void integrate_vg(const EngineDev& D, const FrameParams& Pv, const FrameArgs* A,
                                             const FrameParams& R, const ViewGrid& V, uint32_t vtag, int nint,
                                             DeleteLds& L) {
  const ViewFuse F{R, V, vtag};
  const int narr = (int)gridDim.x;
  if ((int)blockIdx.x < nint) {
    integrate_body<Graph, false>(D, Pv, A, nint, L, narr, &F);
    return;
  }
  const int w = ((int)blockIdx.x - nint) * 256 + (int)threadIdx.x;  // (one occupancy word per thread)
  if (V.n && threadIdx.x < 256) {
    const int ox = view_origin(R.wt.x, R.voxel, V.half), oy = view_origin(R.wt.y, R.voxel, V.half),
              oz = view_origin(R.wt.z, R.voxel, V.half);
    unsigned long long occ = D.occ[w];
    while (occ) {
      const int b = __ffsll((long long)occ) - 1;
      occ &= occ - 1;
      const Ent en = load_ent(D.table, (uint32_t)(w * 64 + b));
      const int lx = en.x - ox, ly = en.y - oy, lz = en.z - oz;
      if ((unsigned)lx >= (unsigned)V.n || (unsigned)ly >= (unsigned)V.n || (unsigned)lz >= (unsigned)V.n ||
          !local_idx(en.idx))
        continue;
      const int k = ((lz >> 2) * V.nb + (ly >> 2)) * V.nb + (lx >> 2);
      __hip_atomic_store(&V.cell[view_cell(k, lx, ly, lz)], (V.gen << kViewIdxBits) | (uint32_t)en.idx,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      V.flags[k] = 1;
      V.flags[V.nbw * 32 + ((lz >> 4) * V.ns + (ly >> 4)) * V.ns + (lx >> 4)] = 1;
    }
  }
  __shared__ int s_last;
  if (!arrive_last(D.arrive + kArrIntegrate, 0ull, &s_last, true, (uint32_t)narr)) return;
  if (Graph) {  // (integrate_body's graph parameters: the frame's camera, the carving tail)
    FrameParams P = A->P;
    P.tail = kTailResolve;
    integrate_tail(D, P, L, &F);
  } else {
    integrate_tail(D, Pv, L, &F);
  }
}
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_INTEGRATE_WAVES, TSDF_INTEGRATE_WAVES))) void k_integrate_vg(
    EngineDev D, FrameParams Pv, FrameParams R, ViewGrid V, uint32_t vtag, int nint) {
  __shared__ DeleteLds L;
  integrate_vg<false>(D, Pv, nullptr, R, V, vtag, nint, L);
}
// the graph-captured form (a render graph's update node): camera, render camera, grid and release tag
// from the frame's argument block
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_INTEGRATE_WAVES, TSDF_INTEGRATE_WAVES))) void k_integrate_vg_g(
    EngineDev D, const FrameArgs* __restrict__ A, int nint) {
  __shared__ DeleteLds L;
  integrate_vg<true>(D, FrameParams{}, A, A->R, A->V, A->vtag, nint, L);
}

// =============================================================================================
// Pipelined frames (tsdf_integrate on one volume; DESIGN.md 4 "Pipelined frames"): k_frame.
// TSDFGrid::Integrate (voxel_tsdf.cu:347-375) of frame b is allocation -> visibility -> update ->
// carving, and frame b + 1 needs frame b's carving before its own allocation. The update of a block
// reads only that block and the frame, and a carving only deletes blocks that were its own frame's
// carve candidates, so the blocks frame b sees that were not frame b - 1's candidates can be updated
// before frame b - 1's carving has run. One launch per frame in a stream does:
//  * workgroup 0: frame b - 1's carving (its candidates, listed by last launch's update), then frame
//    b's allocation (its new keys, inserted by last launch's tiles), each published with a flag;
//  * frame b's update: the blocks of b's visible lists (last launch's sweep) right away, except frame
//    b - 1's candidates (ctag), which wait for the carving flag and are updated if it kept them
//    (rtag); the blocks b's allocation creates, once its flag is up (kPipeFreshWG workgroups);
//  * frame c = b + 1's ingest: pixel records, DDA, tile dedupe and all-corners test, and the sweep's
//    listing at once; after the allocation flag the tiles probe and insert (a found key records its
//    order in D.fo: the next launch's carving re-inserts the keys it deletes) and the sweep re-tests
//    the occupancy words the carving and the allocation changed (swdirty).
// Every operation reads the data it would read in the unpipelined frame order, so the results are
// identical (tests/test_gpu_pipeline.py). Frame f's lists, counts and candidates live in its view
// (frame_view); nothing a launch reads is written by the same launch except through the two flags.
// The waits cannot deadlock: workgroup 0 is dispatched first and waits for nothing. Every wait is
// bounded (TSDF_STATUS_PIPELINE_TIMEOUT).
// =============================================================================================

// frame f's statistics from its update workgroups' counters (the update ran in an earlier launch),
// zeroed for frame f + 2. Wave 0.
__device__ __forceinline__ void pipe_frame_stats(const EngineDev& D, uint32_t f) {
  const int t = threadIdx.x;
  if (t >= 64) return;
  unsigned long long* base = D.pipe + kPipeStats + (size_t)(f & 1u) * (kPipeStatLines * 16);
  const unsigned long long w = base[16 * t], te = base[16 * t + 1];
  base[16 * t] = 0ull;
  base[16 * t + 1] = 0ull;
  unsigned long long vis = w >> 40, upd = w & ((1ull << 40) - 1ull), tmax = te;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    vis += __shfl_xor(vis, o, 64);
    upd += __shfl_xor(upd, o, 64);
    const unsigned long long m = __shfl_xor(tmax, o, 64);
    tmax = m > tmax ? m : tmax;
  }
  if (t == 0) {
    const unsigned long long t0 = D.pipe[kPipeT0 + 16 * (f & 1u)];
    D.ctr->n_vis = (int32_t)vis;
    D.ctr->last_updated = upd;
    D.ctr->total_visible += vis;
    D.ctr->total_updated += upd;
    D.ctr->frames += 1ull;
    if (tmax > t0) D.ctr->integrate_ticks += tmax - t0;
  }
}

// every store of the calling workgroup drained (each wave's vmcnt(0)), then a workgroup barrier: a
// flag stored after this publishes them (sc1 stores + drained wait + flag, MI355X_MICROARCH.md)
__device__ __forceinline__ void drain_barrier() {
  __builtin_amdgcn_s_waitcnt(0);
  lds_barrier();
}
// one copy of a launch flag per XCD (8 lines), set by an agent-scope atomic exchange: the only
// global_atomic_swap_x2 in k_frame, so tests/test_isa.py can pin that a drained barrier precedes it
__device__ __forceinline__ void publish_flags(unsigned long long* flags, uint32_t tag) {
  if (threadIdx.x < 8)
    (void)__hip_atomic_exchange(flags + 16 * threadIdx.x, (unsigned long long)tag, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------
// The head's fast path (k_frame workgroup 0): frame b - 1's carving and frame b's allocation as the
// commit-all fast paths resolve_delete_fast + resolve_alloc_fast would run them one after the other,
// but with the allocation's inputs -- its new keys, their candidate orders, their buckets, the free
// stack's top -- loaded in the same two round trips as the carving's, before the carving commits.
// The carving changes what the allocation reads in three known ways, applied from LDS instead of
// re-reading: the entries it clears (a key's bucket then has that slot empty), the blocks it pushes on
// the free stack (popped first, in reverse push order) and the keys carved_key would re-insert into
// the new-key set (then this path is not taken). Anything outside both fast paths' conditions returns
// false before a global write, and the sequential resolvers run. Results are identical either way
// (tests/test_gpu_pipeline.py, test_gpu_fullsize.py: the oracle decides).
// ---------------------------------------------------------------------------------------------
#ifdef TSDF_NO_HEAD_FAST
__device__ constexpr bool head_fast_off() { return true; }
#else
__device__ constexpr bool head_fast_off() { return false; }
#endif
constexpr int kHeadCleared = 1024;  // set of the entries the carving clears (<= 2 kRT), open addressing
struct HeadLds {
  uint32_t ev[2 * kRT];         // entries of the released candidates (push rank = number smaller)
  int32_t pushed[2 * kRT];      // pool index pushed at rank r
  uint32_t cleared[kHeadCleared];
  uint32_t lock[kFastLockSlots];  // the allocation's bucket locks
  uint32_t ordv[kRT];           // candidate orders of the owned keys (pop ranks)
  int32_t htop[kRT];            // the free stack's top before the carving: heap[free0 - 1 - i]
  int scan[24];
};
__device__ __forceinline__ void cleared_insert(uint32_t* S, uint32_t e) {
  uint32_t h = mix32(e) & (kHeadCleared - 1);
  for (int p = 0; p < kHeadCleared; ++p) {
    const uint32_t prev = atomicCAS(&S[h], 0u, e + 1u);
    if (prev == 0u || prev == e + 1u) return;
    h = (h + 1) & (kHeadCleared - 1);
  }
}
__device__ __forceinline__ bool cleared_has(const uint32_t* S, uint32_t e) {
  uint32_t h = mix32(e) & (kHeadCleared - 1);
  for (int p = 0; p < kHeadCleared; ++p) {
    const uint32_t v = S[h];
    if (v == e + 1u) return true;
    if (v == 0u) return false;
    h = (h + 1) & (kHeadCleared - 1);
  }
  return false;
}
// Both round trips, the decision, and (when taken) every commit of the carving and the allocation,
// issued together: the two write no common word (an entry the carving clears and a key then takes is
// written by the allocation alone -- the key's full entry supersedes the cleared one, and its occupancy
// bit stays set), so one drain before the two flags orders them (the sequential resolvers drain twice).
// No load follows a store (each counter update is computed from round trip 1's values; a load behind
// the stores would wait for all of them -- gfx950 counts stores in vmcnt). Returns false, with nothing
// written, when the launch is outside the fast paths.
__device__ __forceinline__ bool head_fast(const EngineDev& D, const PipeArgs& A, HeadLds& L) {
  const int t = threadIdx.x, wave = t >> 6;
  TSDF_STAMP(D, 4, 0);
  const unsigned long long tick0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t fcv = A.fid_carve, fo_fid = A.fid_alloc;
  const VisRec* cand = D.cand + (size_t)(fcv & 1u) * (size_t)D.cand_cap;
  const int32_t* ncand = reinterpret_cast<const int32_t*>(D.pipe + kPipeNCand + 16 * (fcv & 1u));
  // ---- round trip 1: both counts, the counters, the candidate records and the new-key list
  const int nc = ld_co(ncand);
  const int na = ld_co(&D.ctr->nk_count);
  const int free0 = D.ctr->free_count;
  const uint32_t epoch0 = D.ctr->lock_epoch;
  const unsigned long long tot_del = D.ctr->total_deleted, tot_alloc = D.ctr->total_alloc;
  const unsigned long long ticks_del = D.ctr->resolve_delete_ticks, ticks_alloc = D.ctr->resolve_alloc_ticks;
  const unsigned long long* rq = reinterpret_cast<const unsigned long long*>(cand);
  const unsigned long long a[2] = {ld_co(&rq[2 * t]), ld_co(&rq[2 * (t + kRT)])};
  const unsigned long long key = ld_co(&D.nk_list[t].key);
  const int32_t slot = (int32_t)ld_co(&D.nk_list[t].slot);
  if (nc > 2 * kRT || na > kRT || free0 < 0) return false;  // (uniform)
  // ---- round trip 2: the candidates' buckets and D.fo words, the keys' orders and buckets, heap top
  int16_t x[2] = {0, 0}, z[2] = {0, 0};
  uint32_t cur[2] = {0u, 0u}, rel_e[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
  int32_t idx[2] = {-1, -1};
  bool bad = false, rel[2] = {false, false};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (t + r * kRT >= nc) continue;
    x[r] = (int16_t)(a[r] & 0xFFFF);
    const int16_t y = (int16_t)((a[r] >> 16) & 0xFFFF);
    z[r] = (int16_t)((a[r] >> 32) & 0xFFFF);
    const uint32_t Ab = hash_block(x[r], y, z[r]);
    const Ent s0 = load_ent(D.table, 2 * Ab), s1 = load_ent(D.table, 2 * Ab + 1);
    const unsigned long long fo0 = D.fo[2 * Ab], fo1 = D.fo[2 * Ab + 1];
    const bool in0 = s0.x == x[r] && s0.y == y && s0.z == z[r] && s0.idx >= 0;
    const bool head = !in0 && s1.x == x[r] && s1.y == y && s1.z == z[r] && s1.idx >= 0 && s1.off == 0;
    bad |= !(in0 || head);
    cur[r] = 2 * Ab + (head ? 1u : 0u);
    idx[r] = in0 ? s0.idx : s1.idx;
    rel[r] = (in0 || head) && local_idx(idx[r]);
    if (rel[r]) rel_e[r] = cur[r];
    // carved_key would put the deleted key back into frame b's new-key set: not this path
    bad |= (uint32_t)((head ? fo1 : fo0) >> 32) == ~fo_fid;
  }
  const bool have = t < na;
  uint32_t B = 0u, ord = 0xFFFFFFFFu;
  int16_t kx = 0, ky = 0, kz = 0;
  Ent sa0{}, sa1{};
  if (have) {
    unpack_key(key, kx, ky, kz);
    B = hash_block(kx, ky, kz);
    ord = ld_co(&D.nk_order[slot]);
    sa0 = load_ent(D.table, 2 * B);
    sa1 = load_ent(D.table, 2 * B + 1);
  }
  const int32_t htop = t < min(na, free0) ? D.heap[free0 - 1 - t] : 0;
  for (int i = t; i < kHeadCleared; i += kRT) L.cleared[i] = 0u;
  for (int i = t; i < kFastLockSlots; i += kRT) L.lock[i] = 0u;
  L.ev[t] = rel_e[0];
  L.ev[t + kRT] = rel_e[1];
  L.htop[t] = htop;
  const unsigned long long bb = __ballot(bad), br0 = __ballot(rel[0]), br1 = __ballot(rel[1]);
  if (lane_id() == 0) {
    L.scan[wave] = __popcll(bb);
    L.scan[4 + wave] = __popcll(br0) + __popcll(br1);
  }
  lds_barrier();  // (sets zero, ev / htop / scan written)
  TSDF_STAMP(D, 4, 3);
  if (L.scan[0] + L.scan[1] + L.scan[2] + L.scan[3] != 0) return false;
  const int nrel = L.scan[4] + L.scan[5] + L.scan[6] + L.scan[7];
#pragma unroll
  for (int r = 0; r < 2; ++r)
    if (t + r * kRT < nc) cleared_insert(L.cleared, cur[r]);
  lds_barrier();  // (the cleared set is complete)
  // ---- the allocation against the carved table (resolve_alloc_fast's conditions)
  const bool c0 = have && cleared_has(L.cleared, 2 * B), c1 = have && cleared_has(L.cleared, 2 * B + 1);
  const bool e0 = sa0.idx < 0 || c0, e1 = sa1.idx < 0 || c1;
  const bool abad = have && (!(e0 || e1) || !lock_take2<kFastLockSlots>(L.lock, B));
  const uint32_t e = 2 * B + (e0 ? 0u : 1u);  // the key's entry
  L.ordv[t] = have ? ord : 0xFFFFFFFFu;  // (one volume: every key is owned)
  const unsigned long long ab = __ballot(abad);
  if (lane_id() == 0) L.scan[8 + wave] = __popcll(ab);
  // an entry the carving clears and a key takes: written by the allocation only (L.lock reused after
  // the barrier below as the set of refilled entries -- the allocation's locks are no longer needed)
  lds_barrier();
  if (L.scan[8] + L.scan[9] + L.scan[10] + L.scan[11] != 0 || na > free0 + nrel) return false;
  for (int i = t; i < kHeadCleared; i += kRT) L.cleared[i] = 0u;
  lds_barrier();
  if (have && ((e0 && c0) || (!e0 && c1))) cleared_insert(L.cleared, e);
  lds_barrier();  // (L.cleared: the refilled entries)
  // ---- taken: the carving's commits (resolve_delete_fast) ...
  const int nq = (min(nc, 2 * kRT) + 3) >> 2;
  const uint4* v4 = reinterpret_cast<const uint4*>(L.ev);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (t + r * kRT >= nc) continue;
    const uint32_t c = cur[r];
    if (!cleared_has(L.cleared, c)) {
      // offset 0 and idx -1 (store_off_idx_co without its read: z and the offset share the dword)
      uint32_t* q = reinterpret_cast<uint32_t*>(&D.table[c]);
      st_co(&q[1], (uint32_t)(uint16_t)z[r]);
      st_co(&q[2], 0xFFFFFFFFu);
      atomicAnd(&D.occ[c >> 6], ~(1ull << (c & 63)));
    }
    mark_swept_dirty(D, c);
    if (rel[r]) {  // ReleaseBlock in entry order among the released blocks (entries are unique)
      int rank = 0;
#pragma unroll 2
      for (int j = 0; j < nq; ++j) {
        const uint4 v = v4[j];
        rank += (v.x < c) + (v.y < c) + (v.z < c) + (v.w < c);
      }
      D.heap[free0 + rank] = idx[r];
      L.pushed[rank] = idx[r];
      st_co(&D.rtag[idx[r]], fcv);
    }
  }
  lds_barrier();  // (L.pushed)
  TSDF_STAMP(D, 4, 4);
  const unsigned long long tick1 = __builtin_amdgcn_s_memrealtime();
  // ---- ... and the allocation's (resolve_alloc_fast): pops from the carving's pushes first, then the
  // prefetched top of the stack
  if (have) {
    int prank = 0;  // keys earlier in candidate order (orders are unique per key)
    const uint4* o4 = reinterpret_cast<const uint4*>(L.ordv);
    const int nq2 = (na + 3) >> 2;
#pragma unroll 2
    for (int j = 0; j < nq2; ++j) {
      const uint4 v = o4[j];
      prank += (v.x < ord) + (v.y < ord) + (v.z < ord) + (v.w < ord);
    }
    const int32_t bi = prank < nrel ? L.pushed[nrel - 1 - prank] : L.htop[prank - nrel];
    store_ent_co(D.table, e, kx, ky, kz, 0, bi);
    mark_swept_dirty(D, e);
    atomicOr(&D.occ[e >> 6], 1ull << (e & 63));
    VisRec vr;
    vr.x = kx;
    vr.y = ky;
    vr.z = kz;
    vr.pad = 1;
    vr.idx = bi;
    vr.entry = (int32_t)e;
    st_rec_co(&D.fresh_vis[prank], vr);
    st_co(&D.nk_key[slot], 0ull);
    st_co(&D.nk_order[slot], 0xFFFFFFFFu);
  }
  if (t == 0) {
    const unsigned long long tick2 = __builtin_amdgcn_s_memrealtime();
    D.ctr->lock_epoch = epoch0 + 2u;  // (the carving's launch, then the allocation's)
    D.ctr->free_count = free0 + nrel - na;
    D.ctr->last_deleted = nrel;
    D.ctr->total_deleted = tot_del + (unsigned long long)nrel;
    D.ctr->resolve_delete_ticks = ticks_del + (tick1 - tick0);
    D.ctr->resolve_alloc_ticks = ticks_alloc + (tick2 - tick1);
    st_co(&D.ctr->n_fresh, na);
    st_co(&D.ctr->nk_count, 0);
    D.ctr->last_alloc = na;
    D.ctr->last_new_keys = na;
    D.ctr->total_alloc = tot_alloc + (unsigned long long)na;
  }
  TSDF_STAMP(D, 1, 5);
  return true;
}

// an update workgroup's LDS (pipe_update)
struct PipeUpdLds {
  int upd[4], vis[4];
  int ncand;
  VisRec cand[kIntegrateCandBuf];
  VisRec def[kPipeDefer];
  VisRec list[kPipeList];
  int n, ndef;
  float pmin[2 * kPipeList];
  int pdone[kPipeList];
  uint32_t fb;
};
// one allocation for the launch's parts (a workgroup runs one part)
union FrameLds {
  DeleteLds del;
  IngestLds<1024> ing;
  HeadLds head;
  PipeUpdLds upd;
};

__device__ __forceinline__ void merge_cands_inbox(const EngineDev& D, VisRec* cand, int32_t* ncand, const ShardRec* __restrict__ cands_in,
                                  int cap, int nshard, int* s_base);

// workgroup 0: frame fid_carve's carving, then frame fid_alloc's allocation, each published. A shard's
// pipelined frame first lists every shard's candidates of fid_carve (the all-gathered inbox).
__device__ __forceinline__ void pipe_head(const EngineDev& D, const FrameParams& Pu, const PipeArgs& A, FrameLds& U) {
  __shared__ int s_base[kMaxShards + 1];
  const int t = threadIdx.x;
  // one volume's carving + allocation: the combined fast path (head_fast) when the launch is within it:
  // both commit before one drain, then both flags
  bool fast = false;
  if (A.has_carve && A.has_alloc && !A.cands_in && !A.cands_out && !resolve_fast_off() && !head_fast_off()) {
    fast = head_fast(D, A, U.head);
    if (!fast) lds_barrier();  // (the sequential resolvers below reuse the LDS)
  }
  if (A.has_carve) {  // (the view's pointers as scalars: a copied EngineDev view can land in scratch)
    const uint32_t f = A.fid_carve;
    VisRec* cand = D.cand + (size_t)(f & 1u) * (size_t)D.cand_cap;
    int32_t* ncand = reinterpret_cast<int32_t*>(D.pipe + kPipeNCand + 16 * (f & 1u));
    if (!fast) {
      if (A.cands_in) merge_cands_inbox(D, cand, ncand, A.cands_in, A.cand_cap, A.nshard, s_base);
      resolve_delete_wg(D, cand, ncand, 0, U.del, f, A.has_alloc ? A.fid_alloc : 0u);
    }
    lds_barrier();
    // the carved frame's candidate count and band counts start empty for frame fid_carve + 2 / + 3
    if (t < kBands) st_co(&D.band[(size_t)(f % 3u) * kBands * kBandStride + t * kBandStride], 0);
    if (t == 0) st_co(ncand, 0);
  }
  // (a shard: the owned entries this launch's allocation leaves without voxels are listed from here;
  // without an allocation the list is the last one's, packed by this launch's update)
  if (t == 0 && A.cands_out && A.has_alloc) st_co(&D.ctr->n_pend, 0);
  if (!fast) {
    drain_barrier();
    publish_flags(D.pipe + kPipeCarved, A.tag);
    TSDF_STAMP_WG(D, 8, 0, 3);
    if (A.has_alloc) resolve_alloc_wg(D, Pu, A.range, 1, U.ing.u.res);
  }
  drain_barrier();
  const unsigned long long t_pub = __builtin_amdgcn_s_memrealtime();
  if (fast) {
    publish_flags(D.pipe + kPipeCarved, A.tag);
    TSDF_STAMP_WG(D, 8, 0, 3);
  }
  publish_flags(D.pipe + kPipeAlloc, A.tag);
  TSDF_STAMP_WG(D, 8, 0, 4);
  if (t == 0) {
    D.pipe[kPipeAPub + 16 * (A.fid_new & 1u)] = t_pub;
    if (A.has_alloc) {  // frame fid_alloc's ingest span (last launch): allocation flag -> last tile / sweep end
      unsigned long long* ie = D.pipe + kPipeIngEnd + 16 * (A.fid_alloc & 1u);
      const unsigned long long a0 = D.pipe[kPipeAPub + 16 * (A.fid_alloc & 1u)], a1 = *ie;
      if (a1 > a0) D.ctr->ingest_ticks += a1 - a0;
      *ie = 0ull;
    }
  }
  if (A.has_carve) pipe_frame_stats(D, A.fid_carve);  // off the chain
}

// One update workgroup of frame b (Db = frame_view(D, b), b = A.fid_alloc). kind 0: b's listed blocks
// (its band lists, then its fresh list when it was built by an earlier launch), XCD-split like
// k_integrate; kind 1 (workgroup wi of kPipeFreshWG): the blocks this launch's allocation creates,
// after its flag. Frame b - 1's carve candidates among the listed blocks (ctag) are deferred to the
// end of the workgroup's work, after the carving flag, and updated unless the carving released them
// (rtag); more than kPipeDefer of them: the workgroup waits for the carving at once.
// The work alternates between collecting up to kPipeList records into LDS (the list walk, the tag
// tests, the waits) and updating them in a loop that does nothing else: the walk's scalar state then
// stays out of the update loop, whose scalar registers are the camera and the pool's (in one loop the
// two spilled ~230 SGPRs to VGPR lanes, read back in every block's update).
// a candidate of frame fc the carving has run for: kept unless released (one lane's atomic read: rtag
// was written through by workgroup 0 on another XCD)
__device__ __forceinline__ bool pipe_kept(uint32_t* rtag, int32_t idx, uint32_t fc, int lane) {
  uint32_t v = 0u;
  if (lane == 0) v = __hip_atomic_fetch_or(&rtag[idx], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint32_t)__builtin_amdgcn_readfirstlane(v) != fc;
}
// wave_wait_tag: wait_tag for one wave (lane 0 polls; no workgroup barrier)
__device__ __forceinline__ void wave_wait_tag(const unsigned long long* flag, uint32_t tag, uint32_t* status) {
  if (lane_id() == 0) {
    uint32_t n = 0;
    while ((uint32_t)__hip_atomic_fetch_or(const_cast<unsigned long long*>(flag), 0ull, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) != tag) {
      __builtin_amdgcn_s_sleep(TSDF_PIPE_SLEEP);
      if (++n > (1u << 22)) {
        atomicOr(status, 64u);  // TSDF_STATUS_PIPELINE_TIMEOUT
        break;
      }
    }
  }
}
// pipe_kept for one record per lane (each lane's own atomic read of its block's release tag)
__device__ __forceinline__ bool lane_kept(uint32_t* rtag, int32_t idx, uint32_t fc) {
  return __hip_atomic_fetch_or(&rtag[idx], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != fc;
}
// (D: the base view; frame b's lists are addressed through scalar pointers here -- an EngineDev view
// copied by value, or captured by reference in a lambda, can be materialised in scratch)
__device__ __forceinline__ void pipe_update(const EngineDev& D, const FrameParams& P, const PipeArgs& A, int kind, int wi,
                                            PipeUpdLds& L) {
  int* s_upd = L.upd;
  int* s_vis = L.vis;
  int& s_ncand = L.ncand;
  VisRec* s_cand = L.cand;  // this workgroup's carve candidates
  VisRec* s_def = L.def;    // deferred (candidate of frame b - 1) blocks
  VisRec* s_list = L.list;  // the records of one collection
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave >> 1, hf = wave & 1;
  const bool t0 = threadIdx.x == 0;
  const uint32_t fb = A.fid_alloc, fc = A.fid_carve;
  // frame b's view (frame_view)
  const VisRec* vis = D.vis + (size_t)(fb & 1u) * kBands * (size_t)D.nblocks;
  VisRec* cand = D.cand + (size_t)(fb & 1u) * (size_t)D.cand_cap;
  int32_t* ncand = reinterpret_cast<int32_t*>(D.pipe + kPipeNCand + 16 * (fb & 1u));
  const unsigned long long* carved = D.pipe + kPipeCarved + (blockIdx.x & 7) * 16;
  if (t0) s_ncand = 0;  // (ordered before its first use by the loop's barriers)
  if (kind == 0 && wi == 0 && t0)  // the update's device-clock start
    st_co(D.pipe + kPipeT0 + 16 * (fb & 1u), (unsigned long long)__builtin_amdgcn_s_memrealtime());
  int bst = 0;
  int nvis = 0, nband = 0, p = 0, p_hi = 0, pstep = 1;
  bool carved_known = false;
  // order 3: the whole update after the allocation flag -- no update traffic beside the head's
  // carving and allocation (their chains of dependent round trips stretch ~4x under it), the new
  // blocks listed after the band lists, and no deferral (the head publishes the carving first)
  const bool after_alloc = kind == 0 && A.order >= 3;
  if (kind == 0) {
    if (after_alloc) {
      wait_tag(D.pipe + kPipeAlloc + (blockIdx.x & 7) * 16, A.tag, &D.ctr->status);
      carved_known = true;
    }
    bst = band_starts_p(D.band + (size_t)(fb % 3u) * kBands * kBandStride, lane, &nvis);
    nband = nvis;
    if (A.fresh_ready) nvis += D.ctr->n_fresh;
    else if (after_alloc) nvis += ld_co(&D.ctr->n_fresh);
    // group g = blockIdx % 8 (one XCD) takes the g-th contiguous eighth of the pairs in band order
    // (a compact image region: its pixel records stay in that XCD's L2). (Measured and not kept:
    // pairs taken from 8 per-XCD queues by atomics, two at a time -- the update span grew 28 -> 38 us.)
    const int g = wi & 7, npairs = (nvis + 1) >> 1;
    p = (int)(((long long)npairs * g) >> 3) + (wi >> 3);
    p_hi = (int)(((long long)npairs * (g + 1)) >> 3);
    pstep = A.nint >> 3;
  } else {
    wait_tag(D.pipe + kPipeAlloc + (blockIdx.x & 7) * 16, A.tag, &D.ctr->status);
    nvis = ld_co(&D.ctr->n_fresh);
    p = wi;
    p_hi = (nvis + 1) >> 1;
    pstep = kPipeFreshWG;
  }
  const bool chk = A.has_carve && kind == 0;
  const uint32_t* ct = D.ctag + (size_t)(fc & 1u) * D.nblocks;
  int my_upd = 0, my_vis = 0, ndef = 0;
  bool def_done = false;
  const bool fresh_co = kind != 0 || (after_alloc && !A.fresh_ready);  // (written in this launch)
  // the collection is wave 0's: one record per lane (its list record and candidate tag gathered
  // together, two dependent round trips per collection instead of two per record), compacted into
  // s_list by ballot; the deferred candidates' release tags likewise one per lane
  int& s_n = L.n;
  int& s_ndef = L.ndef;
  float* s_pmin = L.pmin;  // the two halves' carve minima of each collected record
  int* s_pdone = L.pdone;  // halves of the record done
  uint32_t& s_fb = L.fb;   // fb for the candidate path (read from LDS: in a register the
                           // frame id was spilled to scratch, reloaded behind a vmcnt(0))
  if (t0) s_fb = fb;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  if (t0) s_ndef = 0;  // (ordered before its first read by the loop's barrier)
  for (;;) {  // (all control flow below is workgroup-uniform; thread 0 writes the LDS lists)
    // ---- collect: the next records of the list walk, or (at its end) the deferred ones
    int n = 0;
    lds_barrier();  // (every wave has read the previous collection's s_n / s_ndef)
    if (p < p_hi) {
      const int npr = min((p_hi - p + pstep - 1) / pstep, kPipeList / 2);  // pairs in this collection
      if (wave == 0) {
        const int b = 2 * (p + (lane >> 1) * pstep) + (lane & 1);
        const bool valid = lane < 2 * npr && b < nvis;
        // the band of list index b: the last band whose start is <= b (starts non-decreasing)
        int bd = 0, bs = 0;
#pragma unroll
        for (int k = 1; k < kBands; ++k) {
          const int sk = __builtin_amdgcn_readlane(bst, k);
          if (b >= sk) {
            bd = k;
            bs = sk;
          }
        }
        VisRec r{};
        if (valid) {
          if (b >= nband)
            r = fresh_co ? ld_rec_co(&D.fresh_vis[b - nband]) : D.fresh_vis[b - nband];
          else
            r = vis[(size_t)bd * D.nblocks + (size_t)(b - bs)];
        }
        const bool cand = valid && chk && r.pad == 0 && ct[r.idx] == fc;  // a candidate of frame b - 1
        bool take = valid && !cand;
        const unsigned long long cm = __ballot(cand);
        if (cm) {
          const int nc = __popcll(cm);
          if (!carved_known && ndef + nc <= kPipeDefer) {  // deferred to the end
            if (cand) s_def[ndef + __popcll(cm & lt_mask)] = r;
            ndef += nc;
          } else {
            if (!carved_known) wave_wait_tag(carved, A.tag, &D.ctr->status);
            carved_known = true;
            if (cand) take = lane_kept(D.rtag, r.idx, fc);
          }
        }
        const unsigned long long tm = __ballot(take);
        if (take) s_list[__popcll(tm & lt_mask)] = r;
        s_pdone[lane] = 0;
        if (lane == 0) {
          s_n = __popcll(tm);
          s_ndef = ndef;
        }
      }
      p += npr * pstep;
    } else if (!def_done && s_ndef > 0) {  // (s_ndef: read before the next collection's barrier)
      if (wave == 0) {
        if (!carved_known) wave_wait_tag(carved, A.tag, &D.ctr->status);
        carved_known = true;
        bool take = false;
        VisRec r{};
        if (lane < ndef) {
          r = s_def[lane];
          take = lane_kept(D.rtag, r.idx, fc);
        }
        const unsigned long long tm = __ballot(take);
        if (take) s_list[__popcll(tm & lt_mask)] = r;
        s_pdone[lane] = 0;
        if (lane == 0) s_n = __popcll(tm);
      }
      def_done = true;
    } else {
      break;
    }
    lds_barrier();  // (publishes s_list, s_n, s_ndef)
    n = s_n;
#ifdef TSDF_DIAG_STAMPS
    if (t0 && D.dbg && blockIdx.x < (unsigned)kDiagMaxWg) {  // collect ends: first (3), last (4); records (5)
      unsigned long long* q = D.dbg + ((size_t)8 * kDiagMaxWg + blockIdx.x) * kDiagStamps;
      const unsigned long long tnow = __builtin_amdgcn_s_memrealtime();
      if (q[5] == 0ull) q[3] = tnow;
      q[4] = tnow;
      q[5] += (unsigned long long)n + 1ull;
    }
#endif
    // ---- update: the two pairs of waves take records pair, pair + 2, ...; no workgroup barrier: the
    // two waves of a record combine their carve minima through LDS (the second to finish decides), so
    // every wave runs its records at its own pace and one wave's memory waits overlap the others' work
    for (int k = pair; k < n; k += 2) {
      const VisRec r = s_list[k];
      float mn = __builtin_inff();
      update_block<false>(D, P, r, lane, hf, mn, my_upd);
      my_vis += hf == 0 ? 1 : 0;
      mn = wave_min_u(mn);
      if (lane == 0) {
        s_pmin[2 * k + hf] = mn;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // (LDS only: pool stores stay in flight)
        if (atomicAdd(&s_pdone[k], 1) == 1) {  // the record's other half is done too
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
          const float m2 = fminf(mn, s_pmin[2 * k + (hf ^ 1)]);
          if (m2 >= 0.9f) {  // space_carving_kernel threshold (voxel_tsdf.cu:227, :485)
            const uint32_t f = s_fb;
            D.ctag[(size_t)(f & 1u) * D.nblocks + r.idx] = f;  // (read by the next launch's update)
            const int kc = atomicAdd(&s_ncand, 1);
            if (kc < kIntegrateCandBuf) {
              s_cand[kc] = r;
            } else {  // buffer full (heavy carving): this one now
              const int kg = atomicAdd(ncand, 1);
              if (kg < D.cand_cap) st_rec_co(&cand[kg], r);
              else atomicOr(&D.ctr->status, 16u);  // (a list longer than the pool: internal error)
            }
          }
        }
      }
    }
  }
  // the workgroup's carve candidates (read by the next launch's carving) and statistics
  const int tot = wave_sum(my_upd);
  if (lane == 0) {
    s_upd[wave] = tot;
    s_vis[wave] = my_vis;
  }
  lds_barrier();
  const int nc = min(s_ncand, kIntegrateCandBuf);
  if (wave == 0 && nc > 0) {
    int k0 = 0;
    if (lane == 0) k0 = atomicAdd(ncand, nc);
    k0 = __shfl(k0, 0, 64);
    if (lane < nc && k0 + lane < D.cand_cap) st_rec_co(&cand[k0 + lane], s_cand[lane]);
  }
  if (t0) {
    const unsigned long long upd = (unsigned long long)(s_upd[0] + s_upd[1] + s_upd[2] + s_upd[3]);
    const unsigned long long nv = (unsigned long long)(s_vis[0] + s_vis[1] + s_vis[2] + s_vis[3]);
    unsigned long long* st = D.pipe + kPipeStats + (size_t)(fb & 1u) * (kPipeStatLines * 16) +
                             (blockIdx.x % kPipeStatLines) * 16;
    if (nv | upd) atomicAdd(st, (nv << 40) | upd);
    atomicMax(st + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
  if (A.cands_out) {  // a shard's pipelined frame: the last update workgroup fills the exchange slot
    __shared__ int s_last;
    const int nold = A.nint, nfr = pipe_fresh_wgs(A);
    const uint32_t idx = (uint32_t)(kind ? nold + wi : wi);  // (this workgroup among the update's)
    if (arrive_last(D.arrive + kArrIntegrate, 0ull, &s_last, true, (uint32_t)(nold + nfr), idx)) {
      if (t0) arrive_reset(D.arrive + kArrIntegrate);
      pack_cands_wg(D, cand, ncand, A.cands_out, A.cand_cap, A.cands_dst, A.ndst);
    }
  }
}

#ifndef TSDF_FRAME_WAVES
#define TSDF_FRAME_WAVES TSDF_INTEGRATE_WAVES
#endif
// grid: kPipeHead head workgroups (0: carving + allocation), A.nint update workgroups (listed blocks),
// kPipeFreshWG (this launch's new blocks), then frame c's A.tiles pixel tiles and kVisWorkgroups
// sweep workgroups -- each part only when the launch has it
// (diagnostic build: each workgroup's part code, start and end into D.dbg kernel 8 -- 1 head, 2 fresh
// update, 3 listed update, 4 tile, 5 sweep; the head's carving / allocation ends at 3 / 4)
// Wave priorities of the parts (s_setprio: the SIMD's issue arbitration among its waves): the head
// (carving and allocation, which the fresh updates and the tiles' probes wait for) highest, the
// update (the launch's critical path) next, the tiles and the sweep lowest. Driver command, same
// box, interleaved (scripts/ab.sh lib, 4 runs each): 22.63k frames/s against 22.36k without
// priorities; head 3 / update 3 and head 3 / update 1 alike within noise; tiles above the update
// 19.6-19.9k. Experiment builds override them (-DTSDF_PRIO_HEAD=0 ...; 0 = no s_setprio).
#ifndef TSDF_PRIO_HEAD
#define TSDF_PRIO_HEAD 3
#endif
#ifndef TSDF_PRIO_UPD
#define TSDF_PRIO_UPD 2
#endif
#ifndef TSDF_PRIO_TILE
#define TSDF_PRIO_TILE 0
#endif
__device__ __forceinline__ int frame_part(const EngineDev& D, const FrameParams& Pu, const FrameParams& Pn,
                                          const PipeArgs& A, FrameLds& U) {
  int w = (int)blockIdx.x;
  if (w < kPipeHead) {
    if (w != 0) return 0;
    if (TSDF_PRIO_HEAD) __builtin_amdgcn_s_setprio(TSDF_PRIO_HEAD);
    pipe_head(D, Pu, A, U);
    return 1;
  }
  w -= kPipeHead;
  if (A.order == 4)  // every part after the head's carving and allocation
    wait_tag(D.pipe + kPipeAlloc + (blockIdx.x & 7) * 16, A.tag, &D.ctr->status);
  const int nfr = pipe_fresh_wgs(A);
  if (w < nfr) {  // the blocks this launch's allocation creates (they wait for it: dispatched early)
    if (TSDF_PRIO_UPD) __builtin_amdgcn_s_setprio(TSDF_PRIO_UPD);
    pipe_update(D, Pu, A, 1, w, U.upd);
    return 2;
  }
  w -= nfr;
  // the other parts in the launch's grid order: update (u), tiles (t), sweep (s)
  const int nold = A.has_update ? A.nint : 0, ns = A.has_frame ? kVisWorkgroups : 0;
  // (order r runs the parts r, r + 1, r + 2 mod 3; scalar selects, no indexed arrays: those live in
  // scratch)
  int part = -1, o = w;
  const int ord = A.order == 3 ? 1 : (A.order == 4 ? 0 : A.order);
  for (int k = 0; k < 3; ++k) {
    const int q = (ord + k) % 3;
    const int nq = q == 0 ? nold : (q == 1 ? A.tile_wgs : ns);
    if (o < nq) {
      part = q;
      break;
    }
    o -= nq;
  }
  if (part < 0) return 0;  // (a graph's grid is sized for the largest launch)
  if (part == 0) {
    // (its XCD split takes o % 8 as the XCD: exact when the parts before it are multiples of 8 long,
    // as at 640x480; correct either way)
    if (TSDF_PRIO_UPD) __builtin_amdgcn_s_setprio(TSDF_PRIO_UPD);
    pipe_update(D, Pu, A, 0, o, U.upd);
    return 3;
  }
  if (TSDF_PRIO_TILE) __builtin_amdgcn_s_setprio(TSDF_PRIO_TILE);
  const unsigned long long* aflag = D.pipe + kPipeAlloc + (blockIdx.x & 7) * 16;
  if (part == 1) {
    // tiles_per_wg consecutive tiles per workgroup (TSDF_FRAME_TILES_PER_WG; 1 shipped): with 2 every
    // tile workgroup is resident beside the update from the start, but its tiles run one after the
    // other -- driver 22.2k frames/s against 23.2k at 1 (3: 20.4k, 4: 18.1k; same box)
    const int t0 = o * A.tiles_per_wg, t1 = min(A.tiles, t0 + A.tiles_per_wg);
    for (int t = t0; t < t1; ++t) {
      if (t != t0) __syncthreads();  // (the previous tile's probes read the LDS key set)
      ingest_tile<1024, kTileChained>(D, Pn, Pn.depth, Pn.rgb, Pn.ht, Pn.lt, A.tiles_x, t, U.ing, aflag, A.tag,
                                      A.fid_new);
    }
  } else
    vis_sweep_chained<1024>(frame_view(D, A.fid_new), Pn, o, U.ing, aflag, A.tag);
  if (threadIdx.x == 0)  // the ingest's span ends with its last workgroup
    atomicMax(D.pipe + kPipeIngEnd + 16 * (A.fid_new & 1u), (unsigned long long)__builtin_amdgcn_s_memrealtime());
  return 3 + part;
}
__device__ __forceinline__ void frame_body(const EngineDev& D, const FrameParams& Pu, const FrameParams& Pn,
                                           const PipeArgs& A, FrameLds& U) {
#ifdef TSDF_DIAG_STAMPS
  const unsigned long long d_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int code = frame_part(D, Pu, Pn, A, U);
#ifdef TSDF_DIAG_STAMPS
  if (threadIdx.x == 0 && D.dbg && blockIdx.x < (unsigned)kDiagMaxWg) {
    unsigned long long* q = D.dbg + ((size_t)8 * kDiagMaxWg + blockIdx.x) * kDiagStamps;
    q[0] = (unsigned long long)code;
    q[1] = d_t0;
    q[2] = __builtin_amdgcn_s_memrealtime();
  }
#else
  (void)code;
#endif
}
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_FRAME_WAVES, TSDF_FRAME_WAVES))) void k_frame(
    EngineDev D, FrameParams Pu, FrameParams Pn, PipeArgs A) {
  __shared__ FrameLds U;
  frame_body(D, Pu, Pn, A, U);
}
// the graph-captured form: its arguments from the FrameArgs block the graph's first node uploads
__global__ __launch_bounds__(kIntegrateThreads)
__attribute__((amdgpu_waves_per_eu(TSDF_FRAME_WAVES, TSDF_FRAME_WAVES))) void k_frame_g(
    EngineDev D, const FrameArgs* __restrict__ FA) {
  __shared__ FrameLds U;
  const PipeArgs A = FA->pipe;
  const FrameParams Pu = FA->Pu, Pn = FA->P;
  frame_body(D, Pu, Pn, A, U);
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
// every shard's candidate slot (nshard slots of cap records) listed as D.cand / *D.ncand: the candidate
// set of one volume, so that every shard's index takes the same deletes
__device__ __forceinline__ void merge_cands_inbox(const EngineDev& D, VisRec* cand, int32_t* ncand, const ShardRec* __restrict__ cands_in,
                                  int cap, int nshard, int* s_base) {
  if (threadIdx.x == 0) {
    // the union is listed in cand (D.cand_cap records; the resolver's D.pairs scratch holds at
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
    st_co(ncand, run);
    if (ovf) atomicOr(&D.ctr->status, 16u);  // TSDF_STATUS_SHARD_OVERFLOW
  }
  __syncthreads();
  unsigned long long* cq = reinterpret_cast<unsigned long long*>(cand);
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
__device__ __forceinline__ void resolve_delete_merged(EngineDev D, const VisRec* __restrict__ recs,
                                                      const int32_t* __restrict__ count, int direct,
                                                      const ShardRec* __restrict__ cands_in, int cap,
                                                      int nshard) {
  __shared__ DeleteLds L;
  __shared__ int s_base[kMaxShards + 1];
  if (cands_in) merge_cands_inbox(D, D.cand, D.ncand, cands_in, cap, nshard, s_base);
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
  resolve_delete_merged(D, D.cand, D.ncand, 0, A->cands_in, A->cand_cap, A->nshard);
}


}  // namespace tsdf
