// tsdf_fuse.hip -- the fused integrate kernel and the space-carving resolver.
#include "tsdf_block.h"
#include "tsdf_kernels.h"

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

// 64 VGPRs: 8 waves per SIMD (65 without the bound: 7). Graph: the graph-captured form reads its
// camera from the FrameArgs block the graph's first node uploads.
// The visible blocks are the sweep's band lists (blocks that existed before the frame) followed by
// the blocks k_resolve_alloc created (D.fresh_vis, flagged fresh).
template <bool Graph>
__global__ __launch_bounds__(kIntegrateThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_integrate_t(
    EngineDev D, FrameParams Pv, const FrameArgs* __restrict__ A) {
  const FrameParams P = Graph ? A->P : Pv;
  __shared__ float s_min[4];
  __shared__ int s_upd[4];
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
  const int g = blockIdx.x & 7, ngrp = gridDim.x >> 3;
  const int rx0 = (lane & 1) * 4, ry = (lane >> 1) & 7, rz = (lane >> 4) + 4 * hf;
  const int off = (hf * 256 + lane * 4) * 4;
  const float neg_trunc = -P.trunc;
  int my_upd = 0;
  TSDF_STAMP(D, 3, 0);
  // device-clock duration of this launch: start stamp by WG 0 (dispatched first), end stamp per WG;
  // k_resolve_delete takes the max (bench cross-check of the HIP-event timing)
  if (blockIdx.x == 0 && threadIdx.x == 0) D.wg_end[2 * kIntegrateGrid] = __builtin_amdgcn_s_memrealtime();
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
          px[j] = D.pixA[img];
          lg[j] = D.pixB[img];
#endif
        }
      }
      // ---- pass 2: tsdf_integrate_kernel's update (voxel_tsdf.cu:174-203), branch-free on
      // packed pairs; each voxel's result is kept only where it is updated (the reference's
      // conditions: in image, 0 < d <= max_depth, sdf > -trunc).
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j0 = 2 * k, j1 = 2 * k + 1;
        const v2f d = v2(px[j0].x, px[j1].x), rng = v2(px[j0].y, px[j1].y);
        const v2f w_new = v2(px[j0].z, px[j1].z);
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
      if (upd_mask || fresh) {
#endif
        pool_st(blk + off, ts);
        pool_st(blk + kProbOffset + off, pr);
        pool_stu(blk + kRgbwOffset + off, cw);
      }
      my_upd += __popc(upd_mask);
    }
    mn = wave_min(mn);
    if (lane == 0) s_min[wave] = mn;
    __syncthreads();
    if (hf == 0 && lane == 0 && b < nvis) {
      const float m2 = fminf(s_min[wave], s_min[wave + 1]);
      if (m2 >= 0.9f) {  // space_carving_kernel threshold (voxel_tsdf.cu:227, :485)
        const int k = atomicAdd(&D.ctr->n_cand, 1);
        D.cand[k] = r;
      }
    }
    __syncthreads();
  }
  // updated-voxel count: one plain store per workgroup, summed by k_resolve_delete (no atomics)
  const int tot = wave_sum(my_upd);
  if (lane == 0) s_upd[wave] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    D.wg_upd[blockIdx.x] = s_upd[0] + s_upd[1] + s_upd[2] + s_upd[3];
    D.wg_end[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  }
  TSDF_STAMP(D, 3, 1);
}
template __global__ void k_integrate_t<false>(EngineDev, FrameParams, const FrameArgs*);
template __global__ void k_integrate_t<true>(EngineDev, FrameParams, const FrameArgs*);

// ---------------------------------------------------------------------------------------------
// k_resolve_delete: VoxelHashTable::Delete (voxel_hash.cu:122-171) for every carve candidate in
// hash-entry order (the reference deletes from the entry-ordered visible list). Slot-0 deletes are
// lock free and touch only their own entry; list-head / list-element deletes lock the key's
// bucket and only the first of them per bucket proceeds. The two kinds modify disjoint entries,
// so a whole 1024-candidate round commits at once; ReleaseBlock's stack order is a prefix sum.
// direct: the test path -- recs[0..*count) are keys in list order, one key per round.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kResolveThreads) void k_resolve_delete(EngineDev D,
                                                                    const VisRec* __restrict__ recs,
                                                                    const int32_t* __restrict__ count,
                                                                    int direct) {
  __shared__ ResolveLds L;
  __shared__ unsigned long long s_te[kResolveThreads / 64];
  const int t = threadIdx.x;
  TSDF_STAMP(D, 4, 0);
  // every global value the prologue needs is loaded up front, so they share one memory round
  // trip instead of four dependent ones (counters, per-workgroup sums, candidate count)
  const int n = *count;
  uint32_t epoch0 = 0u;
  int free0 = 0;
  unsigned long long t_start = 0ull;
  int nfresh = 0;
  if (t == 0) {
    epoch0 = D.ctr->lock_epoch;
    free0 = D.ctr->free_count;
    if (!direct) {
      t_start = D.wg_end[2 * kIntegrateGrid];
      nfresh = D.ctr->n_fresh;
    }
  }
  int u = 0, bc = 0;
  unsigned long long te = 0ull;
  if (!direct) {  // voxels updated by both k_integrate launches: sum of their per-workgroup counts
    for (int i = t; i < D.integrate_grid; i += kResolveThreads) {
      u += D.wg_upd[i];
      te = max(te, D.wg_end[i]);  // device clock of the main launch
    }
    if (t < kBands) bc = D.band[t * kBandStride];  // visible = listed by the sweep + created
  }
  claims_clear(L);
  if (t == 0) {
    L.epoch = epoch0 + 1;
    D.ctr->lock_epoch = L.epoch;
    L.sfree = free0;
    L.nalloc = 0;  // deletions
  }
  if (!direct) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) te = max(te, (unsigned long long)__shfl_xor(te, o, 64));
    if ((t & 63) == 0) s_te[t >> 6] = te;
    int tot, nband;
    (void)block_excl_scan(u, L.scan, &tot);  // (its barriers also publish s_te)
    (void)block_excl_scan(bc, L.scan, &nband);
    if (t == 0) {
      unsigned long long tend = 0ull;
      for (int w = 0; w < kResolveThreads / 64; ++w) tend = max(tend, s_te[w]);
      D.ctr->last_updated = (unsigned long long)tot;
      D.ctr->integrate_ticks += tend - t_start;
      D.ctr->n_vis = nband + nfresh;
    }
  }
  __syncthreads();
  auto keyf = [&](int i) -> uint32_t { return (uint32_t)recs[i].entry; };
  const int width = direct ? 1 : stream_prepare(L, n, kNumEntry, keyf);
  const int nbatch = direct ? n : (n <= kBatch ? (n > 0 ? 1 : 0) : ((n - 1) >> 10) + 1);
  TSDF_STAMP(D, 4, 1);
  for (int j = 0; j < nbatch; ++j) {
    int m;
    if (direct) {
      if (t == 0) L.batch[0] = (unsigned long long)(uint32_t)j;
      m = 1;
      __syncthreads();
    } else {
      m = stream_batch(L, n, width, j, keyf);
    }
    for (int base = 0; base < m; base += kResolveThreads) {
      const bool have = base + t < m;
      int kind = 0;  // 1 slot 0, 2 list head, 3 list element
      uint32_t A = 0, prev = 0, cur = 0;
      Ent ecur = {}, eprev = {};
      if (have) {
        const VisRec r = recs[(int)(L.batch[base + t] & 0xFFFFFFFFu)];
        A = hash_block(r.x, r.y, r.z);
        const Ent s0 = load_ent(D.table, 2 * A);
        if (s0.x == r.x && s0.y == r.y && s0.z == r.z && s0.idx >= 0) {
          kind = 1;
          cur = 2 * A;
          ecur = s0;
        } else {
          const Ent hd = load_ent(D.table, 2 * A + 1);
          if (hd.x == r.x && hd.y == r.y && hd.z == r.z && hd.idx >= 0) {
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
              if (bc.x == r.x && bc.y == r.y && bc.z == r.z && bc.idx >= 0) {
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
        if (kind >= 2) claim(L, A, (uint32_t)t);
      }
      __syncthreads();
      bool ok = false;
      int32_t released = -1;
      if (kind == 1) {
        ok = true;
      } else if (kind >= 2 && claim_winner(L, A) == (uint32_t)t) {
        ok = D.lock_tag[A] != L.epoch;
        D.lock_tag[A] = L.epoch;
      }
      if (ok) {
        if (kind == 1) {  // voxel_hash.cu:126-135
          released = ecur.idx;
          store_off_idx(D.table, cur, 0, -1);
        } else if (kind == 2) {  // :137-152 (cur aliases the head when the list is empty)
          released = eprev.idx;
          const int16_t noff = ecur.off ? (int16_t)(eprev.off + ecur.off) : (int16_t)0;
          store_ent(D.table, prev, ecur.x, ecur.y, ecur.z, noff, ecur.idx);
          store_off_idx(D.table, cur, 0, -1);
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
          store_off(D.table, prev, noff);
          store_off_idx(D.table, cur, 0, -1);
        }
        atomicAnd(&D.occ[cur >> 6], ~(1ull << (cur & 63)));
      }
      // ReleaseBlock (voxel_mem.cu:54-59) of the blocks this engine holds (a shard deletes every
      // shard's candidates from its index, and releases only its own pool blocks)
      const bool rel = ok && local_idx(released);
      int nok;
      const int rank = block_excl_scan(rel ? 1 : 0, L.scan, &nok);
      if (rel) D.heap[L.sfree + rank] = released;
      claims_clear(L);
      __syncthreads();
      if (t == 0) {
        L.sfree += nok;
        L.nalloc += nok;
      }
      __syncthreads();
    }
  }
  TSDF_STAMP(D, 4, 2);
  if (t == 0) {
    D.ctr->free_count = L.sfree;
    if (!direct) {
      D.ctr->last_deleted = L.nalloc;
      D.ctr->total_deleted += (unsigned long long)L.nalloc;
      D.ctr->total_visible += (unsigned long long)D.ctr->n_vis;
      D.ctr->total_updated += D.ctr->last_updated;
      D.ctr->frames += 1ull;
      D.ctr->n_cand = 0;  // the next frame's lists start empty (its sweep runs before allocation)
    }
  }
  if (!direct && t < kBands) D.band[t * kBandStride] = 0;
}

// ---------------------------------------------------------------------------------------------
// Sharded frames: the carve-candidate exchange. k_cand_pack writes this shard's
// candidates (its own blocks) into its outbox slot; after the all-gather, k_cand_gather lists every
// shard's slot as the delete resolver's input -- the candidate set of one volume -- so every
// shard's index takes the same deletes (the resolver sorts by hash entry, the reference's order).
// One workgroup each (a few hundred candidates per frame).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_cand_pack(EngineDev D, ShardRec* __restrict__ out, int cap) {
  const int n = D.ctr->n_cand;
  for (int i = threadIdx.x; i < min(n, cap); i += blockDim.x) {
    const VisRec c = D.cand[i];
    ShardRec r;
    r.x = c.x;
    r.y = c.y;
    r.z = c.z;
    r.pad = 0;
    r.val = (uint32_t)c.entry;
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

__global__ __launch_bounds__(1024) void k_cand_gather(EngineDev D, const ShardRec* __restrict__ in, int cap,
                                                      int nshard) {
  __shared__ int s_base[kMaxShards + 1];
  if (threadIdx.x == 0) {
    int run = 0;
    for (int s = 0; s < nshard; ++s) {
      s_base[s] = run;
      run += min((int)in[(size_t)s * (cap + 1)].val, cap);
    }
    s_base[nshard] = run;
    D.ctr->n_cand = run;
  }
  __syncthreads();
  for (int s = 0; s < nshard; ++s) {
    const ShardRec* slot = in + (size_t)s * (cap + 1) + 1;
    const int n = s_base[s + 1] - s_base[s];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const ShardRec r = slot[i];
      VisRec c;
      c.x = r.x;
      c.y = r.y;
      c.z = r.z;
      c.pad = 0;
      c.idx = -1;
      c.entry = (int32_t)r.val;
      D.cand[s_base[s] + i] = c;
    }
  }
}

}  // namespace tsdf
