// tsdf_raycast.h -- the raycast march (ray_cast_kernel, utils/tsdf/voxel_tsdf.cu:232-307): used by
// k_raycast (tsdf_extract.hip) and by the fused render + ingest launch k_render_ingest (tsdf_alloc.hip).
#pragma once

#include "tsdf_block.h"
#include "tsdf_kernels.h"

// The library is built without packed fp32 (Makefile NOPK); the raycast kernels (k_raycast*,
// k_render_ingest*) turn it back on: their march keeps independent x / y / z work to pair, and on the
// C5 loop they measured faster with it (8.07-8.09k frames/s vs 7.85-7.89k without; k_raycast 59.3 vs
// 60.9 us; profiles/ab/r6_no_packed_fp32_ab.txt). The host pass of a kernel ignores the attribute.
#define TSDF_RAY_PK __attribute__((target("packed-fp32-ops")))
#pragma clang diagnostic ignored "-Wignored-attributes"

namespace tsdf {

// One ray's block cache (the reference's per-thread VoxelBlock cache, voxel_hash.cuh:124-161): the
// block of the last lookup and its pool index (-1: missing), and the empty region around it: 0 none,
// 1 its brick holds no block, 2 its superbrick holds none.
struct RayCache {
  int bx, by, bz;
  int32_t idx;
  int empty;
};
struct RayView {
  const uint32_t* cell;
  const uint32_t* bits;  // LDS copy of the bitmaps (bricks, then superbricks)
  int n, nb, ns, nbw, ox, oy, oz;
  uint32_t gen;
};
__device__ __forceinline__ void ray_block(const EngineDev& D, const RayView& R, RayCache& c, int bx,
                                          int by, int bz) {
  if (bx == c.bx && by == c.by && bz == c.bz) return;
  c.bx = bx;
  c.by = by;
  c.bz = bz;
  c.empty = 0;
  const int lx = bx - R.ox, ly = by - R.oy, lz = bz - R.oz;
  const int n = R.n;
  if ((unsigned)lx < (unsigned)n && (unsigned)ly < (unsigned)n && (unsigned)lz < (unsigned)n) {
    // brick and superbrick words read together (one LDS round trip, not two in sequence)
    const int k = ((lz >> 2) * R.nb + (ly >> 2)) * R.nb + (lx >> 2);
    const int q = ((lz >> 4) * R.ns + (ly >> 4)) * R.ns + (lx >> 4);
    const uint32_t wb = R.bits[k >> 5], ws = R.bits[R.nbw + (q >> 5)];
    if (!((wb >> (k & 31)) & 1u)) {
      c.idx = -1;
      c.empty = 2 - (int)((ws >> (q & 31)) & 1u);
      return;
    }
    const uint32_t v = R.cell[view_cell(k, lx, ly, lz)];
    c.idx = (v >> kViewIdxBits) == R.gen ? (int32_t)(v & ((1u << kViewIdxBits) - 1)) : -1;
    return;
  }
  const int32_t e = find_local(D.table, (int16_t)bx, (int16_t)by, (int16_t)bz);  // outside the grid / none
  c.idx = e < 0 ? -1 : D.table[e].z;
}
// The march's lookup of block (bx, by, bz) after its region was left: ray_block without the block
// cache (a step that leaves the region reads another block, except on an entry face, where the
// lookup repeats and returns the same) and with 32-bit index arithmetic (the cell offset from a
// scalar base). *empty as RayCache.empty.
__device__ __forceinline__ int32_t march_lookup(const EngineDev& D, const RayView& R, int bx, int by, int bz,
                                                int& empty) {
  empty = 0;
  const int lx = bx - R.ox, ly = by - R.oy, lz = bz - R.oz;
  const unsigned n = (unsigned)R.n;
  if ((unsigned)lx < n && (unsigned)ly < n && (unsigned)lz < n) {
    const uint32_t nb = (uint32_t)R.nb, ns = (uint32_t)R.ns;
    const uint32_t k = __umul24(__umul24((uint32_t)lz >> 2, nb) + ((uint32_t)ly >> 2), nb) + ((uint32_t)lx >> 2);
    const uint32_t q = __umul24(__umul24((uint32_t)lz >> 4, ns) + ((uint32_t)ly >> 4), ns) + ((uint32_t)lx >> 4);
    const uint32_t wb = R.bits[k >> 5], ws = R.bits[R.nbw + (q >> 5)];
    if (!((wb >> (k & 31)) & 1u)) {
      empty = 2 - (int)((ws >> (q & 31)) & 1u);
      return -1;
    }
    const uint32_t off = ((k << 6) | (((uint32_t)lz & 3) << 4) | (((uint32_t)ly & 3) << 2) | ((uint32_t)lx & 3)) * 4u;
    const uint32_t v = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(R.cell) + off);
    return (v >> kViewIdxBits) == R.gen ? (int32_t)(v & ((1u << kViewIdxBits) - 1)) : -1;
  }
  const int32_t e = find_local(D.table, (int16_t)bx, (int16_t)by, (int16_t)bz);  // outside the grid / none
  return e < 0 ? -1 : D.table[e].z;
}
__device__ __forceinline__ int voxel_off(int16_t px, int16_t py, int16_t pz) {
  return (px & 7) + (py & 7) * kBlockLen + (pz & 7) * kBlockLen * kBlockLen;
}
// Retrieve<VoxelTSDF>(point, cache).tsdf: VoxelTSDF() default +1 (voxel_types.cu:9) when missing
__device__ __forceinline__ float ray_tsdf(const EngineDev& D, const RayView& R, RayCache& c, int16_t px,
                                          int16_t py, int16_t pz) {
  ray_block(D, R, c, px >> kBlockLenBits, py >> kBlockLenBits, pz >> kBlockLenBits);
  if (c.idx < 0) return 1.0f;
  return reinterpret_cast<const float*>(D.pool + (size_t)c.idx * kBlockBytes)[voxel_off(px, py, pz)];
}

// The hit of ray_cast_kernel (voxel_tsdf.cu:259-300) at position hp: binary search between
// hp - step and hp, the voxel's colour / probability and the central-difference normal.
__device__ __forceinline__ void ray_shade(const EngineDev& D, const RayView& R, RayCache& c, f3 hp, f3 sg,
                                       f3 dw, uchar4* __restrict__ rgba, uchar4* __restrict__ normal, int idx) {
  f3 p1 = {hp.x - sg.x, hp.y - sg.y, hp.z - sg.z};
  f3 p2 = hp;
  f3 mid = {(p1.x + p2.x) / 2, (p1.y + p2.y) / 2, (p1.z + p2.z) / 2};
  for (;;) {
    const f3 dd = {p1.x - p2.x, p1.y - p2.y, p1.z - p2.z};
    if (!((double)dot3(dd, dd) > .1)) break;
    if (ray_tsdf(D, R, c, round_s16(mid.x), round_s16(mid.y), round_s16(mid.z)) < 0)
      p2 = mid;
    else
      p1 = mid;
    mid.x = (p1.x + p2.x) / 2;
    mid.y = (p1.y + p2.y) / 2;
    mid.z = (p1.z + p2.z) / 2;
  }
  const int16_t fx = round_s16(mid.x), fy = round_s16(mid.y), fz = round_s16(mid.z);
  uint32_t col = 0;
  float prob = 0.0f;  // VoxelRGBW() / VoxelSEGM() defaults
  ray_block(D, R, c, fx >> kBlockLenBits, fy >> kBlockLenBits, fz >> kBlockLenBits);
  if (c.idx >= 0) {
    const uint8_t* blk = D.pool + (size_t)c.idx * kBlockBytes;
    const int o = voxel_off(fx, fy, fz);
    col = reinterpret_cast<const uint32_t*>(blk + kRgbwOffset)[o];
    prob = reinterpret_cast<const float*>(blk + kProbOffset)[o];
  }
  const float gxp = ray_tsdf(D, R, c, (int16_t)(fx + 1), fy, fz);
  const float gxn = ray_tsdf(D, R, c, (int16_t)(fx - 1), fy, fz);
  const float gyp = ray_tsdf(D, R, c, fx, (int16_t)(fy + 1), fz);
  const float gyn = ray_tsdf(D, R, c, fx, (int16_t)(fy - 1), fz);
  const float gzp = ray_tsdf(D, R, c, fx, fy, (int16_t)(fz + 1));
  const float gzn = ray_tsdf(D, R, c, fx, fy, (int16_t)(fz - 1));
  const f3 nr = {gxp - gxn, gyp - gyn, gzp - gzn};
  const f3 nd = {-dw.x, -dw.y, -dw.z};
  const float diff = fmaxf(dot3(nr, nd) / sqrtf(dot3(nr, nr)), 0.0f);
  const float alpha = (float)((double)fmaxf((float)((double)prob - 0.5), 0.0f) / .5);
  const float oma = 1 - alpha;
  if (rgba)
    rgba[idx] = make_uchar4(f2u8(alpha * 255 + oma * (float)(col & 0xFF)), f2u8(oma * (float)((col >> 8) & 0xFF)),
                            f2u8(oma * (float)((col >> 16) & 0xFF)), 255);
  const float sh = oma * diff * 255;
  if (normal) normal[idx] = make_uchar4(f2u8(alpha * 255 + sh), f2u8(sh), f2u8(sh), 255);
}

// The march (DESIGN.md 4 "Raycast") is VALU-issue bound: ~4.7 waves per SIMD each step ~135 times,
// and a step in empty space (most of them) is only the position update and the region test. Along a
// ray each coordinate of the reference's sequential float sums pos_{i+1} = fl(pos_i + step) is
// monotone (the step's sign is fixed, rounding is monotone), so after a lookup the positions never
// cross the region's entry faces again: the test is the three exit faces, s_a * pos_a < e_a per axis
// (s = the step's sign), as one fma each (s_a * pos_a is exact, the sign of the rounded sum is the
// sign of the exact one). The step counter is wave-uniform (scalar).
// wg: this workgroup among the nwg of the raycast (16x16 tiles, gx per row); a launch of its own
// passes its block index, the fused render + ingest launch (k_render_ingest) its raycast part's
__device__ __forceinline__ void raycast(const EngineDev& D, const FrameParams& P, float step_size,
                                        const ViewGrid& V, uint32_t* sbits, uchar4* __restrict__ rgba,
                                        uchar4* __restrict__ normal, int wg, int gx, int nwg) {
  // stage the bitmaps (all threads, before any ray returns)
  const int nw = V.n ? V.nw : 0;
  for (int i = threadIdx.x; i < nw; i += 256) sbits[i] = V.bits[i];
  __syncthreads();
  // XCD-aware tiles: workgroups wg and wg + 8 share an XCD (and its L2), so XCD g takes the g-th
  // contiguous run of 16x16 tiles in raster order -- neighbouring rays' blocks stay in one L2
  const int g = wg & 7, tile = g * (nwg >> 3) + min(g, nwg & 7) + (wg >> 3);
  // each wave an 8x8 quadrant of the tile (a tighter ray bundle than 16x4 rows, whose lanes leave
  // their regions at closer steps, 101.3 vs 103.8 us at C5)
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  // rows [P.row0, P.row0 + P.nrows) of the W x H camera (a band of a sharded render, else all);
  // the outputs hold the band's rows only
  const int x = (tile % gx) * 16 + (wv & 1) * 8 + (ln & 7);
  const int yb = (tile / gx) * 16 + (wv >> 1) * 8 + (ln >> 3);
  const int y = P.row0 + yb;
  const bool valid = x < P.W && yb < P.nrows && y < P.H;
  const int idx = valid ? yb * P.W + x : 0;
  RayView R;
  R.cell = V.cell;
  R.bits = sbits;
  R.n = V.n;
  R.nb = V.nb;
  R.ns = V.ns;
  R.nbw = V.nbw;
  R.gen = V.gen;
  R.ox = view_origin(P.wt.x, P.voxel, V.half);
  R.oy = view_origin(P.wt.y, P.voxel, V.half);
  R.oz = view_origin(P.wt.z, P.voxel, V.half);
  RayCache c;
  c.bx = c.by = c.bz = 0x7FFFFFFF;  // no block (block coordinates are int16)
  c.idx = -1;
  c.empty = 0;
  const f3 pc = pixel_ray(P, valid ? x : 0, valid ? y : 0);
  const float nn = dot3(pc, pc);
  f3 dc = pc;
  if (nn > 0) {
    const float s = sqrtf(nn);
    dc.x = pc.x / s;
    dc.y = pc.y / s;
    dc.z = pc.z / s;
  }
  const f3 dw = qrot(P.wq, dc);
  const f3 sg = {dw.x * step_size / P.voxel, dw.y * step_size / P.voxel, dw.z * step_size / P.voxel};
  const int max_step = __builtin_amdgcn_readfirstlane(f2i(ceilf(P.max_depth / step_size)));  // (uniform)
  // steps i = 1 .. max_step - 1; the comparison of step 1 needs the value at the origin
  f3 pos = {P.wt.x / P.voxel, P.wt.y / P.voxel, P.wt.z / P.voxel};
  bool active = valid && 1 < max_step;
  bool hit = false;
  f3 hit_pos = pos;
  float prev = 1.0f;
  if (active) prev = ray_tsdf(D, R, c, round_s16(pos.x), round_s16(pos.y), round_s16(pos.z));
  pos = {pos.x + sg.x, pos.y + sg.y, pos.z + sg.z};
  // Region of the last lookup: the missing block or the empty brick / superbrick around it (reads +1:
  // no lookup, no hit), or the present block (only the voxel offset and its load), held as its exit
  // faces: inside while fma(pos_a, s_a, ne_a) < 0 on every axis (ne = -e; +inf before the first lookup).
  const f3 sgn = {sg.x >= 0.0f ? 1.0f : -1.0f, sg.y >= 0.0f ? 1.0f : -1.0f, sg.z >= 0.0f ? 1.0f : -1.0f};
  f3 ne = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  int32_t ridx = -1;  // pool index of the present block of the region, -1 missing
#ifdef TSDF_DIAG_STAMPS
  // diagnostic step statistics (per lane), summed per workgroup into D.dbg kernel 5; the wave's
  // start / end clock into kernel 6 (wave w of the workgroup at 2 w / 2 w + 1)
  int d_it = 0, d_blk = 0, d_ld = 0;
  const unsigned long long d_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  // The lanes of a wave step together (a tight per-lane loop through empty regions measured slower:
  // the lanes' dependent loads then no longer overlap in time), over a scalar step counter: a lane
  // that has hit (or never marches) is frozen in an endless empty region -- no lookups, no reads, no
  // state that matters -- so the loop needs no per-lane exit masks (their exec bookkeeping was ~2/3
  // of the march's scalar instructions) and ends when no lane of the wave is live.
  auto in_region = [&](const f3& q) -> bool {
    return fmaxf(fmaxf(fmaf(q.x, sgn.x, ne.x), fmaf(q.y, sgn.y, ne.y)), fmaf(q.z, sgn.z, ne.z)) < 0.0f;
  };
  // (the lane's state as an integer in a VGPR: a bool would live as an exec-style mask whose merges
  // after every branch cost scalar instructions)
  int live = active ? 1 : 0;
  if (!active) ne = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int i = 1; i < max_step; ++i) {
    if (__builtin_amdgcn_ballot_w64(live != 0) == 0ull) break;
    const bool inside = in_region(pos);
#ifdef TSDF_DIAG_STAMPS
    d_it += live != 0;
    d_blk += live != 0 && !inside;
    d_ld += live != 0 && ridx >= 0;
#endif
    // a lane inside an empty region reads +1 and needs nothing else this step (no rounding either:
    // when every lane of the wave is there, the wave skips the block below)
    float cur = 1.0f;
    if (!inside || ridx >= 0) {
      const int16_t px = round_s16(pos.x), py = round_s16(pos.y), pz = round_s16(pos.z);
      if (!inside) {
        const int bx = px >> kBlockLenBits, by = py >> kBlockLenBits, bz = pz >> kBlockLenBits;
        int empty;
        ridx = march_lookup(D, R, bx, by, bz, empty);
        // 2^sh blocks per axis: 0 for a block (present, or missing in an occupied brick), 2 for an
        // empty brick, 4 for an empty superbrick (empty 0 / 1 / 2); selects, not branches
        const int sh = 2 * empty;
        const int rx = (R.ox + (((bx - R.ox) >> sh) << sh)) * kBlockLen;
        const int ry = (R.oy + (((by - R.oy) >> sh) << sh)) * kBlockLen;
        const int rz = (R.oz + (((bz - R.oz) >> sh) << sh)) * kBlockLen;
        const float len = (float)(kBlockLen << sh);
        // faces at r - 0.5 and r + len - 0.5: the exit face of the step's direction, negated
        // (s = +1: pos < hi; s = -1: -pos < -lo)
        const float lx = (float)rx - 0.5f, ly = (float)ry - 0.5f, lz = (float)rz - 0.5f;
        ne = {sgn.x > 0.0f ? -(lx + len) : lx, sgn.y > 0.0f ? -(ly + len) : ly, sgn.z > 0.0f ? -(lz + len) : lz};
      }
      if (ridx >= 0) {
        cur = reinterpret_cast<const float*>(D.pool + (size_t)ridx * kBlockBytes)[voxel_off(px, py, pz)];
        if (prev > 0 && cur <= 0 && (double)(prev - cur) <= 1.5) {
          hit_pos = pos;  // shaded after the march (below)
          live = 0;  // frozen: an endless empty region from here on
          ne = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
          ridx = -1;
        }
      }
    }
    prev = cur;
    pos = {pos.x + sg.x, pos.y + sg.y, pos.z + sg.z};
  }
  hit = active && live == 0;
  // The hits are shaded together after the march: inside it, the lanes of a wave hit at different
  // steps, and each step with a hit ran the whole shading (binary search + 7 lookups) for a few lanes.
  // The shading reads only the static volume (the block cache is a memo), so where it runs changes
  // nothing.
  if (hit) {
#if defined(TSDF_EXP) && (TSDF_EXP & 8)  // experiment build: no shading (timing of the march alone)
    if (rgba) rgba[idx] = make_uchar4(255, 255, 255, 255);
#else
    ray_shade(D, R, c, hit_pos, sg, dw, rgba, normal, idx);
#endif
  } else if (valid) {
    if (rgba) rgba[idx] = make_uchar4(0, 0, 0, 0);
    if (normal) normal[idx] = make_uchar4(0, 0, 0, 0);
  }
#ifdef TSDF_DIAG_STAMPS
  if (D.dbg) {
    int mx_it = d_it;
    for (int o = 32; o > 0; o >>= 1) mx_it = max(mx_it, __shfl_xor(mx_it, o, 64));
    if ((unsigned)wg < (unsigned)kDiagMaxWg) {
      unsigned long long* q = D.dbg + ((size_t)5 * kDiagMaxWg + wg) * kDiagStamps;
      atomicAdd(&q[0], (unsigned long long)d_it);
      atomicAdd(&q[1], (unsigned long long)d_blk);
      atomicAdd(&q[2], (unsigned long long)d_ld);
      atomicAdd(&q[6], (unsigned long long)hit);
      if (lane_id() == 0) {
        atomicAdd(&q[3], (unsigned long long)mx_it);
        atomicAdd(&q[7], 1ull);
        unsigned long long* q6 = D.dbg + ((size_t)6 * kDiagMaxWg + wg) * kDiagStamps;
        q6[2 * (threadIdx.x >> 6)] = d_t0;
        q6[2 * (threadIdx.x >> 6) + 1] = __builtin_amdgcn_s_memrealtime();
      }
    }
  }
#endif
}
}  // namespace tsdf
