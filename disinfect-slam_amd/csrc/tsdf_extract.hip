// tsdf_extract.hip -- extraction side: raycast rendering, voxel query / download, engine
// initialisation and the hash-table / memory-pool level kernels used by the known-answer tests.
#include "tsdf_block.h"
#include "tsdf_kernels.h"

namespace tsdf {

// ---------------------------------------------------------------------------------------------
// initialisation
// ---------------------------------------------------------------------------------------------
__global__ void k_init_table(int4* table) {  // voxel_hash.cu:26-29 (+ zeroed position / offset)
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < kNumEntry) table[e] = make_int4(0, 0, -1, 0);
}
__global__ void k_init_heap(int32_t* heap, int n) {  // voxel_mem.cu:6-11
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) heap[i] = i;
}
// graph frames: the FrameArgs upload (pinned host slot -> device), one wave
__global__ void k_copy_words(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = __builtin_nontemporal_load(src + i);
}
// never-acquired blocks read like the reference's zeroed probability array: log-odds -inf (p 0)
__global__ void k_init_logodds(uint8_t* pool, int nb) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // one float4 per thread
  if (q >= (size_t)nb * (kBlockVolume / 4)) return;
  const float ninf = -__builtin_inff();
  *reinterpret_cast<float4*>(pool + (q >> 7) * kBlockBytes + kProbOffset + (q & 127) * 16) =
      make_float4(ninf, ninf, ninf, ninf);
}

// ---------------------------------------------------------------------------------------------
// query selection: occupancy bitmap -> selected bitmap + per-workgroup counts -> entry order
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int wg_prefix(const int32_t* __restrict__ wgcnt, int nwg, int* scratch,
                                         int* total) {
  int before = 0, all = 0;
  for (int j = threadIdx.x; j < nwg; j += blockDim.x) {
    const int v = wgcnt[j];
    all += v;
    if (j < (int)blockIdx.x) before += v;
  }
  before = wave_sum(before);
  all = wave_sum(all);
  if (lane_id() == 0) {
    scratch[threadIdx.x >> 6] = before;
    scratch[4 + (threadIdx.x >> 6)] = all;
  }
  __syncthreads();
  const int b = scratch[0] + scratch[1] + scratch[2] + scratch[3];
  *total = scratch[4] + scratch[5] + scratch[6] + scratch[7];
  __syncthreads();
  return b;
}

// query predicate: block fully inside the integer cube (check_bound_kernel) or any (check_valid)
__global__ __launch_bounds__(256) void k_query_count(EngineDev D, int use_bounds, short4 lo,
                                                     short4 hi) {
  __shared__ int scratch[4];
  const int w = blockIdx.x * 256 + threadIdx.x;
  unsigned long long occ = D.occ[w], sel = 0ull;
  while (occ) {
    const int b = __ffsll((long long)occ) - 1;
    occ &= occ - 1;
    if (!use_bounds) {
      sel |= 1ull << b;
      continue;
    }
    const Ent en = load_ent(D.table, (uint32_t)(w * 64 + b));
    const int vx = (int16_t)(en.x << kBlockLenBits), vy = (int16_t)(en.y << kBlockLenBits),
              vz = (int16_t)(en.z << kBlockLenBits);
    if (vx >= lo.x && vy >= lo.y && vz >= lo.z && vx + kBlockLen - 1 <= hi.x &&
        vy + kBlockLen - 1 <= hi.y && vz + kBlockLen - 1 <= hi.z)
      sel |= 1ull << b;
  }
  D.visbits[w] = sel;
  const int s = wave_sum(__popcll(sel));
  if (lane_id() == 0) scratch[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) D.wgcnt[blockIdx.x] = scratch[0] + scratch[1] + scratch[2] + scratch[3];
}

// entry-ordered snapshot of the selected entries (gather_visible_blocks_kernel)
__global__ __launch_bounds__(256) void k_vis_emit(EngineDev D, VisRec* __restrict__ out,
                                                  int32_t* __restrict__ out_count) {
  __shared__ int scratch[8];
  __shared__ int scan_scratch[4];
  int total;
  const int base = wg_prefix(D.wgcnt, (int)(kOccWords / 256), scratch, &total);
  const int w = blockIdx.x * 256 + threadIdx.x;
  unsigned long long v = D.visbits[w];
  int blk_total;
  int pos = base + block_excl_scan<4>(__popcll(v), scan_scratch, &blk_total);
  while (v) {
    const int b = __ffsll((long long)v) - 1;
    v &= v - 1;
    const uint32_t e = (uint32_t)(w * 64 + b);
    const Ent en = load_ent(D.table, e);
    VisRec r;
    r.x = en.x;
    r.y = en.y;
    r.z = en.z;
    r.pad = 0;
    r.idx = en.idx;
    r.entry = (int32_t)e;
    out[pos++] = r;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_count = total;
}

// ---------------------------------------------------------------------------------------------
// raycast (ray_cast_kernel, voxel_tsdf.cu:232-307), nearest-voxel lookups
// ---------------------------------------------------------------------------------------------
// View grid of the call (tsdf_kernels.h ViewGrid): every live block inside the cube gets its
// generation-tagged pool index, and its brick's and superbrick's flag bytes are set -- plain byte
// stores of 1 (any number of writers agree), where atomics on shared bitmap words would serialise
// across the XCDs. One thread per occupancy word. k_view_pack then packs the flags into bits.
__device__ __forceinline__ void view_grid(const EngineDev& D, const FrameParams& P, const ViewGrid& V) {
  if (V.n == 0) return;
  const int w = blockIdx.x * 256 + threadIdx.x;
  const int ox = view_origin(P.wt.x, P.voxel, V.half), oy = view_origin(P.wt.y, P.voxel, V.half),
            oz = view_origin(P.wt.z, P.voxel, V.half);
  unsigned long long occ = D.occ[w];
  while (occ) {
    const int b = __ffsll((long long)occ) - 1;
    occ &= occ - 1;
    const Ent en = load_ent(D.table, (uint32_t)(w * 64 + b));
    const int lx = en.x - ox, ly = en.y - oy, lz = en.z - oz;
    if ((unsigned)lx >= (unsigned)V.n || (unsigned)ly >= (unsigned)V.n || (unsigned)lz >= (unsigned)V.n ||
        !local_idx(en.idx))
      continue;
    const int k = ((lz >> 2) * V.nb + (ly >> 2)) * V.nb + (lx >> 2);  // brick
    V.cell[view_cell(k, lx, ly, lz)] = (V.gen << kViewIdxBits) | (uint32_t)en.idx;
    V.flags[k] = 1;
    V.flags[V.nbw * 32 + ((lz >> 4) * V.ns + (ly >> 4)) * V.ns + (lx >> 4)] = 1;
  }
}
__global__ __launch_bounds__(256) void k_view_grid(EngineDev D, FrameParams P, ViewGrid V) {
  view_grid(D, P, V);
}
__global__ __launch_bounds__(256) void k_view_grid_g(EngineDev D, const FrameArgs* __restrict__ A) {
  view_grid(D, A->R, A->V);
}
// one bitmap word per thread from its 32 flag bytes, which it zeroes for the next call
__device__ __forceinline__ void view_pack(const ViewGrid& V) {
  const int w = blockIdx.x * 256 + threadIdx.x;
  if (V.n == 0 || w >= V.nw) return;
  uint4* f = reinterpret_cast<uint4*>(V.flags + (size_t)w * 32);
  const uint4 a = f[0], b = f[1];
  const uint32_t in[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t word = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) word |= ((in[k] >> (8 * j)) & 1u) << (4 * k + j);
  V.bits[w] = word;
  if (a.x | a.y | a.z | a.w) f[0] = make_uint4(0, 0, 0, 0);
  if (b.x | b.y | b.z | b.w) f[1] = make_uint4(0, 0, 0, 0);
}
__global__ __launch_bounds__(256) void k_view_pack(ViewGrid V) { view_pack(V); }
__global__ __launch_bounds__(256) void k_view_pack_g(const FrameArgs* __restrict__ A) { view_pack(A->V); }

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
    prob = prob_of_logodds(reinterpret_cast<const float*>(blk + kProbOffset)[o]);
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
__device__ __forceinline__ void raycast(const EngineDev& D, const FrameParams& P, float step_size,
                                        const ViewGrid& V, uint32_t* sbits, uchar4* __restrict__ rgba,
                                        uchar4* __restrict__ normal) {
  // stage the bitmaps (all threads, before any ray returns)
  const int nw = V.n ? V.nw : 0;
  for (int i = threadIdx.x; i < nw; i += 256) sbits[i] = V.bits[i];
  __syncthreads();
  // XCD-aware tiles: workgroups wg and wg + 8 share an XCD (and its L2), so XCD g takes the g-th
  // contiguous run of 16x16 tiles in raster order -- neighbouring rays' blocks stay in one L2
  const int gx = gridDim.x, nwg = gx * gridDim.y, wg = blockIdx.y * gx + blockIdx.x;
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
  // the lanes' dependent loads then no longer overlap in time).
  int i = 1;
  auto in_region = [&](const f3& q) -> bool {
    return fmaxf(fmaxf(fmaf(q.x, sgn.x, ne.x), fmaf(q.y, sgn.y, ne.y)), fmaf(q.z, sgn.z, ne.z)) < 0.0f;
  };
  while (active) {
    const bool inside = in_region(pos);
#ifdef TSDF_DIAG_STAMPS
    d_it += 1;
    d_blk += !inside;
    d_ld += ridx >= 0;
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
          hit = true;
        }
      }
    }
    prev = cur;
    pos = {pos.x + sg.x, pos.y + sg.y, pos.z + sg.z};
    ++i;
    active = !hit && i < max_step;
  }
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
    const unsigned wg = blockIdx.y * gridDim.x + blockIdx.x;
    if (wg < (unsigned)kDiagMaxWg) {
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
__global__ __launch_bounds__(256) void k_raycast(EngineDev D, FrameParams P, float step_size, ViewGrid V,
                                                 uchar4* __restrict__ rgba, uchar4* __restrict__ normal) {
  extern __shared__ uint32_t sbits[];
  raycast(D, P, step_size, V, sbits, rgba, normal);
}
__global__ __launch_bounds__(256) void k_raycast_g(EngineDev D, const FrameArgs* __restrict__ A) {
  __shared__ uint32_t sbits[kViewGraphBitmapWords];
  const FrameParams R = A->R;
  const ViewGrid V = A->V;
  raycast(D, R, A->step_size, V, sbits, A->rgba, A->normal);
}

// download_tsdf_kernel (voxel_tsdf.cu:34-46): one workgroup of 512 threads per selected block
__global__ __launch_bounds__(512) void k_query_download(EngineDev D, const VisRec* __restrict__ sel,
                                                        float voxel, float4* __restrict__ out) {
  const VisRec r = sel[blockIdx.x];
  const int o = threadIdx.x;
  const int ox = o & 7, oy = (o >> 3) & 7, oz = o >> 6;
  const int16_t gx = (int16_t)((int16_t)(r.x << kBlockLenBits) + ox);
  const int16_t gy = (int16_t)((int16_t)(r.y << kBlockLenBits) + oy);
  const int16_t gz = (int16_t)((int16_t)(r.z << kBlockLenBits) + oz);
  const float ts = reinterpret_cast<const float*>(D.pool + (size_t)r.idx * kBlockBytes)[o];
  out[(size_t)blockIdx.x * kBlockVolume + o] =
      make_float4((float)gx * voxel, (float)gy * voxel, (float)gz * voxel, ts);
}

// ---------------------------------------------------------------------------------------------
// render replicas of a sharded volume: every shard selects the blocks a raycast of
// camera P can read, packs them as {key, payload} records, the records are all-gathered, and a
// scratch engine imports the union and runs the unchanged k_raycast over it. The selection is
// conservative (a superset): the block's bounding sphere, grown by the reach of one lookup (the
// nearest voxel of a ray point, its +-1 gradient neighbours), against the half-spaces of the
// pixel-centre view pyramid and a sphere of the marched ray length around the camera centre.
// Blocks outside it are never read by ray_cast_kernel (voxel_tsdf.cu:232-307), so the replica
// renders exactly what the unsharded volume renders.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool render_needs(const FrameParams& P, const RenderCull& C,
                                             const Ent& en) {
  const float h = 0.5f * (float)(kBlockLen - 1);
  const f3 w = {((float)(int16_t)(en.x << kBlockLenBits) + h) * P.voxel,
                ((float)(int16_t)(en.y << kBlockLenBits) + h) * P.voxel,
                ((float)(int16_t)(en.z << kBlockLenBits) + h) * P.voxel};
  const f3 r = qrot(P.cq, w);
  const f3 c = {r.x + P.ct.x, r.y + P.ct.y, r.z + P.ct.z};
  return c.z >= -C.reach && c.x - C.a0 * c.z >= -C.reach * C.na0 &&
         C.a1 * c.z - c.x >= -C.reach * C.na1 && c.y - C.b0 * c.z >= -C.reach * C.nb0 &&
         C.b1 * c.z - c.y >= -C.reach * C.nb1 && dot3(c, c) <= C.len * C.len;
}
// ---------------------------------------------------------------------------------------------
// Grouped selections of a shard's own blocks for the sharded extraction: one pass over
// the occupancy bitmap sets, per group g, a selection bitmap visbits + g * kOccWords and its
// per-workgroup counts wgcnt + g * (kOccWords / 256); k_vis_emit then lists each group in entry
// order. A block may belong to several groups.
//  kGroupBands: group b = image band b of the render camera -- the block can be read by a ray of
//    the band's rows (render_needs against the band's sub-pyramid: the top / bottom planes of its
//    first and last rows);
//  kGroupHalo: group d = shard d != this one owns one of the block's 26 neighbours -- d's marching
//    cubes of its own blocks read this block (cells reach one sample into every neighbour, and a
//    cell's block is decided by which neighbours exist).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_group_count(EngineDev D, FrameParams P, GroupSel S,
                                                     unsigned long long* __restrict__ visbits,
                                                     int32_t* __restrict__ wgcnt) {
  __shared__ int scratch[4][kMaxGroups];
  const int w = blockIdx.x * 256 + threadIdx.x;
  // this thread's word of every group's bitmap (thread-exclusive: plain read-modify-writes)
  for (int g = 0; g < S.ngroups; ++g) visbits[(size_t)g * kOccWords + w] = 0ull;
  unsigned long long occ = D.occ[w];
  while (occ) {
    const int b = __ffsll((long long)occ) - 1;
    occ &= occ - 1;
    const Ent en = load_ent(D.table, (uint32_t)(w * 64 + b));
    unsigned long long groups = 0ull;
    if (S.mode == kGroupBands) {
      RenderCull C = S.cull;
      for (int g = 0; g < S.ngroups; ++g) {
        C.b0 = S.b0[g];
        C.b1 = S.b1[g];
        C.nb0 = S.nb0[g];
        C.nb1 = S.nb1[g];
        if (render_needs(P, C, en)) groups |= 1ull << g;
      }
    } else {
      for (int n = 0; n < 27; ++n) {
        if (n == 13) continue;
        const int16_t nx = (int16_t)(en.x + n % 3 - 1), ny = (int16_t)(en.y + (n / 3) % 3 - 1),
                      nz = (int16_t)(en.z + n / 9 - 1);
        if (find_entry(D.table, nx, ny, nz) >= 0)
          groups |= 1ull << brick_owner(nx, ny, nz, (uint32_t)P.shard_count);
      }
      groups &= ~(1ull << P.shard_index);
    }
    while (groups) {
      const int g = __ffsll((long long)groups) - 1;
      groups &= groups - 1;
      visbits[(size_t)g * kOccWords + w] |= 1ull << b;
    }
  }
  for (int g = 0; g < S.ngroups; ++g) {
    const int c = wave_sum(__popcll(visbits[(size_t)g * kOccWords + w]));
    if (lane_id() == 0) scratch[threadIdx.x >> 6][g] = c;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < S.ngroups; g += 256)
    wgcnt[(size_t)g * (kOccWords / 256) + blockIdx.x] = scratch[0][g] + scratch[1][g] + scratch[2][g] + scratch[3][g];
}

// selection into D.visbits + per-workgroup counts; k_vis_emit then lists it in entry order
__global__ __launch_bounds__(256) void k_render_count(EngineDev D, FrameParams P, RenderCull C) {
  __shared__ int scratch[4];
  const int w = blockIdx.x * 256 + threadIdx.x;
  unsigned long long occ = D.occ[w], sel = 0ull;
  while (occ) {
    const int b = __ffsll((long long)occ) - 1;
    occ &= occ - 1;
    if (render_needs(P, C, load_ent(D.table, (uint32_t)(w * 64 + b)))) sel |= 1ull << b;
  }
  D.visbits[w] = sel;
  const int s = wave_sum(__popcll(sel));
  if (lane_id() == 0) scratch[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) D.wgcnt[blockIdx.x] = scratch[0] + scratch[1] + scratch[2] + scratch[3];
}
// one workgroup per selected block: 16-B key header + the 6 KiB block record, 16 B per lane
__global__ __launch_bounds__(256) void k_render_pack(EngineDev D, const VisRec* __restrict__ sel,
                                                     uint8_t* __restrict__ out) {
  const VisRec r = sel[blockIdx.x];
  uint8_t* dst = out + (size_t)blockIdx.x * kBlockRecBytes;
  const uint4* src = reinterpret_cast<const uint4*>(D.pool + (size_t)r.idx * kBlockBytes);
  if (threadIdx.x == 0) {
    const short4 h = make_short4(r.x, r.y, r.z, 0);
    uint4 head;
    __builtin_memcpy(&head, &h, 8);
    head.z = 0u;
    head.w = 0u;
    *reinterpret_cast<uint4*>(dst) = head;
  }
  for (int i = threadIdx.x; i < kBlockBytes / 16; i += 256)
    reinterpret_cast<uint4*>(dst + 16)[i] = src[i];
}
// import: one workgroup per record writes its payload over its block; records whose key is still
// missing after a resolver launch (bucket-lock losers, retried) are counted
__global__ __launch_bounds__(256) void k_import_payload(EngineDev D, const uint8_t* __restrict__ recs,
                                                        int32_t* missing) {
  const uint8_t* src = recs + (size_t)blockIdx.x * kBlockRecBytes;
  const short4 h = *reinterpret_cast<const short4*>(src);
  const int32_t e = find_local(D.table, h.x, h.y, h.z);
  if (e < 0) {
    if (threadIdx.x == 0) atomicAdd(missing, 1);
    return;
  }
  uint4* dst = reinterpret_cast<uint4*>(D.pool + (size_t)D.table[e].z * kBlockBytes);
  for (int i = threadIdx.x; i < kBlockBytes / 16; i += 256)
    dst[i] = reinterpret_cast<const uint4*>(src + 16)[i];
}

// ---------------------------------------------------------------------------------------------
// test-level kernels (VoxelHashTable::Retrieve / assignment, VoxelMemPool acquire / release)
// ---------------------------------------------------------------------------------------------
__global__ void k_hash_retrieve(EngineDev D, const int16_t* __restrict__ pts, int n,
                                uint32_t* rgbw, float* tsdf, float* prob, short4* bpo,
                                int32_t* bidx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int16_t x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
  const int16_t bx = (int16_t)(x >> 3), by = (int16_t)(y >> 3), bz = (int16_t)(z >> 3);
  const int32_t e = find_local(D.table, bx, by, bz);
  const int o = (x & 7) + (y & 7) * 8 + (z & 7) * 64;
  if (e < 0) {
    rgbw[i] = 0;
    tsdf[i] = 1.0f;
    prob[i] = 0.0f;
    bpo[i] = make_short4(bx, by, bz, -1);
    bidx[i] = -1;
    return;
  }
  const Ent en = load_ent(D.table, (uint32_t)e);
  const uint8_t* blk = D.pool + (size_t)en.idx * kBlockBytes;
  rgbw[i] = reinterpret_cast<const uint32_t*>(blk + kRgbwOffset)[o];
  tsdf[i] = reinterpret_cast<const float*>(blk)[o];
  prob[i] = prob_of_logodds(reinterpret_cast<const float*>(blk + kProbOffset)[o]);
  bpo[i] = make_short4(en.x, en.y, en.z, en.off);
  bidx[i] = en.idx;
}
__global__ void k_hash_assign(EngineDev D, const int16_t* __restrict__ pts, int n,
                              const uint32_t* __restrict__ rgbw, int* missing) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int16_t x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
  const int32_t e = find_local(D.table, (int16_t)(x >> 3), (int16_t)(y >> 3), (int16_t)(z >> 3));
  if (e < 0) {
    atomicAdd(missing, 1);
    return;
  }
  const int o = (x & 7) + (y & 7) * 8 + (z & 7) * 64;
  uint8_t* blk = D.pool + (size_t)D.table[e].z * kBlockBytes;
  reinterpret_cast<uint32_t*>(blk + kRgbwOffset)[o] = rgbw[i];
}
// sequential AquireBlock x n (voxel_mem.cu:37-52); -1 when the pool is empty
__global__ void k_pool_acquire(EngineDev D, int n, int32_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int k = 0; k < n; ++k) {
    const int i = D.ctr->free_count;
    if (i < 1) {
      out[k] = -1;
      continue;
    }
    D.ctr->free_count = i - 1;
    const int32_t idx = D.heap[i - 1];
    uint8_t* blk = D.pool + (size_t)idx * kBlockBytes;
    for (int v = 0; v < kBlockVolume; ++v) {
      reinterpret_cast<float*>(blk)[v] = -1.0f;
      reinterpret_cast<float*>(blk + kProbOffset)[v] = 0.0f;  // p = 0.5
      reinterpret_cast<uint32_t*>(blk + kRgbwOffset)[v] = 0u;  // weight 0 (rgb defined as 0)
    }
    out[k] = idx;
  }
}
__global__ void k_pool_release(EngineDev D, const int32_t* idx, int n) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int k = 0; k < n; ++k) {
    const int i = D.ctr->free_count;
    D.ctr->free_count = i + 1;
    D.heap[i] = idx[k];
  }
}
__global__ void k_pool_weight(EngineDev D, int32_t block, int set, uint8_t w, uint8_t* out) {
  const int v = threadIdx.x;
  uint8_t* blk = D.pool + (size_t)block * kBlockBytes + kRgbwOffset;
  if (set)
    blk[4 * v + 3] = w;
  else
    out[v] = blk[4 * v + 3];
}
// debug dump: table -> (x, y, z, off) int16 + idx int32; pool -> SoA
__global__ void k_dump_table(EngineDev D, short4* pos, int32_t* idx) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kNumEntry) return;
  const Ent en = load_ent(D.table, e);
  pos[e] = make_short4(en.x, en.y, en.z, en.off);
  idx[e] = en.idx;
}
__global__ void k_dump_pool(EngineDev D, float* tsdf, float* prob, uint32_t* rgbw) {
  const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= (size_t)D.nblocks * kBlockVolume) return;
  const size_t b = v >> kBlockVolumeBits, o = v & (kBlockVolume - 1);
  const uint8_t* blk = D.pool + b * kBlockBytes;
  tsdf[v] = reinterpret_cast<const float*>(blk)[o];
  prob[v] = prob_of_logodds(reinterpret_cast<const float*>(blk + kProbOffset)[o]);
  rgbw[v] = reinterpret_cast<const uint32_t*>(blk + kRgbwOffset)[o];
}

}  // namespace tsdf
