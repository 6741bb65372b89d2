// tsdf_extract.hip -- extraction side: raycast rendering, voxel query / download, engine
// initialisation and the hash-table / memory-pool level kernels used by the known-answer tests.
#include "tsdf_block.h"
#include "tsdf_kernels.h"
#include "tsdf_raycast.h"

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
// never-acquired blocks read like the reference's zeroed probability array (p 0)
__global__ void k_init_prob(uint8_t* pool, int nb) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // one float4 per thread
  if (q >= (size_t)nb * (kBlockVolume / 4)) return;
  *reinterpret_cast<float4*>(pool + (q >> 7) * kBlockBytes + kProbOffset + (q & 127) * 16) =
      make_float4(0.f, 0.f, 0.f, 0.f);
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

__global__ __launch_bounds__(256) TSDF_RAY_PK void k_raycast(EngineDev D, FrameParams P, float step_size, ViewGrid V,
                                                 uchar4* __restrict__ rgba, uchar4* __restrict__ normal) {
  extern __shared__ uint32_t sbits[];
  raycast(D, P, step_size, V, sbits, rgba, normal, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x,
          gridDim.x * gridDim.y);
}
__global__ __launch_bounds__(256) TSDF_RAY_PK void k_raycast_g(EngineDev D, const FrameArgs* __restrict__ A) {
  __shared__ uint32_t sbits[kViewGraphBitmapWords];
  const FrameParams R = A->R;
  const ViewGrid V = A->V;
  raycast(D, R, A->step_size, V, sbits, A->rgba, A->normal, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x,
          gridDim.x * gridDim.y);
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
  prob[i] = reinterpret_cast<const float*>(blk + kProbOffset)[o];
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
      reinterpret_cast<float*>(blk + kProbOffset)[v] = 0.5f;  // p = 0.5
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
  prob[v] = reinterpret_cast<const float*>(blk + kProbOffset)[o];
  rgbw[v] = reinterpret_cast<const uint32_t*>(blk + kRgbwOffset)[o];
}

}  // namespace tsdf
