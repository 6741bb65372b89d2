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
  int pos = base + block_excl_scan(__popcll(v), scan_scratch, &blk_total);
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
struct VoxRef {
  const uint8_t* blk;
  int o;
};
__device__ __forceinline__ bool voxel_ref(const EngineDev& D, int16_t px, int16_t py, int16_t pz,
                                          VoxRef& ref) {
  const int16_t bx = (int16_t)(px >> kBlockLenBits), by = (int16_t)(py >> kBlockLenBits),
                bz = (int16_t)(pz >> kBlockLenBits);
  const int32_t e = find_local(D.table, bx, by, bz);
  if (e < 0) return false;
  const int32_t idx = D.table[e].z;
  ref.blk = D.pool + (size_t)idx * kBlockBytes;
  ref.o = (px & 7) + (py & 7) * kBlockLen + (pz & 7) * kBlockLen * kBlockLen;
  return true;
}
__device__ __forceinline__ float retrieve_tsdf(const EngineDev& D, int16_t x, int16_t y, int16_t z) {
  VoxRef r;
  if (!voxel_ref(D, x, y, z, r)) return 1.0f;  // VoxelTSDF() default (voxel_types.cu:9)
  return reinterpret_cast<const float*>(r.blk)[r.o];
}

__device__ __forceinline__ void raycast(EngineDev D, FrameParams P, float step_size,
                                        uchar4* __restrict__ rgba, uchar4* __restrict__ normal) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15);
  const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= P.W || y >= P.H) return;
  const int idx = y * P.W + x;
  const f3 pc = pixel_ray(P, x, y);
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
  const int max_step = f2i(ceilf(P.max_depth / step_size));
  f3 pos = {P.wt.x / P.voxel, P.wt.y / P.voxel, P.wt.z / P.voxel};
  float prev = retrieve_tsdf(D, f2s(roundf(pos.x)), f2s(roundf(pos.y)), f2s(roundf(pos.z)));
  pos.x += sg.x;
  pos.y += sg.y;
  pos.z += sg.z;
  for (int i = 1; i < max_step; ++i) {
    const float cur = retrieve_tsdf(D, f2s(roundf(pos.x)), f2s(roundf(pos.y)), f2s(roundf(pos.z)));
    if (prev > 0 && cur <= 0 && (double)(prev - cur) <= 1.5) {
      f3 p1 = {pos.x - sg.x, pos.y - sg.y, pos.z - sg.z};
      f3 p2 = pos;
      f3 mid = {(p1.x + p2.x) / 2, (p1.y + p2.y) / 2, (p1.z + p2.z) / 2};
      for (;;) {
        const f3 dd = {p1.x - p2.x, p1.y - p2.y, p1.z - p2.z};
        if (!((double)dot3(dd, dd) > .1)) break;
        if (retrieve_tsdf(D, f2s(roundf(mid.x)), f2s(roundf(mid.y)), f2s(roundf(mid.z))) < 0)
          p2 = mid;
        else
          p1 = mid;
        mid.x = (p1.x + p2.x) / 2;
        mid.y = (p1.y + p2.y) / 2;
        mid.z = (p1.z + p2.z) / 2;
      }
      const int16_t fx = f2s(roundf(mid.x)), fy = f2s(roundf(mid.y)), fz = f2s(roundf(mid.z));
      uint32_t c = 0;
      float prob = 0.0f;  // VoxelRGBW() / VoxelSEGM() defaults
      VoxRef ref;
      if (voxel_ref(D, fx, fy, fz, ref)) {
        c = reinterpret_cast<const uint32_t*>(ref.blk + kRgbwOffset)[ref.o];
        prob = prob_of_logodds(reinterpret_cast<const float*>(ref.blk + kProbOffset)[ref.o]);
      }
      const f3 nr = {retrieve_tsdf(D, (int16_t)(fx + 1), fy, fz) - retrieve_tsdf(D, (int16_t)(fx - 1), fy, fz),
                     retrieve_tsdf(D, fx, (int16_t)(fy + 1), fz) - retrieve_tsdf(D, fx, (int16_t)(fy - 1), fz),
                     retrieve_tsdf(D, fx, fy, (int16_t)(fz + 1)) - retrieve_tsdf(D, fx, fy, (int16_t)(fz - 1))};
      const f3 nd = {-dw.x, -dw.y, -dw.z};
      const float diff = fmaxf(dot3(nr, nd) / sqrtf(dot3(nr, nr)), 0.0f);
      const float alpha = (float)((double)fmaxf((float)((double)prob - 0.5), 0.0f) / .5);
      const float oma = 1 - alpha;
      if (rgba)
        rgba[idx] = make_uchar4(f2u8(alpha * 255 + oma * (float)(c & 0xFF)),
                                f2u8(oma * (float)((c >> 8) & 0xFF)),
                                f2u8(oma * (float)((c >> 16) & 0xFF)), 255);
      const float sh = oma * diff * 255;
      if (normal) normal[idx] = make_uchar4(f2u8(alpha * 255 + sh), f2u8(sh), f2u8(sh), 255);
      return;
    }
    prev = cur;
    pos.x += sg.x;
    pos.y += sg.y;
    pos.z += sg.z;
  }
  if (rgba) rgba[idx] = make_uchar4(0, 0, 0, 0);
  if (normal) normal[idx] = make_uchar4(0, 0, 0, 0);
}
__global__ __launch_bounds__(256) void k_raycast(EngineDev D, FrameParams P, float step_size,
                                                 uchar4* __restrict__ rgba,
                                                 uchar4* __restrict__ normal) {
  raycast(D, P, step_size, rgba, normal);
}
__global__ __launch_bounds__(256) void k_raycast_g(EngineDev D, const FrameArgs* __restrict__ A) {
  const FrameParams R = A->R;
  raycast(D, R, A->step_size, A->rgba, A->normal);
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
