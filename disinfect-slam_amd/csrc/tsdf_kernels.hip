// tsdf_kernels.hip -- gfx950 kernels of the TSDF semantic-fusion engine.
//
// Per frame (TSDFGrid::Integrate, reference voxel_tsdf.cu:347-375), all on one stream, no host
// round trip (the reference syncs 3+ times per frame, voxel_tsdf.cu:367,374,467-469):
//   k_ingest_dda      pixel tiles: pack the frame, DDA the truncation band, probe the table,
//                     insert missing visible block keys into the per-frame new-key set
//                     (block_allocate_kernel :104-147, VoxelHashTable::Allocate existence check)
//   k_order_mark      new key -> bit at its first candidate index (pixel raster order, DDA step)
//   k_compact_*       ordered bitmap compaction (wave ballot/popcount + block scan)
//   k_resolve_alloc   one workgroup: bucket-lock semantics of VoxelHashTable::Allocate
//                     (voxel_hash.cu:58-120) replayed exactly in candidate order, speculatively
//                     1024 keys at a time; pool acquisition by prefix sum (voxel_mem.cu:37-52)
//   k_fresh_init      AquireBlock's voxel initialisation for this frame's new blocks
//   k_vis_count/emit  visibility over the occupancy bitmap (check_visibility_kernel :82-93,
//                     prefix_sum + gather_visible_blocks_kernel :95-102 in entry order)
//   k_integrate       one wave per visible 8^3 block: fused TSDF + RGB + weight + semantic
//                     log-odds update (tsdf_integrate_kernel :149-205) and the space-carving
//                     minimum (space_carving_kernel :207-230) in registers
//   k_resolve_delete  one workgroup: VoxelHashTable::Delete (voxel_hash.cu:122-171) in entry
//                     order with bucket-lock semantics; ReleaseBlock order by prefix sum
// Extraction: k_raycast (ray_cast_kernel :232-307), k_query_* (check_bound/check_valid/
// download_tsdf kernels :14-46).
#include "tsdf_kernels.h"

namespace tsdf {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int n = __shfl_up(v, o, 64);
    if (l >= o) v += n;
  }
  return v;
}
// exclusive block scan of an int; returns exclusive prefix, *total = block sum.
// scratch: >= blockDim/64 ints of LDS. Must be reached by every thread of the block.
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int* total) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int incl = wave_incl_scan(v);
  if (lane_id() == 63) scratch[w] = incl;
  __syncthreads();
  int before = 0, tot = 0;
  for (int i = 0; i < nw; ++i) {
    const int s = scratch[i];
    if (i < w) before += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return before + incl - v;
}
__device__ __forceinline__ unsigned long long atomic_load_u64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

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

// ---------------------------------------------------------------------------------------------
// new-key set (per frame): open addressing on 64-bit packed keys, min candidate order per key
// ---------------------------------------------------------------------------------------------
__device__ void nk_insert(const EngineDev& D, uint64_t key, uint32_t order) {
  uint32_t h = (uint32_t)mix64(key) & (kNewKeyCap - 1);
  for (int p = 0; p < 256; ++p) {
    unsigned long long cur = D.nk_key[h];
    if (cur == 0ull) cur = atomicCAS(&D.nk_key[h], 0ull, (unsigned long long)key);
    if (cur == 0ull) {
      const int s = atomicAdd(&D.ctr->nk_count, 1);
      D.nk_list[s] = (int32_t)h;
      atomicMin(&D.nk_order[h], order);
      return;
    }
    if (cur == key) {
      atomicMin(&D.nk_order[h], order);
      return;
    }
    h = (h + 1) & (kNewKeyCap - 1);
  }
  atomicOr(&D.ctr->status, 2u);  // TSDF_STATUS_NEWKEY_OVERFLOW
}

// block_allocate_kernel (voxel_tsdf.cu:104-147) up to the Allocate call: per pixel DDA over
// [p - trunc dir, p + trunc dir]; keys whose 8 corners are all in view and that are not in the
// table go to the new-key set with candidate order (y*W + x)*maxs + i. Also packs the frame into
// one 16-B record per pixel {depth, ht, lt, rgb} for the integrate gathers.
__global__ __launch_bounds__(256) void k_ingest_dda(EngineDev D, FrameParams P,
                                                    const float* __restrict__ depth,
                                                    const uint8_t* __restrict__ rgb,
                                                    const float* __restrict__ ht,
                                                    const float* __restrict__ lt) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15);
  const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= P.W || y >= P.H) return;
  const int i = y * P.W + x;
  const float d = depth[i];
  const uint32_t c = (uint32_t)rgb[3 * i] | ((uint32_t)rgb[3 * i + 1] << 8) |
                     ((uint32_t)rgb[3 * i + 2] << 16);
  const float h = ht ? ht[i] : 1.0f;
  const float l = lt ? lt[i] : 1.0f;
  D.pix[i] = make_float4(d, h, l, __uint_as_float(c));
  if (d == 0 || d > P.max_depth) return;
  const f3 pc = pixel_ray(P, x, y);
  const float range = sqrtf(dot3(pc, pc));
  const f3 pcd = {pc.x * d, pc.y * d, pc.z * d};
  const f3 pw = se3_apply(P.wq, P.wt, pcd);
  const f3 dc = {pc.x / range, pc.y / range, pc.z / range};
  const f3 dw = qrot(P.wq, dc);
  const f3 sw = {pw.x - dw.x * P.trunc, pw.y - dw.y * P.trunc, pw.z - dw.z * P.trunc};
  const f3 dg = {dw.x / P.voxel, dw.y / P.voxel, dw.z / P.voxel};
  const f3 sg = {sw.x / P.voxel, sw.y / P.voxel, sw.z / P.voxel};
  const float two_trunc = 2 * P.trunc;
  const f3 rg = {two_trunc * dg.x, two_trunc * dg.y, two_trunc * dg.z};
  const int step_grid = f2i(ceilf(fmaxf(fmaxf(fabsf(rg.x), fabsf(rg.y)), fabsf(rg.z)) / kBlockLen));
  const float div = fmaxf((float)step_grid, 1.0f);
  const f3 st = {rg.x / div, rg.y / div, rg.z / div};
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
    if (P.shard_count > 1 && brick_owner(kx, ky, kz, (uint32_t)P.shard_count) != (uint32_t)P.shard_index)
      continue;
    if (!block_visible<true>(P, kx, ky, kz)) continue;
    if (find_entry(D.table, kx, ky, kz) >= 0) continue;
    nk_insert(D, pack_key(kx, ky, kz), (uint32_t)i * (uint32_t)P.maxs + (uint32_t)s);
  }
}

// test path: keys[n] in list order (VoxelHashTable::Allocate launch of voxel_hash_test.cu)
__global__ void k_keys_to_newset(EngineDev D, const int16_t* __restrict__ keys, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int16_t x = keys[3 * i], y = keys[3 * i + 1], z = keys[3 * i + 2];
    if (find_entry(D.table, x, y, z) >= 0) continue;
    nk_insert(D, pack_key(x, y, z), (uint32_t)i);
  }
}

__global__ void k_order_mark(EngineDev D) {
  const int n = D.ctr->nk_count;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int h = D.nk_list[i];
    const uint32_t o = D.nk_order[h];
    atomicOr(&D.obits[o >> 6], 1ull << (o & 63));
    D.order_slot[o] = h;
  }
}

// ---------------------------------------------------------------------------------------------
// ordered bitmap compaction: 256 threads x 1 word (64 bits) per workgroup
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_compact_count(const unsigned long long* __restrict__ bits,
                                                       int nwords, int32_t* __restrict__ wgcnt) {
  __shared__ int scratch[4];
  const int w = blockIdx.x * 256 + threadIdx.x;
  const int c = w < nwords ? __popcll(bits[w]) : 0;
  const int s = wave_sum(c);
  if (lane_id() == 0) scratch[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) wgcnt[blockIdx.x] = scratch[0] + scratch[1] + scratch[2] + scratch[3];
}

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

// emits the set-bit indices in increasing order into out[], clears the words, writes the total
__global__ __launch_bounds__(256) void k_compact_emit(unsigned long long* __restrict__ bits,
                                                      int nwords,
                                                      const int32_t* __restrict__ wgcnt, int nwg,
                                                      int32_t* __restrict__ out,
                                                      int32_t* __restrict__ out_count) {
  __shared__ int scratch[8];
  __shared__ int scan_scratch[4];
  int total;
  const int base = wg_prefix(wgcnt, nwg, scratch, &total);
  const int w = blockIdx.x * 256 + threadIdx.x;
  unsigned long long v = w < nwords ? bits[w] : 0ull;
  int blk_total;
  int pos = base + block_excl_scan(__popcll(v), scan_scratch, &blk_total);
  if (v) bits[w] = 0ull;
  while (v) {
    const int b = __ffsll((long long)v) - 1;
    v &= v - 1;
    out[pos++] = w * 64 + b;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_count = total;
}

// ---------------------------------------------------------------------------------------------
// allocation resolve: exact replay of VoxelHashTable::Allocate in candidate order
// ---------------------------------------------------------------------------------------------
// Every unique missing key K (in first-candidate order) is evaluated against the current table:
//   SLOT(B, s)   : an empty slot s of its bucket B        -> needs lock B
//   APPEND(L, C) : bucket full -> tail T of B's list (bucket L = T/2), first empty slot-0 entry E
//                  after T (bucket C = E/2)               -> needs lock L, then lock C
// A key's outcome depends on earlier keys only through the buckets it locks (every table write
// happens under those locks), so a chunk of 1024 keys is evaluated speculatively, each key
// claims its buckets (64-bit max of {generation, ~rank}), and the longest prefix of keys that won
// all their claims commits in parallel. The first key of a chunk always wins, so the loop ends.
__global__ __launch_bounds__(kResolveThreads) void k_resolve_alloc(EngineDev D, int count_stats) {
  __shared__ int s_free, s_nfresh, s_first_dirty, s_base, s_nalloc;
  __shared__ uint32_t s_epoch, s_gen;
  __shared__ int s_scan[kResolveThreads / 64];
  const int t = threadIdx.x;
  if (t == 0) {
    s_epoch = D.ctr->lock_epoch + 1;
    D.ctr->lock_epoch = s_epoch;
    s_gen = D.ctr->claim_gen;
    s_free = D.ctr->free_count;
    s_nfresh = 0;
    s_base = 0;
    s_nalloc = 0;
  }
  __syncthreads();
  const int n = D.ctr->n_sorted;
  for (int iter = 0;; ++iter) {
    const int base = s_base;
    if (base >= n) break;
    if (iter > n + 8) {  // unreachable (the first key of a chunk always commits): hang insurance
      if (t == 0) atomicOr(&D.ctr->status, 8u);
      break;
    }
    const uint32_t gen = s_gen + 1;
    const bool have = base + t < n;
    int kind = 0, slot = 0, h = -1;
    uint32_t B = 0, L = 0, C = 0, T = 0, E = 0;
    int16_t kx = 0, ky = 0, kz = 0;
    const unsigned long long tag = ((unsigned long long)gen << 32) | (0xFFFFFFFFull - (uint32_t)t);
    if (have) {
      const int o = D.sorted[base + t];
      h = D.order_slot[o];
      unpack_key(D.nk_key[h], kx, ky, kz);
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
        L = T >> 1;
        uint32_t nx = T;
        for (uint32_t p = 0; p < kNumEntry; ++p) {
          nx = (nx + 1) & kEntryMask;
          if ((nx & 1u) == 0u && load_ent(D.table, nx).idx < 0) break;
        }
        E = nx;
        C = E >> 1;
      }
      if (kind == 1) {
        atomicMax(&D.claim[B], tag);
      } else {
        atomicMax(&D.claim[L], tag);
        atomicMax(&D.claim[C], tag);
      }
    }
    if (t == 0) s_first_dirty = kResolveThreads;
    __syncthreads();
    if (have) {
      bool clean;
      if (kind == 1)
        clean = atomic_load_u64(&D.claim[B]) == tag;
      else
        clean = atomic_load_u64(&D.claim[L]) == tag && atomic_load_u64(&D.claim[C]) == tag;
      if (!clean) atomicMin(&s_first_dirty, t);
    }
    __syncthreads();
    const int first_dirty = s_first_dirty;
    const bool commit = have && t < first_dirty;
    bool ok = false;
    if (commit) {
      const uint32_t ep = s_epoch;
      if (kind == 1) {
        if (D.lock_tag[B] != ep) {
          D.lock_tag[B] = ep;
          ok = true;
        }
      } else if (D.lock_tag[L] != ep) {
        D.lock_tag[L] = ep;
        if (D.lock_tag[C] != ep) {
          D.lock_tag[C] = ep;
          ok = true;
        }
      }
    }
    int nok;
    const int rank = block_excl_scan(ok ? 1 : 0, s_scan, &nok);
    const int free_now = s_free;
    if (ok) {
      const int hi = free_now - 1 - rank;
      if (hi < 0) {
        atomicOr(&D.ctr->status, 1u);  // TSDF_STATUS_POOL_EXHAUSTED (insert dropped)
      } else {
        const int32_t idx = D.heap[hi];
        uint32_t e;
        if (kind == 1) {
          e = 2 * B + (uint32_t)slot;
        } else {
          const uint32_t wrap = E > T ? 0u : kNumEntry;
          store_off(D.table, T, (int16_t)(E + wrap - T));
          e = E;
        }
        store_ent(D.table, e, kx, ky, kz, 0, idx);
        atomicOr(&D.occ[e >> 6], 1ull << (e & 63));
        D.fresh[s_nfresh + rank] = idx;
      }
    }
    if (commit) {
      D.nk_key[h] = 0ull;
      D.nk_order[h] = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (t == 0) {
      const int used = nok < free_now ? nok : (free_now > 0 ? free_now : 0);
      s_free = free_now - used;
      s_nfresh += used;
      s_nalloc += used;
      const int span = n - base < kResolveThreads ? n - base : kResolveThreads;
      s_base = base + (first_dirty < span ? first_dirty : span);
      s_gen = gen;
    }
    __syncthreads();
  }
  if (t == 0) {
    D.ctr->free_count = s_free;
    D.ctr->claim_gen = s_gen;
    D.ctr->n_fresh = s_nfresh;
    D.ctr->nk_count = 0;
    if (count_stats) {
      D.ctr->last_alloc = s_nalloc;
      D.ctr->last_new_keys = n;
      D.ctr->total_alloc += (unsigned long long)s_nalloc;
      D.ctr->last_updated = 0ull;
    }
  }
}

// AquireBlock's initialisation (voxel_mem.cu:43-51): weight 0, tsdf -1, prob 0.5, rgb untouched
__global__ __launch_bounds__(256) void k_fresh_init(EngineDev D) {
  const int n = D.ctr->n_fresh;
  const int quads = n * (kBlockVolume / 4);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += gridDim.x * blockDim.x) {
    const int b = q >> 7, v = (q & 127) * 4;
    uint8_t* blk = D.pool + (size_t)D.fresh[b] * kBlockBytes;
    *reinterpret_cast<float4*>(blk + v * 4) = make_float4(-1.f, -1.f, -1.f, -1.f);
    *reinterpret_cast<float4*>(blk + kProbOffset + v * 4) = make_float4(.5f, .5f, .5f, .5f);
    uint4* cw = reinterpret_cast<uint4*>(blk + kRgbwOffset + v * 4);
    uint4 c = *cw;
    c.x &= 0x00FFFFFFu;
    c.y &= 0x00FFFFFFu;
    c.z &= 0x00FFFFFFu;
    c.w &= 0x00FFFFFFu;
    *cw = c;
  }
}

// ---------------------------------------------------------------------------------------------
// visibility: occupancy bitmap -> visible bitmap (+ per-workgroup counts) -> entry-ordered list
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_vis_count(EngineDev D, FrameParams P) {
  __shared__ int scratch[4];
  const int w = blockIdx.x * 256 + threadIdx.x;  // kOccWords == 256 * 256
  unsigned long long occ = D.occ[w], vis = 0ull;
  while (occ) {
    const int b = __ffsll((long long)occ) - 1;
    occ &= occ - 1;
    const Ent en = load_ent(D.table, (uint32_t)(w * 64 + b));
    if (block_visible<false>(P, en.x, en.y, en.z)) vis |= 1ull << b;
  }
  D.visbits[w] = vis;
  const int s = wave_sum(__popcll(vis));
  if (lane_id() == 0) scratch[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) D.wgcnt[blockIdx.x] = scratch[0] + scratch[1] + scratch[2] + scratch[3];
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
// fused integrate + carve minimum: one wave per visible block, 8 voxels per lane
// ---------------------------------------------------------------------------------------------
// Lane l owns voxels 4l..4l+3 (z = 0..3) and 256+4l..256+4l+3 (z = 4..7), i.e. x = 4(l&1)+j,
// y = (l>>1)&7: every voxel-state access is a 16-B-per-lane, 1-KiB-per-wave coalesced transfer
// inside the block's contiguous 6-KiB record. Pixel data is one 16-B gather per voxel.
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

__global__ __launch_bounds__(256) void k_integrate(EngineDev D, FrameParams P) {
  const int lane = lane_id();
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
  const int nvis = D.ctr->n_vis;
  const int rx0 = (lane & 1) * 4, ry = (lane >> 1) & 7, rz0 = lane >> 4;
  const float neg_trunc = -P.trunc;
  int my_upd = 0;
  for (int b = wave; b < nvis; b += nwaves) {
    const VisRec r = D.vis[b];
    uint8_t* blk = D.pool + (size_t)r.idx * kBlockBytes;
    float4 ts[2], pr[2];
    uint4 cw[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int off = (hf * 256 + lane * 4) * 4;
      ts[hf] = *reinterpret_cast<const float4*>(blk + off);
      pr[hf] = *reinterpret_cast<const float4*>(blk + kProbOffset + off);
      cw[hf] = *reinterpret_cast<const uint4*>(blk + kRgbwOffset + off);
    }
    const int16_t bx = (int16_t)(r.x << kBlockLenBits), by = (int16_t)(r.y << kBlockLenBits),
                  bz = (int16_t)(r.z << kBlockLenBits);
    float mn = __builtin_inff();
    int upd_mask = 0;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int16_t ax = (int16_t)(bx + rx0 + j), ay = (int16_t)(by + ry),
                      az = (int16_t)(bz + rz0 + 4 * hf);
        const f3 pw = {(float)ax * P.voxel, (float)ay * P.voxel, (float)az * P.voxel};
        const f3 pc = se3_apply(P.cq, P.ct, pw);
        const float hx = P.fx * pc.x + P.cx * pc.z;
        const float hy = P.fy * pc.y + P.cy * pc.z;
        const float hz = pc.z;
        const int u = f2i(roundf(hx / hz));
        const int v = f2i(roundf(hy / hz));
        float tsdf = comp(ts[hf], j);
        if (u >= 0 && u < P.W && v >= 0 && v < P.H) {
          const float4 px = D.pix[v * P.W + u];
          const float d = px.x;
          if (!(d == 0 || d > P.max_depth)) {
            const f3 ray = pixel_ray(P, u, v);
            const float range = sqrtf(dot3(ray, ray));
            const float sdf = range * (d - hz);
            if (sdf > neg_trunc) {
              const float tsdf_new = fminf(1.0f, sdf / P.trunc);
              const uint32_t c_old = compu(cw[hf], j);
              const uint32_t c_new = __float_as_uint(px.w);
              const float w_new = (1.0f - d / P.max_depth) * 4.0f;
              const float w_old = (float)(c_old >> 24);
              const float wc = w_old + w_new;
              const float r0 = ((float)(c_old & 0xFF) * w_old + (float)(c_new & 0xFF) * w_new) / wc;
              const float r1 = ((float)((c_old >> 8) & 0xFF) * w_old +
                                (float)((c_new >> 8) & 0xFF) * w_new) / wc;
              const float r2 = ((float)((c_old >> 16) & 0xFF) * w_old +
                                (float)((c_new >> 16) & 0xFF) * w_new) / wc;
              tsdf = (tsdf * w_old + tsdf_new * w_new) / wc;
              const uint32_t wt = f2u8(fminf(roundf(wc), 40.0f));
              const uint32_t c = (uint32_t)f2u8(roundf(r0)) | ((uint32_t)f2u8(roundf(r1)) << 8) |
                                 ((uint32_t)f2u8(roundf(r2)) << 16) | (wt << 24);
              const float p = comp(pr[hf], j);
              const float pos = expf((w_old * logf(p) + w_new * logf(px.y)) / wc);
              const float neg = expf((w_old * logf(1.0f - p) + w_new * logf(px.z)) / wc);
              setc(ts[hf], j, tsdf);
              setc(pr[hf], j, pos / (pos + neg));
              setu(cw[hf], j, c);
              upd_mask |= 1 << (hf * 4 + j);
            }
          }
        }
        mn = fminf(mn, fabsf(tsdf));
      }
    }
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      if (upd_mask & (0xF << (hf * 4))) {
        const int off = (hf * 256 + lane * 4) * 4;
        *reinterpret_cast<float4*>(blk + off) = ts[hf];
        *reinterpret_cast<float4*>(blk + kProbOffset + off) = pr[hf];
        *reinterpret_cast<uint4*>(blk + kRgbwOffset + off) = cw[hf];
      }
    }
    my_upd += __popc(upd_mask);
    mn = wave_min(mn);
    if (lane == 0 && mn >= 0.9f) atomicOr(&D.candbits[b >> 6], 1ull << (b & 63));
  }
  const int tot = wave_sum(my_upd);
  if (lane == 0 && tot) atomicAdd(&D.ctr->last_updated, (unsigned long long)tot);
}

// ---------------------------------------------------------------------------------------------
// delete resolve: VoxelHashTable::Delete in list (entry) order with bucket-lock semantics
// ---------------------------------------------------------------------------------------------
// Slot-0 deletes are lock free and touch only their own entry; list-head / list-element deletes
// lock the key's bucket, and only the first of them per bucket (in order) proceeds. Both kinds
// modify disjoint entries, so a whole chunk commits at once; only the release order onto the
// free-block stack needs a prefix sum. direct != 0: `list` is null and recs[] holds the keys in
// order (test path, one key per step so repeated keys see each other's effect).
__global__ __launch_bounds__(kResolveThreads) void k_resolve_delete(EngineDev D,
                                                                    const int32_t* __restrict__ list,
                                                                    const int32_t* __restrict__ count,
                                                                    const VisRec* __restrict__ recs,
                                                                    int chunk, int carve) {
  __shared__ int s_free, s_ndel;
  __shared__ uint32_t s_epoch, s_gen;
  __shared__ int s_scan[kResolveThreads / 64];
  const int t = threadIdx.x;
  if (t == 0) {
    s_epoch = D.ctr->lock_epoch + 1;
    D.ctr->lock_epoch = s_epoch;
    s_gen = D.ctr->claim_gen;
    s_free = D.ctr->free_count;
    s_ndel = 0;
  }
  __syncthreads();
  const int n = *count;
  for (int base = 0; base < n; base += chunk) {
    const uint32_t gen = s_gen + 1;
    const bool have = t < chunk && base + t < n;
    const unsigned long long tag = ((unsigned long long)gen << 32) | (0xFFFFFFFFull - (uint32_t)t);
    int kind = 0;  // 1 slot0, 2 head, 3 list element
    uint32_t A = 0, prev = 0, cur = 0;
    Ent ecur = {}, eprev = {};
    if (have) {
      const VisRec r = list ? recs[list[base + t]] : recs[base + t];
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
          cur = (uint32_t)(prev + (int32_t)hd.off) & kEntryMask;  // the element moved into head
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
      if (kind >= 2) atomicMax(&D.claim[A], tag);
    }
    __syncthreads();
    bool ok = false;
    int32_t released = -1;
    if (kind == 1) {
      ok = true;
    } else if (kind >= 2 && atomic_load_u64(&D.claim[A]) == tag) {
      ok = D.lock_tag[A] != s_epoch;
      D.lock_tag[A] = s_epoch;
    }
    if (ok) {
      if (kind == 1) {  // voxel_hash.cu:126-135
        released = ecur.idx;
        store_off_idx(D.table, cur, 0, -1);
        atomicAnd(&D.occ[cur >> 6], ~(1ull << (cur & 63)));
      } else if (kind == 2) {  // :137-152 (cur may alias the head when the list is empty)
        released = eprev.idx;
        const int16_t noff = ecur.off ? (int16_t)(eprev.off + ecur.off) : (int16_t)0;
        store_ent(D.table, prev, ecur.x, ecur.y, ecur.z, noff, ecur.idx);
        store_off_idx(D.table, cur, 0, -1);
        atomicAnd(&D.occ[cur >> 6], ~(1ull << (cur & 63)));
      } else {  // :154-170
        released = ecur.idx;
        const int16_t noff = ecur.off ? (int16_t)(eprev.off + ecur.off) : (int16_t)0;
        store_off(D.table, prev, noff);
        store_off_idx(D.table, cur, 0, -1);
        atomicAnd(&D.occ[cur >> 6], ~(1ull << (cur & 63)));
      }
    }
    int nok;
    const int rank = block_excl_scan(ok ? 1 : 0, s_scan, &nok);
    if (ok) D.heap[s_free + rank] = released;  // ReleaseBlock (voxel_mem.cu:54-59)
    __syncthreads();
    if (t == 0) {
      s_free += nok;
      s_ndel += nok;
      s_gen = gen;
    }
    __syncthreads();
  }
  if (t == 0) {
    D.ctr->free_count = s_free;
    D.ctr->claim_gen = s_gen;
    if (carve) {
      D.ctr->last_deleted = s_ndel;
      D.ctr->total_deleted += (unsigned long long)s_ndel;
      D.ctr->total_visible += (unsigned long long)D.ctr->n_vis;
      D.ctr->total_updated += D.ctr->last_updated;
      D.ctr->frames += 1ull;
    }
  }
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
  const int32_t e = find_entry(D.table, bx, by, bz);
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

__global__ __launch_bounds__(256) void k_raycast(EngineDev D, FrameParams P, float step_size,
                                                 uchar4* __restrict__ rgba,
                                                 uchar4* __restrict__ normal) {
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
        prob = reinterpret_cast<const float*>(ref.blk + kProbOffset)[ref.o];
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
// test-level kernels (VoxelHashTable::Retrieve / assignment, VoxelMemPool acquire / release)
// ---------------------------------------------------------------------------------------------
__global__ void k_hash_retrieve(EngineDev D, const int16_t* __restrict__ pts, int n,
                                uint32_t* rgbw, float* tsdf, float* prob, short4* bpo,
                                int32_t* bidx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int16_t x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
  const int16_t bx = (int16_t)(x >> 3), by = (int16_t)(y >> 3), bz = (int16_t)(z >> 3);
  const int32_t e = find_entry(D.table, bx, by, bz);
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
  const int32_t e = find_entry(D.table, (int16_t)(x >> 3), (int16_t)(y >> 3), (int16_t)(z >> 3));
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
      reinterpret_cast<float*>(blk + kProbOffset)[v] = 0.5f;
      blk[kRgbwOffset + 4 * v + 3] = 0;
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
