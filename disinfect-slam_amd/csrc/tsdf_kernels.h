// tsdf_kernels.h -- kernel interface between the kernel files and the engine (tsdf_engine.hip).
#pragma once

#include "tsdf_device.h"

namespace tsdf {

// diagnostic stamp buffer geometry (tsdf_debug_stamps, TSDF_STAMP in tsdf_block.h)
constexpr int kDiagKernels = 9, kDiagMaxWg = 4096, kDiagStamps = 8;

// visible-block lists: one per horizontal image band of the block centre's projection, so the
// integrate kernel can hand each XCD a contiguous, spatially compact slice (its pixel gathers stay
// in that XCD's L2). Counters 128 B apart; list b holds up to nblocks records at vis + b * nblocks.
constexpr int kBands = 16, kBandStride = 32;

// band of a block: the image band its centre projects into (0 when behind the camera)
__device__ __forceinline__ int block_band(const FrameParams& P, int16_t bx, int16_t by, int16_t bz) {
  const float h = 0.5f * (float)(kBlockLen - 1);
  const f3 pw = {((float)(bx << kBlockLenBits) + h) * P.voxel, ((float)(by << kBlockLenBits) + h) * P.voxel,
                 ((float)(bz << kBlockLenBits) + h) * P.voxel};
  const f3 pc = se3_apply(P.cq, P.ct, pw);
  const float v = (P.fy * pc.y + P.cy * pc.z) * __builtin_amdgcn_rcpf(pc.z);
  const float bandf = v * ((float)kBands / (float)P.H);
  return pc.z > 0.f && bandf > 0.f ? min(kBands - 1, f2i(bandf)) : 0;
}

// device pointers of one engine (passed by value to every kernel)
struct EngineDev {
  int4* table;                  // kNumEntry hash entries
  uint32_t* lock_tag;           // kNumBucket bucket locks (== epoch: locked)
  int32_t* heap;                // free-block stack
  uint8_t* pool;                // nblocks x kBlockBytes
  unsigned long long* occ;      // kOccWords occupancy bitmap
  DevCounters* ctr;
  int32_t nblocks;
  int32_t integrate_grid;       // k_integrate workgroups (resident capacity, multiple of 8)
  int32_t integrate_grid_pre;   // k_frame's update workgroups (its resident capacity)
  // per-frame allocation scratch
  unsigned long long* nk_key;   // kNewKeyCap new-key set
  uint32_t* nk_order;           // kNewKeyCap smallest candidate order per key
  NkEnt* nk_list;               // kNewKeyCap occupied slots with their keys
  unsigned long long* pairs;    // max(kNewKeyCap, nblocks): resolver scratch (sort key << 32 | index)
  int32_t* fresh;               // pool indices acquired by the hash-level test path
  // visibility / carving
  VisRec* vis;                  // kBands x nblocks visible blocks (band-major, any order within)
  int32_t* band;                // kBands x kBandStride: record count of each band list
  VisRec* cand;                 // cand_cap carve candidates (any order; sorted by entry)
  int32_t* ncand;               // their count (frame views: one list + count per frame parity)
  int32_t cand_cap;             // records D.cand holds (<= the D.pairs scratch, >= 1024)
  unsigned long long* arrive;   // kArriveWords: last-arriver counters of the frame kernels
  unsigned long long* swdirty;  // kOccWords / 64: occupancy words the carving changed (tsdf_resolve.h)
  VisRec* fresh_vis;            // kNewKeyCap blocks created this frame (k_resolve_alloc frame mode)
  VisRec* pend;                 // kNewKeyCap: a shard's owned entries its exhausted pool left without
                                // voxels this frame (ctr->n_pend); carved in the same frame
  // packed frame: two buffers of max_pixels records each (FrameParams.pix_off selects one)
  float4* pixA;                 // {depth, range, logf(ht), logf(lt)} (sem_logf)
  uint32_t* pixC;               // rgb (r | g << 8 | b << 16)
  // pipelined frames (k_frame): flags, per-frame statistics and the per-pool-block tags
  unsigned long long* pipe;     // kPipeWords (layout below)
  uint32_t* ctag;               // 2 x nblocks: ctag[(f & 1) * nblocks + b] == f: block b was a carve
                                //   candidate of frame f
  uint32_t* rtag;               // nblocks: rtag[b] == f: frame f's carving released block b
  unsigned long long* fo;       // kNumEntry: (~f << 32) | order: frame f's DDA found the key of entry
                                //   e in the table, with this smallest candidate order
  // query scratch
  unsigned long long* visbits;  // kOccWords
  int32_t* wgcnt;               // kOccWords / 256
  unsigned long long* dbg;      // diagnostic stamps (DIAG builds), else unused
};

// View grid of one raycast: a dense cube of n^3 block cells around the camera, wide
// enough for every voxel a ray of the call can read (marched length + binary search + gradient
// neighbours), each cell the block's pool index tagged with the call's generation (stale cells of
// earlier calls read as missing, so nothing is cleared per call), plus occupancy bitmaps of its
// 4^3-block bricks and 16^3-block superbricks that the raycast workgroups stage in LDS to skip empty
// space. n == 0: no grid (a view too deep for it); the raycast then looks every block up in the hash
// table.
constexpr int kViewIdxBits = 22;                  // pool index bits of a cell (gen in the top 10)
constexpr uint32_t kViewGenMax = 1023u;           // generations 1..1023, then the cells are zeroed
constexpr int kViewMaxN = 256;                    // cells per axis at most (64 bricks per axis)
constexpr int kViewBitmapWords = (kViewMaxN / 4) * (kViewMaxN / 4) * (kViewMaxN / 4) / 32 +
                                 (kViewMaxN / 16) * (kViewMaxN / 16) * (kViewMaxN / 16) / 32;
constexpr int kViewGraphBitmapWords = 4608;       // LDS bitmap words of the graph's raycast node
struct ViewGrid {
  uint32_t* cell;          // nb^3 bricks x 64 cells, brick-major: gen << kViewIdxBits | pool index
  uint8_t* flags;          // kViewBitmapWords * 32 bytes: brick / superbrick occupied (1), word w's bits
                           // at bytes [32 w, 32 w + 32); zero between calls (k_view_pack clears them)
  uint32_t* bits;          // the packed bitmaps: nb^3 brick bits, then ns^3 superbrick bits
  int n, nb, ns, half;     // cells, bricks (ceil(n / 4)), superbricks (ceil(nb / 4)) per axis
  int nbw, nw;             // brick words, all bitmap words
  uint32_t gen;
};
// cell of block (lx, ly, lz) of the grid in brick k: the 4x4x4 cells of a brick are one 256-B run, so
// the blocks a ray bundle meets in one brick share cache lines
__device__ __forceinline__ size_t view_cell(int k, int lx, int ly, int lz) {
  return ((size_t)k << 6) | (uint32_t)(((lz & 3) << 4) | ((ly & 3) << 2) | (lx & 3));
}
// origin (block coordinates) of the view grid of camera centre wt: both kernels compute it alike
__device__ __forceinline__ int view_origin(float wt, float voxel, int half) {
  return (f2i(floorf(wt / voxel)) >> kBlockLenBits) - half;
}

// ---- pipelined frames (k_frame, tsdf_fuse.hip; DESIGN.md 4 "Pipelined frames") ----
// A frame f in flight keeps its visible lists at vis + (f & 1) * kBands * nblocks, their counts at
// band + (f % 3) * kBands * kBandStride (reset by f's carving, two launches after the sweep wrote
// them), its carve candidates at cand + (f & 1) * cand_cap with the count in pipe[kPipeNCand + 16 (f & 1)].
// D.pipe layout (u64 words; every hot word on its own 128-B line):
constexpr int kPipeNCand = 0;                   // + 16 p: carve-candidate count of parity p (int32)
constexpr int kPipeCarved = 32;                 // + 16 x: the carving-done flag, copy of XCD x (= tag)
constexpr int kPipeAlloc = kPipeCarved + 128;   // + 16 x: the allocation-done flag (= tag)
constexpr int kPipeT0 = kPipeAlloc + 128;       // + 16 p: first update workgroup's start (parity p)
constexpr int kPipeIngEnd = kPipeT0 + 32;       // + 16 p: the latest sweep / tile workgroup end
constexpr int kPipeAPub = kPipeIngEnd + 32;     // + 16 p: allocation published (the ingest span start)
constexpr int kPipeStats = 512;                 // + 1024 p + 16 i: payload (blocks << 40 | voxels) and,
constexpr int kPipeStatLines = 64;              //   at +1, the latest end stamp of update counter i
constexpr int kPipeWords = kPipeStats + 2 * kPipeStatLines * 16;
constexpr int kFrameUpdWgsPer2Cu = 5;           // default k_frame update workgroups per two CUs (TSDF_FRAME_WG_PER_CU)
constexpr int kPipeHead = 8;                    // workgroups before the update's (0: carving + allocation)
constexpr int kPipeFreshWG = 64;                // workgroups that update the blocks allocated in the launch
constexpr int kPipeDefer = 32;                  // deferred (carve-pending) blocks one update workgroup holds
constexpr int kPipeList = 64;                   // records one update workgroup collects before updating them
// What one k_frame launch does. Frame ids f are engine-wide (1, 2, ...); frame b's update, frame
// b - 1's carving and frame c = b + 1's ingest share the launch (any part may be absent).
struct PipeArgs {
  int has_carve;        // carve frame fid_carve (its candidates, listed by its update last launch)
  int has_alloc;        // allocate frame fid_alloc (= b: its new keys, inserted by last launch's tiles)
  int has_update;       // update frame b's blocks (its lists from last launch's sweep)
  int fresh_ready;      // b's new blocks were listed by an earlier launch (no allocation in this one)
  int has_frame;        // frame c's ingest: pixel records, DDA, probe / insert, visibility sweep
  uint32_t fid_carve, fid_alloc, fid_new;
  uint32_t tag;         // this launch's flag value
  uint32_t range;       // candidate order space of frame b (W H maxs)
  int tiles_x, tiles;   // frame c's pixel tiles
  int tile_wgs;         // the workgroups that run them (tiles_per_wg consecutive tiles each)
  int tiles_per_wg;
  int nint;             // update workgroups (a multiple of 8)
  int order;            // grid order of the parts after the head (TSDF_FRAME_ORDER): 0 fresh, update,
                        //   tiles, sweep; 1 fresh, tiles, sweep, update; 2 fresh, sweep, update, tiles;
                        //   3 tiles, sweep, update, the update after the allocation flag (no fresh
                        //   workgroups: the update takes the new blocks too); 4 update, tiles, sweep,
                        //   every part after the allocation flag (the head's resolvers alone)
  // a shard's pipelined frame (tsdf_integrate_shard_pipe): every shard's carve candidates of frame
  // fid_carve, all-gathered (nshard slots of cand_cap records; merged before the carving), and this
  // shard's slot that the update's last workgroup fills with frame fid_alloc's candidates
  const struct ShardRec* cands_in;
  struct ShardRec* cands_out;
  int cand_cap, nshard;
  // a group's frame (tsdf_group_*): the update's last workgroup writes the slot into each of these
  // ndst slots (device array: this shard's slot of every shard's inbox) instead of cands_out
  struct ShardRec* const* cands_dst;
  int ndst;
};
// frame f's view of the engine: its visible lists, their counts, its carve candidates and count
__device__ __host__ __forceinline__ EngineDev frame_view(const EngineDev& D, uint32_t f) {
  EngineDev V = D;
  V.vis = D.vis + (size_t)(f & 1u) * kBands * (size_t)D.nblocks;
  V.band = D.band + (size_t)(f % 3u) * kBands * kBandStride;
  V.cand = D.cand + (size_t)(f & 1u) * (size_t)D.cand_cap;
  V.ncand = reinterpret_cast<int32_t*>(D.pipe + kPipeNCand + 16 * (f & 1u));
  return V;
}
// the workgroups that update the blocks a launch's allocation creates (orders 0-2)
__device__ __host__ __forceinline__ int pipe_fresh_wgs(const PipeArgs& A) {
  return A.has_update && !A.fresh_ready && A.order < 3 ? kPipeFreshWG : 0;
}
// per-frame arguments of the graph-captured frame loop (tsdf_graph_*): the graph's first node
// copies them from a pinned host slot, every graph kernel reads its camera / frame pointers here
struct FrameArgs {
  FrameParams P;  // integrate camera (cam_T_world, intrinsics, frame size)
  FrameParams R;  // render camera of the raycast node
  const float* depth;
  const uint8_t* rgb;
  const float* ht;
  const float* lt;
  uchar4* rgba;
  uchar4* normal;
  float step_size;  // raycast step (truncation / 2)
  ViewGrid V;       // the raycast node's view grid (n == 0: hash lookups)
  uint32_t vtag;    // the render graph's update node (k_integrate_vg_g): the carving's release tag
  uint32_t range;   // candidate order space W * H * maxs
  int tiles_x, tiles;
  // a shard's graph frame (tsdf_graph_shard_*): the exchange slots of its three segments
  ShardRec* keys_out;        // k_ingest_dda_g's tail packs the slice's keys here (P.tail / P.slot)
  const ShardRec* keys_in;   // k_resolve_alloc_g merges the all-gathered key slots
  int key_cap;
  ShardRec* cands_out;       // k_integrate_t<true, .>'s tail packs the carve candidates here
  const ShardRec* cands_in;  // k_resolve_delete_g merges the all-gathered candidate slots
  int cand_cap, nshard;
  // a pipelined graph frame (k_frame_g): P is the new frame's (depth ... lt set in it), Pu the
  // camera / pixel records of the frame whose allocation and update run, pipe what the launch does
  FrameParams Pu;
  PipeArgs pipe;
  // a render-deferring graph frame: the previous frame's args slot, whose raycast this launch runs
  // beside its ingest (k_render_ingest_g); null: none
  const FrameArgs* prev;
};

__global__ void k_init_table(int4* table);
__global__ void k_copy_words(uint32_t* dst, const uint32_t* src, int n);
__global__ void k_init_heap(int32_t* heap, int n);
__global__ void k_init_prob(uint8_t* pool, int nb);
// last-arriver counters (tsdf_resolve.h arrive_last), one 128-B line each: lines [0, 9) k_ingest_dda,
// [16, 25) k_integrate, line 32 k_integrate's start stamp
// first-level arrival counters per kernel (workgroup b arrives at counter b % kArrGroups: a multiple
// of 8, so every counter's workgroups share an XCD), then one top counter
#ifndef TSDF_ARRIVE_GROUPS
#define TSDF_ARRIVE_GROUPS 8
#endif
constexpr int kArrGroups = TSDF_ARRIVE_GROUPS;
static_assert(kArrGroups % 8 == 0 && kArrGroups <= 128, "arrival counters");
constexpr int kArrStride = (kArrGroups + 1) * 16;  // u64 words of one kernel's counter lines
constexpr int kArrIngest = 0, kArrIntegrate = kArrStride, kArrStart = 2 * kArrStride,
              kArriveWords = 2 * kArrStride + 32;
// per frame (2 launches; the resolvers run in the last workgroup of each)
constexpr int kVisWorkgroups = kOccWords / 256;  // visibility-sweep workgroups of k_ingest_dda
template <int TS>  // LDS key-set slots per tile (tsdf_alloc.hip): 1024 for maxs <= 3, else 2048
__global__ void k_ingest_dda(EngineDev D, FrameParams P, const float* depth, const uint8_t* rgb,
                             const float* ht, const float* lt, int tiles_x, int tiles);
// standalone one-workgroup resolvers (sharded frames after an exchange; the hash-level test path).
// keys_in: optional inbox of nshard key slots merged into the new-key set first.
__global__ void k_resolve_alloc(EngineDev D, FrameParams P, uint32_t range, int frame_mode,
                                const ShardRec* keys_in, int cap, int nshard);
// graph-captured forms of a shard's standalone resolvers (arguments from FrameArgs)
__global__ void k_resolve_alloc_g(EngineDev D, const FrameArgs* A);
__global__ void k_resolve_delete_g(EngineDev D, const FrameArgs* A);
template <bool Graph, bool Raw>
__global__ void k_integrate_t(EngineDev D, FrameParams P, const FrameArgs* A);
__global__ void k_frame(EngineDev D, FrameParams Pu, FrameParams Pn, PipeArgs A);
__global__ void k_frame_g(EngineDev D, const FrameArgs* FA);
// the update of one frame b with its carving in the same launch (unpipelined tail form): see k_integrate_t
// graph-captured forms of the frame kernels: identical bodies, arguments from FrameArgs
template <int TS>
__global__ void k_ingest_dda_g(EngineDev D, const FrameArgs* A);
__global__ void k_raycast_g(EngineDev D, const FrameArgs* A);
// cands_in: optional inbox of nshard carve-candidate slots (then recs / count are D.cand / n_cand)
__global__ void k_resolve_delete(EngineDev D, const VisRec* recs, const int32_t* count, int direct,
                                 const ShardRec* cands_in, int cap, int nshard);
// hash-level test path
__global__ void k_keys_to_newset(EngineDev D, const int16_t* keys, int n);
constexpr int kMaxShards = 64;
// DISINFSystem::feed_rgbd_frame preprocessing (tsdf_frontend.hip); grid (ceil(w / 64), ceil(h / 4))
__global__ void k_rgbd_half(const uint8_t* rgb, const uint16_t* depth, const uint8_t* mask, int W,
                            int H, float alpha, uint8_t* rgb_out, float* depth_out);
__global__ void k_fresh_init(EngineDev D);
// tsdf_integrate_shard_abort: a pending sharded frame's per-frame state back to "between frames"
__global__ void k_shard_abort(EngineDev D);
// extraction
struct MeshParams {
  float voxel, missing;
  int min_weight;
  int own_index, own_count;  // own_count > 1: only blocks whose brick owner is own_index emit (a
                             // shard's part of a sharded mesh; the other selected blocks are its halo)
};
// k_mesh / k_scan_counts read the selected-block count from device memory (*nsel, written by
// k_vis_emit), so a whole extraction is enqueued without a host round trip: k_mesh runs
// min(kMeshGrid, pool blocks) workgroups, one selected block each (the rest exit) and grid-stride
// past kMeshGrid; the emit pass writes nothing when the total exceeds `capacity` triangles. The count
// pass keeps each block's 27 neighbour pool indices in nbr (27 per selected block) and its triangle
// count in counts; the emit pass reads both (no hash probes, blocks without triangles skipped).
constexpr int kMeshGrid = 8192;
template <bool Emit>
__global__ void k_mesh(EngineDev D, const VisRec* sel, const int32_t* nsel, MeshParams M, int32_t* counts,
                       const int32_t* offsets, const int64_t* total, int64_t capacity, int32_t* nbr, float* out);
__global__ void k_scan_counts(const int32_t* counts, const int32_t* nsel, int32_t* offsets, int64_t* total);
__global__ void k_raycast(EngineDev D, FrameParams P, float step_size, ViewGrid V, uchar4* rgba,
                          uchar4* normal);
// frame n's raycast (R, V: its view grid, built before) + frame n + 1's ingest (k_ingest_dda<1024>) in
// one launch: nray raycast workgroups (rgx tiles per row) first, then kVisWorkgroups + tiles (tsdf_alloc.hip)
__global__ void k_render_ingest(EngineDev D, FrameParams R, float step_size, ViewGrid V, uchar4* rgba,
                                uchar4* normal, int rgx, int nray, FrameParams P, const float* depth,
                                const uint8_t* rgb, const float* ht, const float* lt, int tiles_x, int tiles);
// (graph form: A->prev's raycast, none when null, beside A's ingest)
__global__ void k_render_ingest_g(EngineDev D, const FrameArgs* A, int rgx, int nray);
// k_integrate plus the render camera's view grid (the C5 loop's deferred raycast; tsdf_fuse.hip)
__global__ void k_integrate_vg(EngineDev D, FrameParams Pv, FrameParams R, ViewGrid V, uint32_t vtag, int nint);
__global__ void k_integrate_vg_g(EngineDev D, const FrameArgs* A, int nint);
// view grid of a raycast: grid kOccWords / 256 workgroups of 256
__global__ void k_view_grid(EngineDev D, FrameParams P, ViewGrid V);
__global__ void k_view_grid_g(EngineDev D, const FrameArgs* A);
// flags -> bits (and the flags cleared): kViewPackGrid workgroups of 256, one word per thread
constexpr int kViewPackGrid = (kViewBitmapWords + 255) / 256;
__global__ void k_view_pack(ViewGrid V);
__global__ void k_view_pack_g(const FrameArgs* A);
__global__ void k_query_count(EngineDev D, int use_bounds, short4 lo, short4 hi);
__global__ void k_vis_emit(EngineDev D, VisRec* out, int32_t* out_count);
__global__ void k_query_download(EngineDev D, const VisRec* sel, float voxel, float4* out);
// render replicas of a sharded volume (tsdf_render_blocks / tsdf_import_blocks)
constexpr int kBlockRecBytes = 16 + kBlockBytes;  // {int16 x, y, z, 0; 8 zero bytes} + payload
struct RenderCull {
  float a0, a1, b0, b1;      // x/z and y/z of the pixel-centre pyramid's four side planes
  float na0, na1, nb0, nb1;  // their normal lengths sqrt(1 + a^2)
  float reach;               // block bounding radius + lookup reach (m)
  float len;                 // marched ray length + reach (m)
};
__global__ void k_render_count(EngineDev D, FrameParams P, RenderCull C);
// grouped selections (render bands / marching-cubes halo destinations), tsdf_extract.hip
constexpr int kMaxGroups = 64;
constexpr int kGroupBands = 0, kGroupHalo = 1;
struct GroupSel {
  int mode, ngroups;
  RenderCull cull;                 // kGroupBands: the camera's pyramid (b0 / b1 per band below)
  float b0[kMaxGroups], b1[kMaxGroups], nb0[kMaxGroups], nb1[kMaxGroups];
};
__global__ void k_group_count(EngineDev D, FrameParams P, GroupSel S, unsigned long long* visbits,
                              int32_t* wgcnt);
__global__ void k_render_pack(EngineDev D, const VisRec* sel, uint8_t* out);
__global__ void k_import_keys(EngineDev D, const uint8_t* recs, int n);
__global__ void k_import_payload(EngineDev D, const uint8_t* recs, int32_t* missing);
__global__ void k_hash_retrieve(EngineDev D, const int16_t* pts, int n, uint32_t* rgbw,
                                float* tsdf, float* prob, short4* bpo, int32_t* bidx);
__global__ void k_hash_assign(EngineDev D, const int16_t* pts, int n, const uint32_t* rgbw,
                              int* missing);
__global__ void k_pool_acquire(EngineDev D, int n, int32_t* out);
__global__ void k_pool_release(EngineDev D, const int32_t* idx, int n);
__global__ void k_pool_weight(EngineDev D, int32_t block, int set, uint8_t w, uint8_t* out);
__global__ void k_dump_table(EngineDev D, short4* pos, int32_t* idx);
__global__ void k_dump_pool(EngineDev D, float* tsdf, float* prob, uint32_t* rgbw);

}  // namespace tsdf
