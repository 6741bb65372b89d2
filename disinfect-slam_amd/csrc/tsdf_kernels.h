// tsdf_kernels.h -- kernel interface between tsdf_kernels.hip and the engine (tsdf_engine.hip).
#pragma once

#include "tsdf_device.h"

namespace tsdf {

// device pointers of one engine (passed by value to every kernel)
struct EngineDev {
  int4* table;                  // kNumEntry hash entries
  uint32_t* lock_tag;           // kNumBucket
  unsigned long long* claim;    // kNumBucket resolver claims
  int32_t* heap;                // free-block stack
  uint8_t* pool;                // nblocks x kBlockBytes
  unsigned long long* occ;      // kOccWords occupancy bitmap
  DevCounters* ctr;
  int32_t nblocks;
  // per-frame allocation scratch
  unsigned long long* nk_key;   // kNewKeyCap
  uint32_t* nk_order;           // kNewKeyCap
  int32_t* nk_list;             // kNewKeyCap
  unsigned long long* obits;    // candidate-order bitmap
  int32_t* order_slot;          // candidate order -> nk slot
  int32_t* sorted;              // candidate orders of new keys, increasing
  int32_t* fresh;               // pool indices acquired this frame
  // visibility / carving scratch
  unsigned long long* visbits;  // kOccWords
  int32_t* wgcnt;               // per-workgroup compaction counts
  VisRec* vis;                  // visible-block snapshot (entry order)
  unsigned long long* candbits; // carve candidates (bit = visible position)
  int32_t* cand;                // carve candidates, increasing visible position
  float4* pix;                  // packed frame {depth, ht, lt, rgb}
};

__global__ void k_init_table(int4* table);
__global__ void k_init_heap(int32_t* heap, int n);
__global__ void k_ingest_dda(EngineDev D, FrameParams P, const float* depth, const uint8_t* rgb,
                             const float* ht, const float* lt);
__global__ void k_keys_to_newset(EngineDev D, const int16_t* keys, int n);
__global__ void k_order_mark(EngineDev D);
__global__ void k_compact_count(const unsigned long long* bits, int nwords, int32_t* wgcnt);
__global__ void k_compact_emit(unsigned long long* bits, int nwords, const int32_t* wgcnt, int nwg,
                               int32_t* out, int32_t* out_count);
__global__ void k_resolve_alloc(EngineDev D, int count_stats);
__global__ void k_fresh_init(EngineDev D);
__global__ void k_vis_count(EngineDev D, FrameParams P);
__global__ void k_query_count(EngineDev D, int use_bounds, short4 lo, short4 hi);
__global__ void k_vis_emit(EngineDev D, VisRec* out, int32_t* out_count);
__global__ void k_integrate(EngineDev D, FrameParams P);
__global__ void k_resolve_delete(EngineDev D, const int32_t* list, const int32_t* count,
                                 const VisRec* recs, int chunk, int carve);
__global__ void k_raycast(EngineDev D, FrameParams P, float step_size, uchar4* rgba,
                          uchar4* normal);
__global__ void k_query_download(EngineDev D, const VisRec* sel, float voxel, float4* out);
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
