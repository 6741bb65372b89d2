/*
 * tsdf_oracle.h -- CPU restatement of the reference TSDF engine (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X engine in disinfect-slam_amd/. It restates, in plain
 * C11, the semantics of the reference CUDA path yuzhou42/disinfect-slam utils/tsdf (all files) and the
 * helpers it uses in utils/cuda (citations per function in tsdf_oracle.c). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * Pinning: the hash-table / memory-pool semantics are pinned by the reference's own known-answer
 * tests (utils/tests/voxel_hash_test.cu Single/Multiple/Collision, utils/tests/voxel_mem_test.cu
 * Test1), re-run against this oracle in tests/test_oracle_kat.py. Integrate / carve / raycast /
 * query numerics have NO reference golden vectors (the reference cannot be built here: nvcc,
 * Eigen and OpenCV are absent) -- they are "pinned by restatement" (SURVEY.md 8c).
 *
 * Canonical linearisation of the reference's racy allocation: Allocate
 * runs sequentially in candidate order (pixel raster order y, x, then DDA step i) with the exact
 * bucket-lock semantics of voxel_hash.cu:58-120; Delete runs sequentially in visible-block
 * (hash-entry) order. Build with -O2 -ffp-contract=off (no FMA contraction, IEEE float).
 */
#ifndef TSDF_ORACLE_H
#define TSDF_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_grid ora_grid;

typedef struct ora_stats {
  int64_t frames;
  int32_t last_num_visible;   /* N_vis of the last integrate */
  int64_t last_num_updated;   /* N_upd (voxels updated) of the last integrate */
  int32_t last_num_alloc;     /* successful block allocations of the last integrate */
  int32_t last_num_deleted;   /* successful block deletions (space carving) of the last integrate */
  int32_t last_num_candidates;/* unique missing keys attempted in the last allocate launch */
  int32_t active_blocks;      /* NUM_BLOCK - free */
  int32_t last_cross_losses;  /* sharded grids: keys of the last allocate launch that lost a bucket
                                 lock to a key another shard owns */
  int32_t pool_exhausted;     /* sticky: an owned allocation found no free block */
} ora_stats;

/* voxel_tsdf.cu:309 TSDFGrid(voxel_size, truncation); num_block_bits replaces NUM_BLOCK_BITS=18
 * (voxel_mem.cuh:11) so tests can run small pools. */
ora_grid* ora_create(float voxel_size, float truncation, int num_block_bits);
void ora_destroy(ora_grid* g);
/* Spatial sharding (not in the reference): the grid becomes shard
 * `index` of `count` of one volume. It keeps the whole hash index (entries of blocks another shard
 * owns carry idx ORA_FOREIGN = 0x7FFFFFFF: occupied for Allocate / Delete, missing for readers)
 * and holds voxels only for the blocks whose 4^3-block brick hashes to it (ora_block_owner). A
 * shard integrates through the three phases below, with the union of every shard's keys and carve
 * candidates between them; ora_integrate refuses it. count <= 1: one volume. */
void ora_set_shard(ora_grid* g, int index, int count);
/* phase 1: DDA over pixel rows [row_lo, row_hi): unique fully visible keys missing from the index
 * with their smallest candidate order ((y W + x) << 8 | step); returns the count (outputs filled up
 * to capacity). */
int64_t ora_shard_keys(ora_grid* g, const float* depth, int W, int H, const float K[4],
                       const float q[4], const float t[3], float max_depth, int row_lo, int row_hi,
                       int16_t* keys_out, uint64_t* orders_out, int64_t capacity);
/* phase 2: Allocate of the union of all shards' keys in candidate order, then visibility, update
 * and carve test of the owned blocks; returns the owned carve candidates (entry order, outputs
 * filled up to cand_cap). */
int64_t ora_shard_update(ora_grid* g, const int16_t* keys, const uint64_t* orders, int64_t n,
                         const uint8_t* rgb, const float* depth, const float* ht, const float* lt,
                         int W, int H, const float K[4], const float q[4], const float t[3],
                         float max_depth, int16_t* cand_pos, int32_t* cand_entry, int64_t cand_cap);
/* phase 3: Delete of the union of all shards' carve candidates in entry order. */
void ora_shard_delete(ora_grid* g, const int16_t* cand_pos, const int32_t* cand_entry, int64_t n);
/* Marching cubes over the selected blocks (bounds as ora_query, NULL = all); 9 floats per
 * triangle into out (up to capacity triangles); returns the triangle count. See the .c. */
int64_t ora_extract_mesh(const ora_grid* g, const float* bounds, float missing, int min_weight,
                         float* out, int64_t capacity);
/* the oracle's own marching-cubes case table (ora_mc_cases.c): edges 12 x 2 corner pairs, triangle
 * counts per case, triangles 256 x 15 edge indices (-1 padded); returns the triangles per case */
int ora_mc_table(int8_t* edges, uint8_t* ntri, int8_t* tri);
uint32_t ora_block_owner(int16_t x, int16_t y, int16_t z, uint32_t shards);

/* voxel_tsdf.cu:347-375 TSDFGrid::Integrate. rgb: HxWx3 u8; depth/ht/lt: HxW f32 (ht/lt may be
 * NULL -> 1.0, tsdf_module.cc:29-33). K = {fx, fy, cx, cy}; cam_T_world = (q xyzw, t). */
int ora_integrate(ora_grid* g, const uint8_t* rgb, const float* depth, const float* ht,
                  const float* lt, int W, int H, const float K[4], const float q[4],
                  const float t[3], float max_depth);

/* voxel_tsdf.cu:490-506 RayCast (+ ray_cast_kernel :232-307). rgba/normal: HxWx4 u8. */
void ora_raycast(const ora_grid* g, const float K[4], int W, int H, const float q[4],
                 const float t[3], float max_depth, uint8_t* rgba, uint8_t* normal);

/* voxel_tsdf.cu:399-454 GatherValid (bounds == NULL) / GatherVoxels(bounds = xmin,xmax,ymin,ymax,
 * zmin,zmax). Returns number of voxels; out (x,y,z,tsdf float quadruples) filled if non-NULL and
 * capacity suffices. */
int64_t ora_query(const ora_grid* g, const float* bounds, float* out, int64_t capacity);

void ora_get_stats(const ora_grid* g, ora_stats* s);

/* Full state dump (test-only): table entries (x,y,z,offset int16 x4 + idx int32), heap, free
 * counter, SoA voxel pools (tsdf f32, prob f32, rgbw u8x4) of all NUM_BLOCK blocks. Any NULL
 * pointer is skipped. */
void ora_dump(const ora_grid* g, int16_t* entry_pos_off, int32_t* entry_idx, int32_t* heap,
              int32_t* free_count, float* tsdf, float* prob, uint8_t* rgbw);
int32_t ora_num_entries(void);
int32_t ora_num_blocks(const ora_grid* g);

/* --- hash-table / pool level operations (voxel_hash.cu, voxel_mem.cu), used by the KATs --- */
/* One "launch" of Allocate over keys[n] (xyz int16 triples) in list order, then ResetLocks. */
void ora_hash_allocate(ora_grid* g, const int16_t* keys, int n);
/* One "launch" of Delete over keys[n] in list order, then ResetLocks. */
void ora_hash_delete(ora_grid* g, const int16_t* keys, int n);
/* Retrieve (voxel_hash.cuh:104-161) of voxel points[n]: rgbw (u8x4), tsdf, prob, and the block
 * meta found (x,y,z,offset int16 x4, idx int32; idx -1 when missing). */
void ora_hash_retrieve(const ora_grid* g, const int16_t* points, int n, uint8_t* rgbw,
                       float* tsdf, float* prob, int16_t* block_pos_off, int32_t* block_idx);
/* RetrieveMutable + assignment (voxel_hash_test.cu:47-54). Returns #points not found. */
int ora_hash_assign(ora_grid* g, const int16_t* points, int n, const uint8_t* rgbw);
int32_t ora_num_active_blocks(const ora_grid* g);
/* voxel_mem.cu:37-61 AquireBlock / ReleaseBlock sequentially. */
void ora_pool_acquire(ora_grid* g, int n, int32_t* idx_out);
void ora_pool_release(ora_grid* g, const int32_t* idx, int n);
void ora_pool_set_weight(ora_grid* g, int32_t block_idx, uint8_t weight);
void ora_pool_get_weights(const ora_grid* g, int32_t block_idx, uint8_t* out512);
uint32_t ora_hash(int16_t x, int16_t y, int16_t z);

/* DISINFSystem::feed_rgbd_frame preprocessing (disinfect_slam/disinfect_slam.cc:31-64):
 * cv::resize(.., 0.5, 0.5) of rgb (HxWx3 u8), depth (HxW u16) and the optional mask (HxW u8),
 * depth.convertTo(CV_32FC1, 1. / depth_factor), depth = 0 where the resized mask is 0. W and H
 * must be even. OpenCV is not vendored: see the .c for the published algorithm restated. */
void ora_rgbd_half(const uint8_t* rgb, const uint16_t* depth, const uint8_t* mask, int W, int H,
                   float depth_factor, uint8_t* rgb_out, float* depth_out);

/* The logf / expf of the semantic update (voxel_tsdf.cu:196-202), fixed as explicit float
 * algorithms (ora_math.c: why, and how accurate). Test support: ora_math_digest sums a mix of every
 * result over the input bit patterns [lo, hi) (kind 0 logf, 1 expf) for the GPU comparison;
 * ora_math_accuracy compares with the correctly rounded values (out: inputs, differing, max ulp). */
float ora_logf(float x);
float ora_expf(float x);
uint64_t ora_math_digest(int kind, uint64_t lo, uint64_t hi);
void ora_math_accuracy(int kind, uint64_t lo, uint64_t hi, uint64_t step, double* out);

#ifdef __cplusplus
}
#endif
#endif
