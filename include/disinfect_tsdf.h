/*
 * disinfect_tsdf.h -- C ABI of the MI355X (gfx950) TSDF semantic-fusion engine.
 *
 * Drop-in boundary for the TSDF hot path of yuzhou42/disinfect-slam. The reference exposes this
 * path as C++ classes (no FFI): TSDFGrid (utils/tsdf/voxel_tsdf.cuh:32-124), VoxelHashTable
 * (utils/tsdf/voxel_hash.cuh:47-183), VoxelMemPool (utils/tsdf/voxel_mem.cuh:95-174) and the
 * threaded TSDFSystem facade (modules/tsdf_module.h:35-107). Each entry point below names the
 * reference interface it replaces. Plain pointers and sizes only: no HIP, torch or OpenCV types.
 * The C++17 facade in disinfect-slam_amd/host/ rebuilds TSDFGrid / TSDFSystem on top of it.
 *
 * All calls return TSDF_OK (0) or a TSDF_ERR_* code; nothing throws across this boundary
 * (the reference returns void and only printf's CUDA errors in Debug, utils/cuda/errors.cuh:9-29).
 * An engine handle is not thread safe (TSDFGrid is not re-entrant either); TSDFSystem serialises.
 */
#ifndef DISINFECT_TSDF_H
#define DISINFECT_TSDF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSDF_OK 0
#define TSDF_ERR_INVALID_ARG 1
#define TSDF_ERR_OUT_OF_MEMORY 2
#define TSDF_ERR_HIP 3
#define TSDF_ERR_CAPACITY 4 /* caller buffer too small (two-call pattern) */
#define TSDF_ERR_NO_DEVICE 5
#define TSDF_ERR_PIPELINE 6 /* tsdf_synchronize: a pipelined frame's wait timed out since the last report
                               (results wrong); the status bit is cleared once reported */

#define TSDF_MEM_HOST 0   /* pointer is host memory: engine copies it (pageable is fine) */
#define TSDF_MEM_DEVICE 1 /* pointer is device memory on the engine's GPU */

/* status bits (tsdf_stats.status): sticky, cleared by tsdf_get_stats(..., clear=1) */
#define TSDF_STATUS_POOL_EXHAUSTED 1u  /* an allocation found no free block (voxel_mem.cu:39) */
#define TSDF_STATUS_NEWKEY_OVERFLOW 2u /* more new blocks in one frame than the key set holds */
#define TSDF_STATUS_DDA_OVERFLOW 4u    /* a DDA ray took more samples than sized for */
#define TSDF_STATUS_RESOLVE_ABORT 8u   /* allocation resolver made no progress (internal error) */
#define TSDF_STATUS_SHARD_OVERFLOW 16u /* a sharded frame had more keys / candidates than a slot holds */
#define TSDF_STATUS_SHARD_ABORTED 32u  /* a pending sharded frame was aborted (the shards may differ) */
#define TSDF_STATUS_PIPELINE_TIMEOUT 64u /* a pipelined frame's in-kernel wait timed out (internal error) */

typedef struct tsdf_engine tsdf_engine;
typedef struct tsdf_graph tsdf_graph;

typedef struct tsdf_config {
  float voxel_size;   /* [m] TSDFGrid(voxel_size, truncation), voxel_tsdf.cuh:40 */
  float truncation;   /* [m] */
  int max_width;      /* largest integrate / raycast image; reference MAX_IMG_* = 1920x1080 */
  int max_height;     /*   (voxel_tsdf.cu:10-12) */
  int num_block_bits; /* voxel-block pool = 2^bits blocks; reference NUM_BLOCK_BITS 18 */
  int shard_index;    /* spatial sharding: this engine holds the voxels of blocks b with */
  int shard_count;    /*   owner(b) = hash(b >> 2) mod count == index; 1 = unsharded (<= 64) */
  void* stream;       /* hipStream_t to run on when use_stream != 0 (NULL then means the legacy */
  int use_stream;     /*   default stream); use_stream == 0: an engine-owned stream */
} tsdf_config;

/* Fill reference defaults: 5 mm / 3 cm, 1920x1080, 2^18 blocks, unsharded. */
void tsdf_config_default(tsdf_config* cfg);

typedef struct tsdf_intrinsics { /* CameraIntrinsics<float> (utils/cuda/camera.cuh:12-51) */
  float fx, fy, cx, cy;
} tsdf_intrinsics;

typedef struct tsdf_pose { /* SE3<float> cam_T_world (utils/cuda/lie_group.cuh:6-45) */
  float qx, qy, qz, qw;    /* Eigen::Quaternionf coefficients (x, y, z, w) */
  float tx, ty, tz;
} tsdf_pose;

typedef struct tsdf_frame { /* the four cv::Mat inputs of TSDFGrid::Integrate (voxel_tsdf.cuh:58) */
  int width, height;
  const uint8_t* rgb;  /* height x width x 3, RGB order (CV_8UC3) */
  const float* depth;  /* height x width metres (CV_32FC1); 0 = invalid */
  const float* ht;     /* height x width high-touch probability; NULL -> all ones */
  const float* lt;     /* height x width low-touch probability;  NULL -> all ones */
  int mem_kind;        /* TSDF_MEM_HOST or TSDF_MEM_DEVICE (all four pointers alike) */
} tsdf_frame;

typedef struct tsdf_voxel { /* VoxelSpatialTSDF (utils/tsdf/voxel_types.cuh:48-57), 16 B */
  float x, y, z, tsdf;
} tsdf_voxel;

typedef struct tsdf_stats {
  int64_t frames;            /* integrate calls so far */
  int32_t active_blocks;     /* VoxelHashTable::NumActiveBlock (voxel_hash.cu:207) */
  int32_t free_blocks;       /* VoxelMemPool::NumFreeBlocks (voxel_mem.cu:63-67) */
  int32_t last_num_visible;  /* N_vis of the last integrate */
  int32_t last_num_alloc;    /* blocks allocated by the last integrate */
  int32_t last_num_deleted;  /* blocks removed by space carving in the last integrate */
  int32_t last_num_new_keys; /* unique missing visible keys the last DDA produced */
  int64_t last_num_updated;  /* voxels updated by the last integrate */
  int64_t total_visible;     /* sum of N_vis over all integrate calls */
  int64_t total_updated;     /* sum of updated voxels over all integrate calls */
  int64_t total_alloc;
  int64_t total_deleted;
  uint32_t status;           /* TSDF_STATUS_* bits */
  uint32_t reserved;
} tsdf_stats;

typedef struct tsdf_profile { /* device time of the integrate phases between begin/end */
  int64_t frames;      /* integrate calls that were event-timed (every `every`-th call) */
  double ms_allocate;  /* DDA + visibility sweep of the existing blocks (one kernel) + ordered
                          allocation resolve, which lists the new blocks as visible */
  double ms_visible;   /* ~0: visibility runs inside the allocate phase (kept for the layout) */
  double ms_integrate; /* the fused TSDF/RGB/weight/semantic update kernel (+ carve minimum) */
  double ms_carve;     /* space-carving compaction + delete resolve */
  int64_t sum_visible; /* sum of N_vis over the profiled frames */
  int64_t sum_updated; /* sum of updated voxels over the profiled frames */
  double ms_integrate_device; /* k_integrate first-workgroup start -> last-workgroup end, summed
                                 over the profiled frames (in-kernel 100 MHz clock; excludes the
                                 dispatch overhead the HIP events of ms_integrate include) */
  int64_t calls;       /* all integrate calls between begin and end (sum_* and the device
                          clock cover all of them; the ms_* event times only `frames`) */
  /* in-kernel 100 MHz clock, summed over the calls (the two resolvers run inside the ingest and
     update kernels' last-arriving workgroups, so no kernel trace can time them apart): */
  double ms_ingest_device;          /* k_ingest_dda start -> its last workgroup's arrival */
  double ms_resolve_alloc_device;   /* ordered allocation resolve (VoxelHashTable::Allocate) */
  double ms_resolve_delete_device;  /* ordered carving resolve (VoxelHashTable::Delete) */
  int64_t pipelined;   /* pipelined frame launches (k_frame: the previous frame's carving, this
                          frame's allocation and update, the next frame's ingest; their events /
                          device clock include that work) */
} tsdf_profile;

/* ---- engine lifetime: TSDFGrid::TSDFGrid / ~TSDFGrid (voxel_tsdf.cu:309-345) ---- */
int tsdf_create(const tsdf_config* cfg, int device, tsdf_engine** out);
int tsdf_destroy(tsdf_engine* e);

/* TSDFGrid::Integrate (voxel_tsdf.cu:347-375): allocate -> visibility -> update -> carve.
 * Asynchronous on the engine stream when the frame is TSDF_MEM_DEVICE (inputs must stay valid
 * until the next engine call or tsdf_synchronize); host frames are copied before returning.
 * Pipelined frames (one volume, truncation / voxel <= 6 -- at most 3 DDA samples per pixel): the
 * frame's allocation is enqueued at once and its update / carving is deferred; the next
 * tsdf_integrate enqueues it in one launch with the next frame's pixel work, and every other entry
 * point that reads or writes the volume (raycast, query, stats, snapshots, mesh, ..., tsdf_flush,
 * tsdf_synchronize) enqueues it first, so every observable result is that of the frames in order.
 * tsdf_stream_wait / tsdf_stream_signal do not enqueue it (they order the frame's inputs, which the
 * deferred part no longer reads). TSDF_PIPELINE=0 in the environment disables the deferral (on by default). */
int tsdf_integrate(tsdf_engine* e, const tsdf_frame* frame, const tsdf_intrinsics* K,
                   const tsdf_pose* cam_T_world, float max_depth);
/* Enqueue a deferred update (pipelined frames) on the engine stream without waiting for it: after
 * tsdf_flush, a synchronisation of the engine stream covers every frame integrated so far. */
int tsdf_flush(tsdf_engine* e);

/* Sharded volume (no reference counterpart: TSDFGrid is single-GPU). An engine
 * created with shard_count > 1 is shard `shard_index` of one volume: it keeps the whole hash index
 * (VoxelHashTable, voxel_hash.cuh:47-183) and holds the voxels of the blocks whose 4^3-block brick
 * hashes to it (tsdf_block_owner). Every shard applies every Allocate / Delete to its index --
 * another shard's block is an occupied entry without voxels here -- so the bucket-lock outcomes
 * (one structural change per bucket per launch, voxel_hash.cu:80-118,137-170) are those of ONE
 * volume, and the union of the shards equals the unsharded volume block for block and voxel for
 * voxel. TSDFGrid::Integrate (voxel_tsdf.cu:347-375) of a shard is three calls around two
 * exchanges, all asynchronous on the engine stream:
 *   1. tsdf_integrate_shard_begin: the visibility of this shard's blocks and the
 *      block_allocate_kernel DDA (voxel_tsdf.cu:104-147) over slice `slice_index` of `slice_count`
 *      (bands of 16-pixel tile rows). No pixel records are packed: the update in _update gathers
 *      the raw frame again, so a DEVICE frame (depth, rgb, ht, lt) must stay allocated and
 *      unmodified until _update has been enqueued and has run in stream order (a host frame is
 *      staged by _begin and may be reused at once). The keys it finds missing from the index go to
 *      keys_out: one slot of
 *      tsdf_shard_slot_bytes(key_cap) bytes (record 0 = count header, then 16-B records).
 *      slice_count == 1 with keys_out == NULL: every shard runs the whole DDA and finds the same
 *      keys itself, so no key exchange is needed (keys_in NULL below).
 *   2. the caller all-gathers the key slots (e.g. RCCL all-gather over xGMI): keys_in = shard_count
 *      slots, slot s from shard s. tsdf_integrate_shard_update merges them (smallest candidate
 *      order per key = the whole frame's DDA), runs the ordered allocation (pool blocks only for
 *      owned keys), the fused update of this shard's visible blocks, and writes its space-carving
 *      candidates (space_carving_kernel, voxel_tsdf.cu:207-230) to cands_out (one slot).
 *   3. the caller all-gathers the candidate slots; tsdf_integrate_shard_end deletes the union in
 *      hash-entry order (every shard's index) and releases this shard's pool blocks.
 * Exchanges must be ordered between the calls on the engine stream (same stream, or
 * tsdf_stream_wait / tsdf_stream_signal). No other engine call may come between _begin and _end;
 * tsdf_integrate / feed / graph frames refuse a shard. More records than a slot holds set
 * TSDF_STATUS_SHARD_OVERFLOW (the shards then diverge: size the caps for the first frame). */
int64_t tsdf_shard_slot_bytes(int32_t cap);
/* Pipelined sharded frames: ONE exchange per frame (no reference counterpart; the sharded form of
 * TSDFGrid::Integrate, voxel_tsdf.cu:347-375, pipelined like tsdf_integrate). Every shard runs the
 * whole frame's DDA against its copy of the index, so the new keys need no exchange and only the
 * carve candidates cross the shards. Per frame, on every shard: tsdf_integrate_shard_pipe(frame,
 * cands_in, cands_out), then the caller all-gathers cands_out (one slot of
 * tsdf_shard_slot_bytes(cand_cap)) into cands_in (shard_count slots, slot s from shard s) for the next
 * call. The call carves the frame before the previous one (every shard's candidates, from cands_in),
 * allocates and updates the previous frame (this shard's candidates into cands_out) and ingests this
 * one. To complete the frames: call with frame == NULL (and the exchange after each call) until
 * *pending is 0. Until then every other volume entry point returns TSDF_ERR_INVALID_ARG. The frame's
 * buffers are read by this call only. */
int tsdf_integrate_shard_pipe(tsdf_engine* e, const tsdf_frame* frame, const tsdf_intrinsics* K,
                              const tsdf_pose* cam_T_world, float max_depth, const void* cands_in,
                              void* cands_out, int32_t cand_cap, int32_t* pending);
int tsdf_integrate_shard_begin(tsdf_engine* e, const tsdf_frame* frame, const tsdf_intrinsics* K,
                               const tsdf_pose* cam_T_world, float max_depth, int32_t slice_index,
                               int32_t slice_count, void* keys_out, int32_t key_cap);
int tsdf_integrate_shard_update(tsdf_engine* e, const void* keys_in, int32_t key_cap, void* cands_out,
                                int32_t cand_cap);
int tsdf_integrate_shard_end(tsdf_engine* e, const void* cands_in, int32_t cand_cap);
/* Abort a pending sharded frame (e.g. a failed exchange between the phases) or the pending frames of
 * tsdf_integrate_shard_pipe: the engine returns to "between frames" so later calls (a new frame,
 * reset, snapshot_load, ...) work again. Structural changes a phase already made stay, so the shards
 * may no longer agree: TSDF_STATUS_SHARD_ABORTED is set, and the caller should restore every shard
 * from a snapshot (or reset, which also drops pending pipelined shard frames). No pending frame: OK. */
int tsdf_integrate_shard_abort(tsdf_engine* e);

/* ---- A sharded volume owned by the library (SURVEY.md 8b tsdf_create_sharded; no reference
 * counterpart: TSDFGrid, voxel_tsdf.cu:309-375, is single-GPU). ONE volume spatially sharded over n
 * engines of this process -- shard i on devices[i]; a device may repeat (several shards of one GPU) --
 * running the pipelined sharded frames of tsdf_integrate_shard_pipe with the exchange inside the
 * library: each shard's update kernel writes its carve candidates straight into every shard's inbox
 * (device stores, peer stores over xGMI between GPUs; no copy, no host round trip, no collective
 * library), inboxes double-buffered by call parity. Shards of one device share one stream; across
 * devices each call waits for the previous call of every other device (events). The union of the
 * shards equals the unsharded volume block for block and voxel for voxel; truncation / voxel <= 6.
 * cfg: as tsdf_create (shard_index / shard_count / stream are the group's). Frames: host memory, or
 * device memory on devices[0] (copied to the other devices). tsdf_group_integrate is pipelined like
 * tsdf_integrate; every other group call (flush, stats, query, raycast, shard, synchronize) first
 * completes the pending frames. tsdf_group_query returns the unsharded volume's voxels shard by shard
 * (each shard in entry order); tsdf_group_raycast renders exactly what the unsharded volume renders
 * (render replicas into an engine on devices[0]); tsdf_group_shard gives shard i's engine (e.g. for
 * tsdf_debug_dump); tsdf_group_get_stats sums the shards' counts (each holds, acquires, releases,
 * sees and updates its own blocks: the sums are the unsharded volume's), frames and new keys once.
 * n = 1 is one unsharded engine behind the same calls (tsdf_integrate's pipelined frames). */
typedef struct tsdf_group tsdf_group;
int tsdf_group_create(const tsdf_config* cfg, const int* devices, int n, tsdf_group** out);
int tsdf_group_destroy(tsdf_group* g);
int tsdf_group_size(const tsdf_group* g);
int tsdf_group_integrate(tsdf_group* g, const tsdf_frame* frame, const tsdf_intrinsics* K,
                         const tsdf_pose* cam_T_world, float max_depth);
int tsdf_group_flush(tsdf_group* g);
int tsdf_group_synchronize(tsdf_group* g);
int tsdf_group_shard(tsdf_group* g, int index, tsdf_engine** out);
int tsdf_group_get_stats(tsdf_group* g, tsdf_stats* out, int clear_status);
int tsdf_group_query(tsdf_group* g, const float* bounds, tsdf_voxel* out, int64_t capacity, int64_t* count);
int tsdf_group_raycast(tsdf_group* g, const tsdf_intrinsics* K, int width, int height,
                       const tsdf_pose* cam_T_world, float max_depth, uint8_t* rgba, uint8_t* normal,
                       int mem_kind);
/* Orders `stream` (a hipStream_t of devices[0]) after every shard's queued work: a device frame passed to
 * tsdf_group_integrate is read by the group's own streams after the call returns (its launch, and the
 * peer copies to the other devices), so a caller that reuses or frees the frame's memory on its stream
 * calls this first (the Python Group does, after every device-frame integrate) -- the group's analogue of
 * tsdf_stream_signal. Does not complete pending frames and does not wait on the host. */
int tsdf_group_stream_signal(tsdf_group* g, void* stream);

/* Stream ordering with a caller's HIP stream (e.g. torch's current stream) for device buffers
 * passed to an engine that runs on its own stream: tsdf_stream_wait makes the engine stream wait
 * for the work queued on `stream` so far (before the engine reads a buffer the caller wrote);
 * tsdf_stream_signal makes `stream` wait for the engine's queued work (before the caller reads a
 * buffer the engine wrote, or frees one it reads). tsdf_get_stream returns the engine stream. */
int tsdf_stream_wait(tsdf_engine* e, void* stream);
int tsdf_stream_signal(tsdf_engine* e, void* stream);
int tsdf_get_stream(tsdf_engine* e, void** stream);

/* DISINFSystem::feed_rgbd_frame (disinfect_slam/disinfect_slam.cc:31-67) after the pose lookup:
 * cv::resize(x0.5) of rgb (height x width x 3 u8), depth (height x width u16 raw sensor units) and
 * the optional mask (height x width u8, NULL = none), depth.convertTo(CV_32FC1, 1 / depth_factor),
 * depth = 0 where the resized mask is 0, then TSDFGrid::Integrate of the (width/2 x height/2)
 * frame with ht = lt = ones, all on the GPU. width and height must be even (OpenCV's fast 2x2 area
 * path; see csrc/tsdf_frontend.hip). K is the intrinsics of the half-size image. */
int tsdf_feed_rgbd_frame(tsdf_engine* e, const uint8_t* rgb, const uint16_t* depth,
                         const uint8_t* mask, int width, int height, float depth_factor,
                         const tsdf_intrinsics* K, const tsdf_pose* cam_T_world, float max_depth,
                         int mem_kind);
/* The preprocessing step alone: rgb_out (height/2 x width/2 x 3 u8), depth_out (f32), in host or
 * device memory like the inputs (mem_kind). */
int tsdf_rgbd_half(tsdf_engine* e, const uint8_t* rgb, const uint16_t* depth, const uint8_t* mask,
                   int width, int height, float depth_factor, uint8_t* rgb_out, float* depth_out,
                   int mem_kind);

/* Graph-captured frame loop (BASELINE config C5): TSDFGrid::Integrate (+ optionally RayCast of a
 * render camera into device buffers) as ONE hipGraph launch per frame, with the same results as
 * tsdf_integrate + tsdf_raycast(TSDF_MEM_DEVICE). A graph is bound to one engine, one frame size and
 * one render size (0 x 0 = no raycast). tsdf_graph_frame takes device frames (TSDF_MEM_DEVICE) that
 * must stay valid until the frame has run (tsdf_synchronize); rgba / normal are device buffers of
 * render_height x render_width x 4 u8 (either may be NULL). Asynchronous; profiling events are
 * not recorded for graph frames. */
int tsdf_graph_create(tsdf_engine* e, int width, int height, int render_width, int render_height,
                      tsdf_graph** out);
/* A render-deferring graph (the C5 loop's form of tsdf_raycast_deferred): each frame's raycast is
 * rendered by the graph's NEXT launch, in one kernel with that frame's ingest (k_render_ingest_g), or
 * by the engine's next other call (tsdf_flush, tsdf_synchronize, a query, ...), which launches it
 * alone first. So frame i's rgba / normal are complete once tsdf_graph_frame(i + 1) -- or any other
 * call -- has run, in engine-stream order, and must stay valid until then. Images, volume and
 * statistics are identical to tsdf_graph_create's. Views too deep for a view grid render right after
 * their frame's graph launch. */
int tsdf_graph_create_deferred(tsdf_engine* e, int width, int height, int render_width, int render_height,
                               tsdf_graph** out);
/* A batched graph: each hipGraphLaunch runs frames_per_launch (<= 32) consecutive frames -- their
 * arguments uploaded by one node, their nodes back to back -- so the launch's fixed cost (on this ROCm
 * ~13.5 us of idle GPU between launches) is paid once per batch. tsdf_graph_frame writes a
 * frame into the current batch and launches the batch when it is full; the engine's next other call
 * (tsdf_flush, tsdf_synchronize, a query, another graph's frame, ...) launches a partly filled batch
 * first (its frames one by one). So a frame's outputs (its volume update, rgba / normal) are written
 * once its batch has launched, in engine-stream order; everything else as tsdf_graph_create (deferred
 * != 0: tsdf_graph_create_deferred), results identical. */
int tsdf_graph_create_batch(tsdf_engine* e, int width, int height, int render_width, int render_height,
                            int deferred, int frames_per_launch, tsdf_graph** out);
int tsdf_graph_frame(tsdf_graph* g, const tsdf_frame* frame, const tsdf_intrinsics* K,
                     const tsdf_pose* cam_T_world, float max_depth, const tsdf_intrinsics* render_K,
                     const tsdf_pose* render_cam_T_world, uint8_t* rgba, uint8_t* normal);
int tsdf_graph_destroy(tsdf_graph* g);
/* A shard's graph frames (BASELINE config C5 on a sharded volume): the sharded frame of
 * tsdf_integrate_shard_* as three captured segments around the caller's two exchanges --
 *   tsdf_graph_shard_begin: the DDA of slice slice_index of slice_count (keys into keys_out; with
 *     slice_count 1 every shard runs the whole DDA and keys_out / keys_in are unused);
 *   (the caller all-gathers the key slots into keys_in) tsdf_graph_shard_update: merge, allocate,
 *     update this shard's blocks (raw frame), carve candidates into cands_out;
 *   (the caller all-gathers the candidate slots into cands_in) tsdf_graph_shard_end: the deletes.
 * Every buffer is named at _begin (device memory, valid until _end has run). The exchanges are not
 * recorded into the engine's graphs: stream-ordered collectives of another library (RCCL through
 * torch.distributed) cannot be captured into a graph this library owns. Same results as
 * tsdf_integrate_shard_*. */
int tsdf_graph_create_shard(tsdf_engine* e, int width, int height, int slice_index, int slice_count,
                            tsdf_graph** out);
int tsdf_graph_shard_begin(tsdf_graph* g, const tsdf_frame* frame, const tsdf_intrinsics* K,
                           const tsdf_pose* cam_T_world, float max_depth, void* keys_out,
                           const void* keys_in, int32_t key_cap, void* cands_out, const void* cands_in,
                           int32_t cand_cap);
int tsdf_graph_shard_update(tsdf_graph* g);
int tsdf_graph_shard_end(tsdf_graph* g);

/* TSDFGrid::RayCast (voxel_tsdf.cu:490-506; ray_cast_kernel :232-307). rgba / normal are
 * height x width x 4 u8 (either may be NULL), host or device memory per mem_kind. */
int tsdf_raycast(tsdf_engine* e, const tsdf_intrinsics* K, int width, int height,
                 const tsdf_pose* cam_T_world, float max_depth, uint8_t* rgba, uint8_t* normal,
                 int mem_kind);
/* tsdf_raycast into device buffers with its k_raycast launch deferred to the engine's next call: when
 * that call is tsdf_integrate, the raycast runs in ONE launch with the new frame's ingest (pixel
 * records, DDA, visibility sweep, allocation -- which write nothing the raycast reads), filling the
 * slots the latency-bound raycast leaves; any other call (tsdf_flush, tsdf_synchronize, a query, ...)
 * launches it alone first. The images are those of the volume at this call (bit-identical to
 * tsdf_raycast); they are written in engine-stream order by that next call, so a consumer orders
 * after it (or calls tsdf_flush). rgba / normal must stay valid until then. Views too deep for a view
 * grid take tsdf_raycast's immediate path. (The C5 loop: examples/tsdf/online.cc:60 +
 * modules/renderer_module.cc:105 integrate then render every frame.) */
int tsdf_raycast_deferred(tsdf_engine* e, const tsdf_intrinsics* K, int width, int height,
                          const tsdf_pose* cam_T_world, float max_depth, uint8_t* rgba, uint8_t* normal);

/* TSDFGrid::GatherVoxels (bounds = {xmin, xmax, ymin, ymax, zmin, zmax}, voxel_tsdf.cu:427-454)
 * or GatherValid (bounds == NULL, :399-425). Two-call pattern: *count receives the number of
 * voxels (blocks x 512, entry order then OffsetToIndex); out (host) is filled when non-NULL and
 * capacity >= *count, else TSDF_ERR_CAPACITY. */
int tsdf_query(tsdf_engine* e, const float* bounds, tsdf_voxel* out, int64_t capacity,
               int64_t* count);

/* Render replicas of a spatially sharded volume (the raycast composite SURVEY.md 8e
 * names). The blocks a raycast of (K, W, H, pose, max_depth) can read -- a conservative superset --
 * are packed as TSDF_BLOCK_RECORD_BYTES records {int16 x, y, z, 0; 8 zero bytes; the 6 KiB block:
 * tsdf f32[512], prob f32[512], rgbw u8x4[512]} in entry order. Two-call: out == NULL returns
 * *count only; then out must hold capacity >= *count records (host or device memory per mem_kind).
 * tsdf_import_blocks allocates every record's block in the engine (resolver launches until none is
 * missing) and writes its payload; replace != 0 first empties the volume (table, occupancy, free
 * stack, counters; free pool blocks keep stale contents, which nothing reads), so the engine then
 * holds exactly the records' blocks. A scratch engine that imported every shard's records renders
 * with tsdf_raycast exactly what the unsharded volume renders (ray_cast_kernel,
 * voxel_tsdf.cu:232-307). tsdf_reset empties an engine to its state as created (pool included).
 * No reference counterpart: TSDFGrid is single-GPU. */
#define TSDF_BLOCK_RECORD_BYTES 6160
int tsdf_render_blocks(tsdf_engine* e, const tsdf_intrinsics* K, int width, int height,
                       const tsdf_pose* cam_T_world, float max_depth, void* out, int64_t capacity,
                       int64_t* count, int mem_kind);
int tsdf_import_blocks(tsdf_engine* e, const void* records, int64_t n, int mem_kind,
                       int replace);
int tsdf_reset(tsdf_engine* e);
/* The same records for the Query block selection (bounds as tsdf_query, NULL = every live block):
 * a replica that imports every shard's records with bounds NULL is the whole unsharded volume, so
 * its tsdf_extract_mesh equals the unsharded mesh (as a set of triangles). */
int tsdf_pack_blocks(tsdf_engine* e, const float* bounds, void* out, int64_t capacity,
                     int64_t* count, int mem_kind);

/* Sharded extraction that divides the work (no reference counterpart):
 * - tsdf_raycast_rows: rows [row0, row0 + nrows) of the W x H raycast of tsdf_raycast, bit for bit the
 *   same pixels, into rgba / normal of nrows x width x 4 u8 (ray_cast_kernel, voxel_tsdf.cu:232-307).
 * - tsdf_render_bands: the shard's own blocks a raycast of rows [rows[b], rows[b + 1]) can read, for
 *   each band b < nbands (<= 64): the records of tsdf_render_blocks, grouped band by band, counts[b]
 *   per band (a block may be in several bands). Two-call: out == NULL returns the counts. Each rank of
 *   a sharded render sends band b's records to the rank that renders band b (an all-to-all), imports
 *   what it receives into a replica and renders its band with tsdf_raycast_rows.
 * - tsdf_pack_halo: a shard's own blocks that another shard's marching cubes read -- the blocks with a
 *   neighbour (of 26) owned by shard d go to group d (counts[shard_count]); the caller routes group d
 *   to shard d. A replica holding a shard's own blocks (tsdf_pack_blocks) plus the halo it received
 *   meshes that shard's part of the volume with tsdf_extract_mesh_owned.
 * - tsdf_extract_mesh_owned: tsdf_extract_mesh of the blocks whose brick owner
 *   (tsdf_block_owner(., shard_count)) is shard_index; the other selected blocks are read as
 *   neighbours only. The shards' parts together are the volume's mesh (as a set of triangles). */
int tsdf_raycast_rows(tsdf_engine* e, const tsdf_intrinsics* K, int width, int height,
                      const tsdf_pose* cam_T_world, float max_depth, int row0, int nrows, uint8_t* rgba,
                      uint8_t* normal, int mem_kind);
int tsdf_render_bands(tsdf_engine* e, const tsdf_intrinsics* K, int width, int height,
                      const tsdf_pose* cam_T_world, float max_depth, int nbands, const int32_t* rows,
                      void* out, int64_t capacity, int64_t* counts, int mem_kind);
int tsdf_pack_halo(tsdf_engine* e, void* out, int64_t capacity, int64_t* counts, int mem_kind);
int tsdf_extract_mesh_owned(tsdf_engine* e, const float* bounds, float missing_tsdf, int min_weight,
                            int shard_index, int shard_count, float* triangles, int64_t capacity,
                            int64_t* num_triangles, int mem_kind);

/* Marching-cubes mesh of the volume (GPU; replaces Query + KrisLibrary
 * SparseTSDFReconstruction::ExtractMesh in examples/ros_camera_driver/ros_offline.cc:258-318).
 * bounds as tsdf_query (NULL = every allocated block). Samples sit at voxel centres + half a
 * voxel (ros_offline.cc:281-283); a voxel of a selected block contributes its tsdf when its
 * weight >= min_weight (0 = every voxel, like the reference), every other grid point reads
 * missing_tsdf (KrisLibrary defaultValue = truncation distance; 0.99 ~ the reference's auto
 * value). Output: triangles[9 * i .. 9 * i + 8] = three xyz vertices, normals (right-hand
 * rule) toward increasing tsdf; deterministic order (blocks in hash-entry order). Two-call:
 * triangles == NULL returns the count only. mem_kind: where `triangles` lives. A device
 * `triangles` buffer may be passed in ONE call: *num_triangles is always set, and when it
 * exceeds capacity nothing is written and TSDF_ERR_CAPACITY is returned. */
int tsdf_extract_mesh(tsdf_engine* e, const float* bounds, float missing_tsdf, int min_weight,
                      float* triangles, int64_t capacity, int64_t* num_triangles, int mem_kind);

int tsdf_get_stats(tsdf_engine* e, tsdf_stats* out, int clear_status);
int tsdf_synchronize(tsdf_engine* e);
/* mode TSDF_PROFILE_PHASES: HIP events between all four phases of an integrate call;
 * TSDF_PROFILE_INTEGRATE: only the two events bracketing the fused update kernel (the other
 * phase times read 0). Events are recorded on every `every`-th integrate call (1 = all): each
 * event is a queue marker that costs the stream ~3 us, so a timed loop samples. */
#define TSDF_PROFILE_PHASES 0
#define TSDF_PROFILE_INTEGRATE 1
/* TSDF_PROFILE_KERNEL: ms_integrate from two events bound to the k_integrate dispatch itself
 * (hipExtLaunchKernel start/stop events = the kernel's begin/end timestamps, as a kernel trace
 * reports them); adds nothing to the stream, so `every` = 1 times every launch. */
#define TSDF_PROFILE_KERNEL 2
int tsdf_profile_begin(tsdf_engine* e, int mode, int every);
int tsdf_profile_end(tsdf_engine* e, tsdf_profile* out);

/* Snapshot / restore of the whole volume between frames (checkpoint / resume): hash table,
 * occupancy, free-block stack, voxel pool and counters, so a restored engine continues a frame
 * stream bit for bit. Two-call: tsdf_snapshot_bytes, then tsdf_snapshot_save into a host buffer of
 * that size. tsdf_snapshot_load accepts only a snapshot of an engine with the same voxel size,
 * truncation, pool size and shard layout whose counters, free stack and entries are consistent
 * (every pool index in range, each block exactly once on the stack or in the table);
 * TSDF_ERR_INVALID_ARG otherwise, the engine unchanged. */
int tsdf_snapshot_bytes(tsdf_engine* e, int64_t* bytes);
int tsdf_snapshot_save(tsdf_engine* e, void* out, int64_t capacity);
int tsdf_snapshot_load(tsdf_engine* e, const void* in, int64_t size);

/* Test-only full state dump (Query exposes only tsdf): the 2^22-entry hash table as
 * (x, y, z, offset) int16 quadruples + pool idx int32, the free-block heap, the free counter and
 * the SoA voxel pools (tsdf f32, prob f32, rgbw u8x4 per voxel, pool-index major). Host buffers;
 * any NULL pointer is skipped. */
int tsdf_debug_dump(tsdf_engine* e, int16_t* entry_pos_off, int32_t* entry_idx, int32_t* heap,
                    int32_t* free_count, float* tsdf, float* prob, uint8_t* rgbw);
/* Diagnostic builds only (make DIAG=1): per-workgroup 100 MHz phase stamps of the last launch of
 * each frame kernel, [8 kernels][4096 workgroups][8 stamps] u64, cleared after the copy. *enabled
 * reports whether the library was built with stamps. out == NULL only queries enabled. */
int tsdf_debug_stamps(tsdf_engine* e, uint64_t* out, int64_t capacity, int* enabled);
int32_t tsdf_num_entries(void);
int32_t tsdf_num_blocks(const tsdf_engine* e);

/* ---- VoxelHashTable / VoxelMemPool level (voxel_hash.cu, voxel_mem.cu), host arrays ---- */
/* One launch of VoxelHashTable::Allocate over keys (xyz int16 triples) + ResetLocks. Keys are
 * linearised in list order. */
int tsdf_hash_allocate(tsdf_engine* e, const int16_t* keys, int n);
/* One launch of VoxelHashTable::Delete over keys in list order + ResetLocks. */
int tsdf_hash_delete(tsdf_engine* e, const int16_t* keys, int n);
/* VoxelHashTable::Retrieve (voxel_hash.cuh:104-161) of voxel points: rgbw, tsdf, prob (defaults
 * 0 / 1 / 0 when missing) and the block meta (x, y, z, offset; idx -1 if missing). */
int tsdf_hash_retrieve(tsdf_engine* e, const int16_t* points, int n, uint8_t* rgbw, float* tsdf,
                       float* prob, int16_t* block_pos_off, int32_t* block_idx);
/* RetrieveMutable + store of rgbw (voxel_hash_test.cu:47-54); *missing = points not found. */
int tsdf_hash_assign(tsdf_engine* e, const int16_t* points, int n, const uint8_t* rgbw,
                     int* missing);
int tsdf_num_active_blocks(tsdf_engine* e, int32_t* out);
/* VoxelMemPool::AquireBlock / ReleaseBlock, n sequential calls (voxel_mem.cu:37-61). */
int tsdf_pool_acquire(tsdf_engine* e, int n, int32_t* idx_out);
int tsdf_pool_release(tsdf_engine* e, const int32_t* idx, int n);
int tsdf_pool_set_weight(tsdf_engine* e, int32_t block, uint8_t weight);
int tsdf_pool_get_weights(tsdf_engine* e, int32_t block, uint8_t* out512);

/* Hash of a block coordinate (voxel_hash.cu:31-35) and the shard owner of a block. */
uint32_t tsdf_hash_block(int16_t x, int16_t y, int16_t z);
int32_t tsdf_block_owner(int16_t x, int16_t y, int16_t z, int32_t shard_count);

const char* tsdf_error_string(int code);
const char* tsdf_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* DISINFECT_TSDF_H */
