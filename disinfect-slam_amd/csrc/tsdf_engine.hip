// tsdf_engine.hip -- host side of the MI355X TSDF engine: buffers, launch sequence and the C ABI
// declared in include/disinfect_tsdf.h. No HIP type crosses the ABI.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <deque>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "disinfect_tsdf.h"
#include "tsdf_kernels.h"
#include "tsdf_resolve.h"

using namespace tsdf;

namespace {

thread_local std::string g_last_error;

void set_error(const char* what, hipError_t e) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  g_last_error = buf;
}
void set_error(const char* what) { g_last_error = what; }

#define HIP_OK(expr)                  \
  do {                                \
    hipError_t _e = (expr);           \
    if (_e != hipSuccess) {           \
      set_error(#expr, _e);           \
      return TSDF_ERR_HIP;            \
    }                                 \
  } while (0)

#define LAUNCH_OK(what)                        \
  do {                                         \
    hipError_t _e = hipGetLastError();         \
    if (_e != hipSuccess) {                    \
      set_error(what, _e);                     \
      return TSDF_ERR_HIP;                     \
    }                                          \
  } while (0)

// ---- host float math: same expressions (and -ffp-contract=off) as tsdf_device.h / the oracle ----
f3 h_cross(f3 a, f3 b) {
  f3 r;
  r.x = a.y * b.z - a.z * b.y;
  r.y = a.z * b.x - a.x * b.z;
  r.z = a.x * b.y - a.y * b.x;
  return r;
}
f3 h_qrot(quatf q, f3 v) {
  const f3 qv = {q.x, q.y, q.z};
  f3 uv = h_cross(qv, v);
  uv.x += uv.x;
  uv.y += uv.y;
  uv.z += uv.z;
  const f3 c = h_cross(qv, uv);
  f3 r;
  r.x = (v.x + q.w * uv.x) + c.x;
  r.y = (v.y + q.w * uv.y) + c.y;
  r.z = (v.z + q.w * uv.z) + c.z;
  return r;
}
int16_t h_f2s(float f) {
  if (f != f) return 0;
  if (f >= 32767.0f) return 32767;
  if (f <= -32768.0f) return -32768;
  return (int16_t)f;
}

template <typename T>
hipError_t dmalloc(T** p, size_t count) {
  return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(count, 1) * sizeof(T));
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Environment knobs: A/B experiments and tests only (the defaults are the measured best; nothing a
// drop-in caller needs to set). Read once by tsdf_create (read_env_knobs); every other file reads
// none. TSDF_ROCTX (roctx ranges) is read on first use by the tracing wrapper.
//   TSDF_PIPELINE=0               unpipelined frames: two launches per frame (k_ingest_dda, k_integrate)
//   TSDF_PIPE_MAX_PIXELS=n        largest frame (pixels) that is pipelined (default 2^19; C4 above it)
//   TSDF_FRAME_ORDER=0..4         k_frame grid order of its parts (PipeArgs.order; default 2)
//   TSDF_FRAME_WG_PER_CU=n        k_frame update workgroups per CU (default kFrameUpdWgsPer2Cu / 2 = 2.5: 640)
//   TSDF_FRAME_UPD_WGS=n          (A/B) k_frame update workgroups in total (overrides the per-CU count)
//   TSDF_FRAME_TILES_PER_WG=n     (A/B) k_frame pixel tiles per tile workgroup (default 1)
//   TSDF_INTEGRATE_WG_PER_CU=n    cap on k_integrate's resident workgroups per CU
//   TSDF_CAND_CAP=n               (tests) smaller carve-candidate list, to exercise its overflow
//   TSDF_MESH_GRID=n              (tests) fewer k_mesh workgroups, to exercise its grid stride
//   TSDF_RENDER_OVERLAP=1         raycast on a second stream overlapping the next frame
//   TSDF_GRAPH_MEMCPY_NODE=1      (A/B) graph frames upload their arguments with a memcpy node
//   TSDF_FUSE_VIEW_GRID=0         (A/B) the C5 loop's view grid in its own launch (render graphs: own node), not in the update's
//   TSDF_UPLOAD_STREAMS=n         (A/B) host frames: upload streams a frame's copies spread over (1-4, default 2)
// ---------------------------------------------------------------------------------------------
struct EnvKnobs {
  bool pipeline = true;
  int64_t pipe_max_pixels = -1;
  int frame_order = -1, frame_wg_per_cu = 0, integrate_wg_per_cu = 0, cand_cap = 0, mesh_grid = 0;
  int frame_tiles_per_wg = 1, frame_upd_wgs = 0;
  bool render_overlap = false, graph_memcpy_node = false;
  int upload_streams = 2;
  bool fuse_view_grid = true;
};
static EnvKnobs read_env_knobs() {
  EnvKnobs k;
  auto num = [](const char* n, long long dflt) {
    const char* v = std::getenv(n);
    return v ? std::atoll(v) : dflt;
  };
  auto flag = [](const char* n, bool dflt) {
    const char* v = std::getenv(n);
    return v ? v[0] == '1' : dflt;
  };
  if (const char* v = std::getenv("TSDF_PIPELINE")) k.pipeline = v[0] != '0';
  k.pipe_max_pixels = num("TSDF_PIPE_MAX_PIXELS", -1);
  k.frame_order = (int)std::max(-1ll, num("TSDF_FRAME_ORDER", -1));
  k.frame_wg_per_cu = (int)num("TSDF_FRAME_WG_PER_CU", 0);
  k.frame_tiles_per_wg = (int)std::max(1ll, num("TSDF_FRAME_TILES_PER_WG", 1));
  k.frame_upd_wgs = (int)num("TSDF_FRAME_UPD_WGS", 0);
  k.integrate_wg_per_cu = (int)num("TSDF_INTEGRATE_WG_PER_CU", 0);
  k.cand_cap = (int)num("TSDF_CAND_CAP", 0);
  k.mesh_grid = (int)num("TSDF_MESH_GRID", 0);
  k.render_overlap = flag("TSDF_RENDER_OVERLAP", false);
  k.graph_memcpy_node = flag("TSDF_GRAPH_MEMCPY_NODE", false);
  k.upload_streams = (int)num("TSDF_UPLOAD_STREAMS", 2);
  k.fuse_view_grid = flag("TSDF_FUSE_VIEW_GRID", true);
  return k;
}

struct tsdf_engine {
  tsdf_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // render stream: k_raycast runs here so that the next frame's ingest (which writes neither the
  // pool nor the view grid) overlaps it; every other call first joins it (join_render)
  hipStream_t rstream = nullptr;
  hipEvent_t rs_ready = nullptr, rs_done = nullptr;
  bool render_pending = false;
  // measured (r3, C5 loop, same box, interleaved): 5.44k frames/s with the overlap against 5.81k
  // without -- the two cross-stream event waits per frame and the ingest's workgroups beside the
  // raycast's cost more than the overlap hides. Off by default; TSDF_RENDER_OVERLAP=1 enables it.
  bool render_overlap = false;
  // a deferred raycast (tsdf_raycast_deferred): its view grid is built; the k_raycast launch waits
  // for the engine's next call -- fused with the next frame's ingest (k_render_ingest) when that call
  // is tsdf_integrate, alone otherwise (join_render)
  struct DeferredRender {
    bool pending = false;
    FrameParams P{};
    ViewGrid V{};
    float step = 0.f;
    uchar4* rgba = nullptr;
    uchar4* normal = nullptr;
  } rd;
  // the deferred raycast of a render-deferring graph frame (tsdf_graph_create_deferred): its args slot
  // (camera, view grid, outputs) on the device; taken up by the graph's next frame (k_render_ingest_g),
  // launched alone (k_raycast_g) by any other call
  struct DeferredGraphRender {
    bool pending = false;
    const tsdf_graph* g = nullptr;
    const FrameArgs* args = nullptr;
    int W = 0, H = 0;
  } rdg;
  // a batched graph (tsdf_graph_create_batch) whose current batch holds frames not launched yet:
  // every other call launches them first (join_render -> graph_flush_batch)
  struct tsdf_graph* gbatch = nullptr;
  EngineDev D{};
  int maxs = 3;
  int64_t order_range = 0;  // candidate order space: max_pixels * maxs
  int64_t max_pixels = 0;
  // host-frame staging
  // host frames (TSDF_MEM_HOST, voxel_tsdf.cu:358-365): two staging slots filled on the upload stream
  // (a copy engine) while the engine stream runs the previous frames; slot k at offset k * max_pixels
  uint8_t* s_rgb = nullptr;
  float* s_depth = nullptr;
  float* s_ht = nullptr;
  float* s_lt = nullptr;
  // upload streams: a frame's copies spread over them (several DMA engines share the host link)
  static constexpr int kUpStreams = 4;
  hipStream_t ustream[kUpStreams] = {};
  hipEvent_t up_done[2][kUpStreams] = {};  // slot k's copies on stream j complete (the engine stream waits)
  int up_nstreams = 0;                     // streams the pending upload used
  hipEvent_t up_free[2] = {nullptr, nullptr};  // slot k's last reader launched before this (the upload waits)
  bool up_used[2] = {false, false};       // up_free[k] has been recorded
  int up_next = 0;                        // the slot of the next host frame
  int up_pending = -1;                    // the slot of a frame whose reading launch is not enqueued yet
  // raycast / query / test scratch
  uchar4* rc_rgba = nullptr;
  uchar4* rc_norm = nullptr;
  // raycast view grid (tsdf_kernels.h ViewGrid): cells, the two brick bitmaps, generation
  uint32_t* vg_cell = nullptr;
  int64_t vg_cap = 0;  // cells
  uint8_t* vg_flags = nullptr;
  uint32_t* vg_bits = nullptr;
  uint32_t vg_gen = 0;
  uint64_t vg_calls = 0;
  VisRec* q_sel = nullptr;
  int32_t* q_count = nullptr;
  float4* q_out = nullptr;
  int64_t q_out_cap = 0;
  // grouped selections (render bands / halo destinations): per group a bitmap, its per-workgroup
  // counts, the emitted list and its count
  unsigned long long* g_visbits = nullptr;
  int32_t* g_wgcnt = nullptr;
  VisRec* g_sel = nullptr;
  int32_t* g_count = nullptr;
  int g_cap = 0;  // groups
  // mesh extraction scratch
  int32_t* m_counts = nullptr;
  int32_t* m_offsets = nullptr;
  int64_t* m_total = nullptr;
  int32_t* m_nbr = nullptr;     // k_mesh: 27 neighbour pool indices per selected block
  int mesh_grid = 0;            // k_mesh workgroups: min(kMeshGrid, pool blocks)
  float* m_out = nullptr;
  int64_t m_out_cap = 0;  // triangles
  int16_t* t_keys = nullptr;
  VisRec* t_recs = nullptr;
  int32_t* t_count = nullptr;
  int32_t* t_i32 = nullptr;
  uint32_t* t_u32 = nullptr;
  float* t_f0 = nullptr;
  float* t_f1 = nullptr;
  short4* t_s4 = nullptr;
  int t_cap = 0;
  DevCounters* h_ctr = nullptr;  // pinned readback
  // profiling
  bool profiling = false;
  int prof_mode = TSDF_PROFILE_PHASES;
  int prof_every = 1;        // event-time every n-th integrate call
  int64_t prof_calls = 0;    // integrate calls since profile_begin
  int64_t prof_pipelined = 0;  // update launches with the next frame's pixel tiles since profile_begin
  // a deque: a deferred frame (pipelined, sharded) keeps a pointer to its events across later calls
  std::deque<std::array<hipEvent_t, 5>> events;
  size_t ev_used = 0;
  unsigned long long prof_vis0 = 0, prof_upd0 = 0, prof_ticks0 = 0, prof_ing0 = 0, prof_ra0 = 0, prof_rd0 = 0;
  // sharded frame (tsdf_integrate_shard_*): 0 idle, 1 after _begin, 2 after _update
  hipEvent_t order_ev = nullptr;  // tsdf_stream_wait / _signal
  int shard_phase = 0;
  bool shard_keys_packed = false;  // _begin wrote a key slot (split DDA): _update merges an inbox
  FrameParams shard_P{};
  std::array<hipEvent_t, 5>* shard_ev = nullptr;
  // pipelined frames (tsdf_integrate on one volume, k_frame): what the next launch
  // continues. kPipeNone: nothing pending. kPipeU: frame p_fid's ingest and allocation ran
  // (k_ingest_dda), its update is pending. kPipeCAU: frame p_carve's carving and frame p_fid's
  // allocation and update are pending (p_fid's tiles probed and inserted its keys, its sweep listed
  // its blocks). Every other entry point first completes them (flush_pending).
  bool pipeline = true;
  int64_t pipe_max_pixels = (int64_t)1 << 19;  // larger frames take two launches (pipe_frame_size)
  static constexpr int kPipeNone = 0, kPipeU = 1, kPipeCAU = 2, kPipeAU = 3, kPipeC = 4;  // kPipeAU:
  // p_fid's allocation and update are pending with no carving (after a graph frame that started a
  // stream); kPipeC: only p_fid's carving is pending (a shard's pipelined frames, between flush steps)
  int ps = kPipeNone;
  uint32_t fid_next = 1;  // engine-wide frame ids (views, tags; never 0)
  uint32_t p_carve = 0, p_fid = 0;
  FrameParams p_P{};      // frame p_fid's camera / frame / pixel-record buffer
  bool p_sampled = false;  // kPipeU: the frame was sampled for profiling (its update, when flushed
                           //   as k_integrate, takes an event pair then)
  uint32_t pipe_tag = 0;  // one per k_frame launch: its flags' value
  int frame_order = 2;    // PipeArgs.order (TSDF_FRAME_ORDER): sweep, update, tiles (measured best)
  EnvKnobs env;           // the environment's A/B and test knobs, read once at tsdf_create
  // feed_rgbd_frame staging: raw full-size inputs (host frames) and the half-size outputs
  uint8_t* fe_rgb = nullptr;
  uint16_t* fe_depth = nullptr;
  uint8_t* fe_mask = nullptr;
  int64_t fe_in_cap = 0;  // pixels
  uint8_t* fe_out_rgb = nullptr;
  float* fe_out_depth = nullptr;
  int64_t fe_out_cap = 0;
};

namespace {

void free_all(tsdf_engine* e) {
  EngineDev& D = e->D;
  void* ptrs[] = {D.pipe,    D.ctag,     D.rtag,     D.fo,
                  D.table,   D.lock_tag, D.heap,     D.pool,    D.occ,
                  D.ctr,     D.nk_key,   D.nk_order, D.nk_list, D.pairs, D.fresh,
                  e->fe_rgb, e->fe_depth, e->fe_mask, e->fe_out_rgb, e->fe_out_depth,
                  D.vis,     D.band,    D.cand,     D.arrive, D.swdirty, D.fresh_vis, D.pend, D.pixA, D.pixC,     D.visbits,    D.wgcnt, D.dbg,
                  e->s_rgb,  e->s_depth, e->s_ht,    e->s_lt,   e->rc_rgba,   e->rc_norm,
                  e->vg_cell, e->vg_flags, e->vg_bits, e->g_visbits, e->g_wgcnt, e->g_sel, e->g_count,
                  e->q_sel,  e->q_count, e->q_out, e->m_counts, e->m_offsets, e->m_total, e->m_nbr, e->m_out,   e->t_keys, e->t_recs,    e->t_count,
                  e->t_i32,  e->t_u32,   e->t_f0,    e->t_f1,   e->t_s4};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (e->h_ctr) (void)hipHostFree(e->h_ctr);
  for (auto& ev : e->events)
    for (hipEvent_t x : ev) (void)hipEventDestroy(x);
  if (e->order_ev) (void)hipEventDestroy(e->order_ev);
  if (e->rstream) (void)hipStreamDestroy(e->rstream);
  for (int j = 0; j < tsdf_engine::kUpStreams; ++j) {
    if (e->ustream[j]) (void)hipStreamDestroy(e->ustream[j]);
    for (int k = 0; k < 2; ++k)
      if (e->up_done[k][j]) (void)hipEventDestroy(e->up_done[k][j]);
  }
  for (int k = 0; k < 2; ++k) {
    if (e->up_free[k]) (void)hipEventDestroy(e->up_free[k]);
  }
  if (e->rs_ready) (void)hipEventDestroy(e->rs_ready);
  if (e->rs_done) (void)hipEventDestroy(e->rs_done);
  if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
}

FrameParams make_params(const tsdf_engine* e, const tsdf_intrinsics* K, int W, int H,
                        const tsdf_pose* p, float max_depth) {
  FrameParams P{};
  P.fx = K->fx;
  P.fy = K->fy;
  P.cx = K->cx;
  P.cy = K->cy;
  P.ifx = 1.0f / K->fx;  // CameraIntrinsics::Inverse (camera.cuh:34-39)
  P.ify = 1.0f / K->fy;
  P.icx = -K->cx * P.ifx;
  P.icy = -K->cy * P.ify;
  P.cq = {p->qx, p->qy, p->qz, p->qw};
  P.ct = {p->tx, p->ty, p->tz};
  // SE3::Inverse on the host (lie_group.cuh:22-24); squaredNorm as a Packet4f reduction
  const float n2 = (p->qx * p->qx + p->qz * p->qz) + (p->qy * p->qy + p->qw * p->qw);
  if (n2 > 0.0f)
    P.wq = {-p->qx / n2, -p->qy / n2, -p->qz / n2, p->qw / n2};
  else
    P.wq = {0.f, 0.f, 0.f, 0.f};
  const f3 nt = {-p->tx, -p->ty, -p->tz};
  P.wt = h_qrot(P.wq, nt);
  P.voxel = e->cfg.voxel_size;
  P.trunc = e->cfg.truncation;
  P.inv_trunc = 1.0f / e->cfg.truncation;
  P.inv_voxel = 1.0f / e->cfg.voxel_size;
  P.inv_max_depth = 1.0f / max_depth;
  P.max_depth = max_depth;
  P.W = W;
  P.H = H;
  P.maxs = e->maxs;
  P.shard_index = e->cfg.shard_index;
  P.shard_count = e->cfg.shard_count;
  P.tile_lo = 0;
  P.tile_hi = 1 << 30;
  P.tail = kTailResolve;
  P.slot_cap = 0;
  P.slot = nullptr;
  P.pack_pixels = 1;
  P.row0 = 0;
  P.nrows = H;
  P.depth = nullptr;
  P.rgb = nullptr;
  P.ht = nullptr;
  P.lt = nullptr;
  P.pix_off = 0;  // pixel-record buffer 0 (a pipelined frame may take buffer 1)
  return P;
}

int ensure_test_cap(tsdf_engine* e, int n) {
  if (n <= e->t_cap) return TSDF_OK;
  (void)hipFree(e->t_keys);
  (void)hipFree(e->t_recs);
  (void)hipFree(e->t_i32);
  (void)hipFree(e->t_u32);
  (void)hipFree(e->t_f0);
  (void)hipFree(e->t_f1);
  (void)hipFree(e->t_s4);
  // nothing dangles if an allocation below fails: tsdf_destroy frees what was allocated
  e->t_keys = nullptr;
  e->t_recs = nullptr;
  e->t_i32 = nullptr;
  e->t_u32 = nullptr;
  e->t_f0 = nullptr;
  e->t_f1 = nullptr;
  e->t_s4 = nullptr;
  e->t_cap = 0;
  const int cap = std::max(n, 1024);
  HIP_OK(dmalloc(&e->t_keys, (size_t)cap * 3));
  HIP_OK(dmalloc(&e->t_recs, (size_t)cap));
  HIP_OK(dmalloc(&e->t_i32, (size_t)cap));
  HIP_OK(dmalloc(&e->t_u32, (size_t)cap));
  HIP_OK(dmalloc(&e->t_f0, (size_t)cap));
  HIP_OK(dmalloc(&e->t_f1, (size_t)cap));
  HIP_OK(dmalloc(&e->t_s4, (size_t)cap));
  e->t_cap = cap;
  return TSDF_OK;
}

// the allocation resolver as its own launch: hash-level test path and imports (frame_mode 0)
int launch_resolve_alloc(tsdf_engine* e, const FrameParams& P, uint32_t range, int frame_mode) {
  hipLaunchKernelGGL(k_resolve_alloc, dim3(1), dim3(kRT), 0, e->stream, e->D, P, range, frame_mode,
                     (const ShardRec*)nullptr, 0, 0);
  if (!frame_mode)
    hipLaunchKernelGGL(k_fresh_init, dim3(512), dim3(256), 0, e->stream, e->D);
  LAUNCH_OK("allocate");
  return TSDF_OK;
}

// the engine stream waits for a raycast still running on the render stream
// (keep_deferred: a deferred raycast stays pending -- tsdf_stream_wait orders the engine stream after
// another stream's work, which the raycast may follow as well; wait_overlap false: launch the deferred
// raycasts only, without joining a TSDF_RENDER_OVERLAP raycast on the render stream -- the next
// frame's ingest writes nothing it reads; keep_graph: the graph frame that renders rdg itself calls)
int graph_flush_batch(tsdf_graph* g);
int join_render(tsdf_engine* e, bool keep_deferred = false, bool wait_overlap = true, bool keep_graph = false) {
  if (e->gbatch) {  // the frames of a batched graph not launched yet, before anything else
    int rc = graph_flush_batch(e->gbatch);
    if (rc) return rc;
  }
  if (e->rdg.pending && !keep_deferred && !keep_graph) {  // (a graph frame's deferred raycast: its args slot)
    e->rdg.pending = false;
    const dim3 rgrid((e->rdg.W + 15) / 16, (e->rdg.H + 15) / 16);
    hipLaunchKernelGGL(k_raycast_g, rgrid, dim3(256), 0, e->stream, e->D, e->rdg.args);
    HIP_OK(hipGetLastError());
  }
  if (e->rd.pending && !keep_deferred) {  // a deferred raycast no ingest took up: launched alone, before anything else
    e->rd.pending = false;
    const tsdf_engine::DeferredRender& r = e->rd;
    const dim3 rgrid((r.P.W + 15) / 16, (r.P.nrows + 15) / 16);
    hipLaunchKernelGGL(k_raycast, rgrid, dim3(256), (size_t)r.V.nw * 4, e->stream, e->D, r.P, r.step, r.V, r.rgba,
                       r.normal);
    HIP_OK(hipGetLastError());
  }
  if (!e->render_pending || !wait_overlap) return TSDF_OK;
  e->render_pending = false;
  HIP_OK(hipStreamWaitEvent(e->stream, e->rs_done, 0));
  return TSDF_OK;
}
#define JOIN_RENDER(e)              \
  do {                              \
    int _rc = join_render(e);       \
    if (_rc) return _rc;            \
  } while (0)

int flush_pending(tsdf_engine* e);
// every entry point that reads or writes the volume (or orders against it) first enqueues a deferred
// update (pipelined frames) and joins the render stream
#define ENTER(e)                       \
  do {                                 \
    int _rc = join_render(e);          \
    if (_rc) return _rc;               \
    _rc = flush_pending(e);            \
    if (_rc) return _rc;               \
  } while (0)

int read_counters(tsdf_engine* e) {
  ENTER(e);
  HIP_OK(hipMemcpyAsync(e->h_ctr, e->D.ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

}  // namespace

// roctx ranges around the C-ABI calls (SURVEY.md 5 tracing): host-side enqueue intervals that
// `rocprofv3 --marker-trace` lines up with the kernels they launch. Off unless TSDF_ROCTX=1.
namespace {
bool roctx_on() {
  static const bool on = [] {
    const char* v = std::getenv("TSDF_ROCTX");
    return v && v[0] == '1';
  }();
  return on;
}
struct TraceRange {
  const bool on;
  explicit TraceRange(const char* name) : on(roctx_on()) {
    if (on) roctxRangePushA(name);
  }
  ~TraceRange() {
    if (on) roctxRangePop();
  }
};
}  // namespace

extern "C" {

void tsdf_config_default(tsdf_config* c) {
  if (!c) return;
  c->voxel_size = 0.005f;
  c->truncation = 0.03f;
  c->max_width = 1920;
  c->max_height = 1080;
  c->num_block_bits = 18;
  c->shard_index = 0;
  c->shard_count = 1;
  c->stream = nullptr;
  c->use_stream = 0;
}

const char* tsdf_error_string(int code) {
  switch (code) {
    case TSDF_OK: return "ok";
    case TSDF_ERR_INVALID_ARG: return "invalid argument";
    case TSDF_ERR_OUT_OF_MEMORY: return "out of device memory";
    case TSDF_ERR_HIP: return "HIP runtime error";
    case TSDF_ERR_CAPACITY: return "output buffer too small";
    case TSDF_ERR_NO_DEVICE: return "no HIP device";
    case TSDF_ERR_PIPELINE: return "pipelined frame wait timed out";
    default: return "unknown error";
  }
}
const char* tsdf_last_error(void) { return g_last_error.c_str(); }
void tsdf_set_last_error(const char* what) { g_last_error = what ? what : ""; }

uint32_t tsdf_hash_block(int16_t x, int16_t y, int16_t z) { return hash_block(x, y, z); }
int32_t tsdf_block_owner(int16_t x, int16_t y, int16_t z, int32_t n) {
  return (int32_t)brick_owner(x, y, z, (uint32_t)(n < 1 ? 1 : n));
}
int32_t tsdf_num_entries(void) { return (int32_t)kNumEntry; }
int32_t tsdf_num_blocks(const tsdf_engine* e) { return e ? e->D.nblocks : 0; }

namespace {
// empty volume: table, occupancy, free stack, voxel pool, counters and key sets (tsdf_create,
// tsdf_reset); with_pool false leaves the voxel pool as it is (tsdf_import_blocks replace: every
// block that becomes live is written by the import, free blocks are never read)
bool init_state(tsdf_engine* e, bool with_pool = true) {
  hipStream_t s = e->stream;
  const EngineDev& D = e->D;
  const int nb = D.nblocks;
  bool ok = true;
  ok &= hipMemsetAsync(D.lock_tag, 0, sizeof(uint32_t) * kNumBucket, s) == hipSuccess;
  if (with_pool) ok &= hipMemsetAsync(D.pool, 0, (size_t)nb * kBlockBytes, s) == hipSuccess;
  ok &= hipMemsetAsync(D.occ, 0, sizeof(unsigned long long) * kOccWords, s) == hipSuccess;
  ok &= hipMemsetAsync(D.nk_key, 0, sizeof(unsigned long long) * kNewKeyCap, s) == hipSuccess;
  ok &= hipMemsetAsync(D.nk_order, 0xFF, sizeof(uint32_t) * kNewKeyCap, s) == hipSuccess;
  ok &= hipMemsetAsync(D.band, 0, sizeof(int32_t) * 3 * kBands * kBandStride, s) == hipSuccess;
  ok &= hipMemsetAsync(D.pipe, 0, sizeof(unsigned long long) * kPipeWords, s) == hipSuccess;
  ok &= hipMemsetAsync(D.ctag, 0, sizeof(uint32_t) * 2 * (size_t)nb, s) == hipSuccess;
  ok &= hipMemsetAsync(D.rtag, 0, sizeof(uint32_t) * (size_t)nb, s) == hipSuccess;
  ok &= hipMemsetAsync(D.fo, 0xFF, sizeof(unsigned long long) * (size_t)kNumEntry, s) == hipSuccess;
  ok &= hipMemsetAsync(D.visbits, 0, sizeof(unsigned long long) * kOccWords, s) == hipSuccess;
  ok &= hipMemsetAsync(D.arrive, 0, sizeof(unsigned long long) * kArriveWords, s) == hipSuccess;
  ok &= hipMemsetAsync(D.swdirty, 0, sizeof(unsigned long long) * (kOccWords / 64), s) == hipSuccess;
  DevCounters c0{};
  c0.free_count = nb;
  ok &= hipMemcpyAsync(D.ctr, &c0, sizeof(c0), hipMemcpyHostToDevice, s) == hipSuccess;
  hipLaunchKernelGGL(k_init_table, dim3(kNumEntry / 256), dim3(256), 0, s, D.table);
  hipLaunchKernelGGL(k_init_heap, dim3((nb + 255) / 256), dim3(256), 0, s, D.heap, nb);
  if (with_pool)
    hipLaunchKernelGGL(k_init_prob, dim3((unsigned)(((size_t)nb * (kBlockVolume / 4) + 255) / 256)),
                       dim3(256), 0, s, D.pool, nb);
  ok &= hipGetLastError() == hipSuccess;
  ok &= hipStreamSynchronize(s) == hipSuccess;
  return ok;
}

}  // namespace

int tsdf_create(const tsdf_config* cfg_in, int device, tsdf_engine** out) {
  if (!out) return TSDF_ERR_INVALID_ARG;
  *out = nullptr;
  tsdf_config cfg;
  if (cfg_in)
    cfg = *cfg_in;
  else
    tsdf_config_default(&cfg);
  if (!(cfg.voxel_size > 0) || !(cfg.truncation > 0) || cfg.max_width <= 0 ||
      cfg.max_height <= 0 || cfg.num_block_bits < 1 || cfg.num_block_bits > 22 ||
      cfg.shard_count < 1 || cfg.shard_count > kMaxShards || cfg.shard_index < 0 ||
      cfg.shard_index >= cfg.shard_count) {
    set_error("tsdf_create: invalid config");
    return TSDF_ERR_INVALID_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
    set_error("tsdf_create: no such HIP device");
    return TSDF_ERR_NO_DEVICE;
  }
  HIP_OK(hipSetDevice(device));
  tsdf_engine* e = new tsdf_engine();
  e->cfg = cfg;
  e->env = read_env_knobs();
  e->device = device;
  // DDA samples per pixel: step_grid = ceil(max|2 trunc dir / voxel| / 8) + 1 (voxel_tsdf.cu:136)
  e->maxs = (int)std::ceil(2.0 * cfg.truncation / cfg.voxel_size * 1.0001 / kBlockLen) + 1;
  e->max_pixels = (int64_t)cfg.max_width * cfg.max_height;
  e->order_range = e->max_pixels * e->maxs;
  if (e->maxs > kMaxDdaSamples || e->order_range > kMaxOrderRange) {
    delete e;
    set_error("tsdf_create: truncation / voxel ratio or image size beyond the supported "
              "candidate order space (maxs <= 6, width*height*maxs <= 8M)");
    return TSDF_ERR_INVALID_ARG;
  }
  const int nb = 1 << cfg.num_block_bits;
  EngineDev& D = e->D;
  D.nblocks = nb;
  auto fail = [&](int code) {
    free_all(e);
    delete e;
    return code;
  };
#define ALLOC(ptr, n)                                 \
  do {                                                \
    hipError_t _e = dmalloc(&(ptr), (size_t)(n));     \
    if (_e != hipSuccess) {                           \
      set_error("tsdf_create: hipMalloc " #ptr, _e);  \
      return fail(TSDF_ERR_OUT_OF_MEMORY);            \
    }                                                 \
  } while (0)
  ALLOC(D.table, kNumEntry);
  ALLOC(D.lock_tag, kNumBucket);
  ALLOC(D.heap, nb);
  ALLOC(D.pool, (size_t)nb * kBlockBytes);
  ALLOC(D.occ, kOccWords);
  ALLOC(D.ctr, 1);
  ALLOC(D.nk_key, kNewKeyCap);
  ALLOC(D.nk_order, kNewKeyCap);
  ALLOC(D.nk_list, kNewKeyCap);
  ALLOC(D.pairs, std::max<size_t>(kNewKeyCap, (size_t)nb));
  ALLOC(D.fresh, kNewKeyCap);
  // two frames' visible lists, three frames' band counts (pipelined frames: frame_view)
  ALLOC(D.vis, (size_t)2 * kBands * nb);
  ALLOC(D.band, 3 * kBands * kBandStride);
  ALLOC(D.pipe, kPipeWords);
  ALLOC(D.ctag, (size_t)2 * nb);
  ALLOC(D.rtag, nb);
  ALLOC(D.fo, kNumEntry);
  // carve candidates of one frame: a shard's list takes every shard's (their visible blocks and the
  // entries exhausted pools left without voxels), so it is sized like the resolver's D.pairs scratch;
  // more are clamped with TSDF_STATUS_SHARD_OVERFLOW. TSDF_CAND_CAP (tests) sets a smaller list.
  D.cand_cap = (int32_t)std::max<size_t>(kNewKeyCap, (size_t)nb);
  if (e->env.cand_cap > 0) D.cand_cap = std::min(D.cand_cap, std::max(1024, e->env.cand_cap));
  ALLOC(D.cand, (size_t)2 * D.cand_cap);  // two frames' lists (frame_view)
  ALLOC(D.arrive, kArriveWords);
  ALLOC(D.swdirty, kOccWords / 64);
  ALLOC(D.fresh_vis, kNewKeyCap);
  ALLOC(D.pend, kNewKeyCap);
  {  // one resident wave of k_integrate workgroups: no second-round stragglers
    int per_cu = 0, ncu = 0;
    // (a shard's raw-frame variant is sized by its own occupancy)
    const void* kfn = cfg.shard_count > 1 ? reinterpret_cast<const void*>(k_integrate_t<false, true>)
                                          : reinterpret_cast<const void*>(k_integrate_t<false, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kIntegrateThreads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
      return fail(TSDF_ERR_HIP);
    if (e->env.integrate_wg_per_cu > 0) per_cu = std::min(per_cu, e->env.integrate_wg_per_cu);
    D.integrate_grid = std::max(8, std::min(kIntegrateGrid, (per_cu * ncu) & ~7));
    int per_cu_pre = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_pre, reinterpret_cast<const void*>(k_frame),
                                                     kIntegrateThreads, 0) != hipSuccess)
      return fail(TSDF_ERR_HIP);
    // 2.5 update workgroups per CU by default (of 6 that fit): the other slots take the sweep's and
    // the tiles' workgroups from the start. Round 6, final build (exact semantic chain, 6 waves per
    // SIMD, no packed fp32): 640 update workgroups 20.94-20.99k frames/s on the driver command, 704
    // 20.8-21.0k, 768 20.6k, 896 20.2k (profiles/ab/r6_upd_wgs_nopk_ab.txt); with packed fp32 768 was
    // ahead (19.6k vs 18.7-19.4k at 640). Round 5 (log-odds state, 7 waves): 640 23.9k, 768
    // 23.3-23.5k, 512 23.4-23.7k; earlier rounds: 4 per CU 22.0-22.5k, 5 21.0-21.3k, 7 18.5-18.7k
    int upd = kFrameUpdWgsPer2Cu * ncu / 2;
    if (e->env.frame_wg_per_cu > 0) upd = e->env.frame_wg_per_cu * ncu;
    if (e->env.frame_upd_wgs > 0) upd = e->env.frame_upd_wgs;
    D.integrate_grid_pre = std::max(8, std::min({kIntegrateGrid, upd, per_cu_pre * ncu}) & ~7);
  }
  ALLOC(D.pixA, 2 * e->max_pixels);  // two buffers: a pipelined frame's and the next one's
  ALLOC(D.pixC, 2 * e->max_pixels);
  e->pipeline = e->env.pipeline;
  if (e->env.pipe_max_pixels >= 0) e->pipe_max_pixels = e->env.pipe_max_pixels;
  if (e->env.frame_order >= 0) e->frame_order = std::min(4, e->env.frame_order);
  ALLOC(D.visbits, kOccWords);
  ALLOC(D.wgcnt, kOccWords / 256);
  ALLOC(D.dbg, (size_t)kDiagKernels * kDiagMaxWg * kDiagStamps);
  if (hipMemset(D.dbg, 0, (size_t)kDiagKernels * kDiagMaxWg * kDiagStamps * 8) != hipSuccess)
    return fail(TSDF_ERR_HIP);
  ALLOC(e->s_rgb, 2 * e->max_pixels * 3);  // two upload slots (host frames)
  ALLOC(e->s_depth, 2 * e->max_pixels);
  ALLOC(e->s_ht, 2 * e->max_pixels);
  ALLOC(e->s_lt, 2 * e->max_pixels);
  ALLOC(e->rc_rgba, e->max_pixels);
  ALLOC(e->rc_norm, e->max_pixels);
  ALLOC(e->vg_flags, (size_t)kViewBitmapWords * 32);
  ALLOC(e->vg_bits, kViewBitmapWords);
  if (hipMemset(e->vg_flags, 0, (size_t)kViewBitmapWords * 32) != hipSuccess)
    return fail(TSDF_ERR_HIP);
  ALLOC(e->q_sel, nb);
  ALLOC(e->q_count, 1);
  ALLOC(e->m_counts, nb);
  ALLOC(e->m_offsets, nb);
  ALLOC(e->m_total, 1);
  ALLOC(e->m_nbr, (size_t)27 * nb);
  e->mesh_grid = std::min(kMeshGrid, nb);
  if (e->env.mesh_grid > 0) e->mesh_grid = std::min(e->mesh_grid, e->env.mesh_grid);
  ALLOC(e->t_count, 1);
#undef ALLOC
  D = frame_view(D, 0u);  // the base view (sharded / graph / hash-level paths): frame parity 0
  if (hipHostMalloc(reinterpret_cast<void**>(&e->h_ctr), sizeof(DevCounters)) != hipSuccess)
    return fail(TSDF_ERR_OUT_OF_MEMORY);
  if (cfg.use_stream) {  // the caller's stream; NULL is the legacy default stream (torch's default)
    e->stream = reinterpret_cast<hipStream_t>(cfg.stream);
  } else {
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
      return fail(TSDF_ERR_HIP);
    e->own_stream = true;
  }
  for (int j = 0; j < tsdf_engine::kUpStreams; ++j) {
    if (hipStreamCreateWithFlags(&e->ustream[j], hipStreamNonBlocking) != hipSuccess)
      return fail(TSDF_ERR_HIP);
    for (int k = 0; k < 2; ++k)
      if (hipEventCreateWithFlags(&e->up_done[k][j], hipEventDisableTiming) != hipSuccess)
        return fail(TSDF_ERR_HIP);
  }
  for (int k = 0; k < 2; ++k)
    if (
        hipEventCreateWithFlags(&e->up_free[k], hipEventDisableTiming) != hipSuccess)
      return fail(TSDF_ERR_HIP);
  if (hipStreamCreateWithFlags(&e->rstream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->rs_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->rs_done, hipEventDisableTiming) != hipSuccess)
    return fail(TSDF_ERR_HIP);
  e->render_overlap = e->env.render_overlap;
  if (!init_state(e)) {
    set_error("tsdf_create: initialisation failed");
    return fail(TSDF_ERR_HIP);
  }
  *out = e;
  return TSDF_OK;
}

int tsdf_destroy(tsdf_engine* e) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  (void)hipSetDevice(e->device);
  (void)join_render(e);  // (a deferred raycast's outputs are still written)
  if (e->rstream) (void)hipStreamSynchronize(e->rstream);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  free_all(e);
  delete e;
  return TSDF_OK;
}

int tsdf_synchronize(tsdf_engine* e) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  // a pipelined frame whose in-kernel wait timed out has wrong results: an error here, not only a
  // status bit. The status word is read on the engine stream into the pinned counter
  // mirror (no device-wide sync); the timeout bit is reported once and then cleared, so the next
  // synchronize reports only a new timeout (the flags are per-launch tags: later launches are not
  // affected). TSDF_STATUS_PIPELINE_TIMEOUT stays visible in tsdf_get_stats until then.
  HIP_OK(hipMemcpyAsync(&e->h_ctr->status, &e->D.ctr->status, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  if (e->h_ctr->status & TSDF_STATUS_PIPELINE_TIMEOUT) {
    const uint32_t st = e->h_ctr->status & ~(uint32_t)TSDF_STATUS_PIPELINE_TIMEOUT;
    HIP_OK(hipMemcpyAsync(&e->D.ctr->status, &st, sizeof(st), hipMemcpyHostToDevice, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    set_error("tsdf_synchronize: a pipelined frame's in-kernel wait timed out (TSDF_STATUS_PIPELINE_TIMEOUT)");
    return TSDF_ERR_PIPELINE;
  }
  return TSDF_OK;
}

namespace {

// the launch that reads the pending uploaded frame has been enqueued on the engine stream: its slot is
// free for an upload once the engine stream gets here
// and the call returns only once the upload is complete: the caller may reuse its host buffers (the
// reference's synchronous cudaMemcpy contract)
int upload_release(tsdf_engine* e) {
  if (e->up_pending < 0) return TSDF_OK;
  const int k = e->up_pending;
  e->up_pending = -1;
  HIP_OK(hipEventRecord(e->up_free[k], e->stream));
  e->up_used[k] = true;
  for (int j = 0; j < e->up_nstreams; ++j) HIP_OK(hipEventSynchronize(e->up_done[k][j]));
  return TSDF_OK;
}

// the next profiling event set (a std::deque: push_back never moves the sets earlier frames hold)
int take_events(tsdf_engine* e, std::array<hipEvent_t, 5>** out) {
  if (e->ev_used == e->events.size()) {
    std::array<hipEvent_t, 5> a{};
    // (no system-scope fence when an event completes: with it, the dispatch an event pair is bound to
    // ran ~6 us longer than the others -- 50.1 vs 44.3 us in the driver command's kernel trace)
    for (auto& x : a) HIP_OK(hipEventCreateWithFlags(&x, hipEventDisableSystemFence));
    e->events.push_back(a);
  }
  *out = &e->events[e->ev_used++];
  return TSDF_OK;
}

// Phase 1 of a frame: stage host inputs, then (launch) k_ingest_dda on view Dv (the frame's lists,
// counts and candidates: frame_view): pixel records for the whole frame, the DDA over tiles of slice
// `slice_index` of `slice_count` -- contiguous bands of tile rows --, the visibility of the existing
// blocks, and the allocation in its last workgroup. *P / *ev carry the frame to the later phases.
int frame_ingest(tsdf_engine* e, const EngineDev& Dv, const tsdf_frame* f, const tsdf_intrinsics* K,
                 const tsdf_pose* pose, float max_depth, int slice_index, int slice_count, FrameParams* P,
                 std::array<hipEvent_t, 5>** ev_out, void* keys_out = nullptr, int key_cap = 0,
                 bool launch = true, int pix_buf = 0) {
  if (!e || !f || !K || !pose || !f->depth || !f->rgb || f->width <= 0 || f->height <= 0 ||
      (int64_t)f->width * f->height > e->max_pixels || f->width > e->cfg.max_width ||
      f->height > e->cfg.max_height || (f->ht == nullptr) != (f->lt == nullptr) ||
      slice_count < 1 || slice_index < 0 || slice_index >= slice_count) {
    set_error("tsdf_integrate: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  const int W = f->width, H = f->height;
  const size_t np = (size_t)W * H;
  hipStream_t s = e->stream;
  const float* depth = f->depth;
  const uint8_t* rgb = f->rgb;
  const float* ht = f->ht;
  const float* lt = f->lt;
  if (f->mem_kind == TSDF_MEM_HOST) {  // voxel_tsdf.cu:358-365 (H2D; pageable or pinned host memory)
    // The upload runs on the upload streams into the next of two staging slots, beside the frames the
    // engine stream is still running; the engine stream waits for it (up_done) and the slot's next
    // upload waits until the launch reading this frame is enqueued and done (up_free, recorded by
    // upload_release). The call returns once the copies are complete, so the caller may reuse its
    // buffers (the reference's synchronous cudaMemcpy contract).
    if (int rc = upload_release(e)) return rc;
    const int k = e->up_next;
    e->up_next ^= 1;
    // the copies round-robin over the upload streams (TSDF_UPLOAD_STREAMS, default 2): the copies run on several DMA
    // engines at once; the engine stream waits for each
    const int nu = std::max(1, std::min(e->env.upload_streams, (int)tsdf_engine::kUpStreams));
    const void* src[4] = {rgb, depth, ht, lt};
    const size_t bytes[4] = {np * 3, np * 4, np * 4, np * 4};
    void* dst[4] = {e->s_rgb + (size_t)k * e->max_pixels * 3, e->s_depth + (size_t)k * e->max_pixels,
                    e->s_ht + (size_t)k * e->max_pixels, e->s_lt + (size_t)k * e->max_pixels};
    const int ncopy = ht ? 4 : 2;
    e->up_nstreams = std::min(nu, ncopy);
    for (int j = 0; j < e->up_nstreams; ++j)
      if (e->up_used[k]) HIP_OK(hipStreamWaitEvent(e->ustream[j], e->up_free[k], 0));
    for (int c = 0; c < ncopy; ++c)
      HIP_OK(hipMemcpyAsync(dst[c], src[c], bytes[c], hipMemcpyHostToDevice, e->ustream[c % e->up_nstreams]));
    for (int j = 0; j < e->up_nstreams; ++j) {
      HIP_OK(hipEventRecord(e->up_done[k][j], e->ustream[j]));
      HIP_OK(hipStreamWaitEvent(s, e->up_done[k][j], 0));
    }
    rgb = static_cast<const uint8_t*>(dst[0]);
    depth = static_cast<const float*>(dst[1]);
    if (ht) {
      ht = static_cast<const float*>(dst[2]);
      lt = static_cast<const float*>(dst[3]);
    }
    // (the host waits for the copies in upload_release, after the launch that reads them is enqueued:
    // the enqueue overlaps the transfer)
    e->up_pending = k;
  } else if (f->mem_kind != TSDF_MEM_DEVICE) {
    set_error("tsdf_integrate: bad mem_kind");
    return TSDF_ERR_INVALID_ARG;
  }
  *P = make_params(e, K, W, H, pose, max_depth);
  P->depth = depth;
  P->rgb = rgb;
  P->ht = ht;
  P->lt = lt;
  P->pix_off = pix_buf ? (int)e->max_pixels : 0;  // which of the two pixel-record buffers
  // a shard's k_integrate reads the raw frame: no whole-frame pixel pass in its ingest
  P->pack_pixels = e->cfg.shard_count > 1 ? 0 : 1;
  const int tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16;
  P->tile_lo = 0;
  P->tile_hi = tiles_x * tiles_y;
  if (slice_count > 1) {  // contiguous bands of tile rows
    const int rows = (tiles_y + slice_count - 1) / slice_count;
    P->tile_lo = std::min(tiles_y, slice_index * rows) * tiles_x;
    P->tile_hi = std::min(tiles_y, (slice_index + 1) * rows) * tiles_x;
  }
  const int tiles = P->tile_hi - P->tile_lo;  // the launch covers the DDA's tiles only
  if (keys_out) {  // the last workgroup packs the keys for the exchange instead of resolving them
    P->tail = kTailPack;
    P->slot = reinterpret_cast<ShardRec*>(keys_out);
    P->slot_cap = key_cap;
  }
  std::array<hipEvent_t, 5>* ev = nullptr;
  if (e->profiling && (e->prof_calls++ % e->prof_every) == 0) {
    int rc = take_events(e, &ev);
    if (rc) return rc;
  }
  *ev_out = ev;
  if (!launch) return TSDF_OK;
  if (ev && e->prof_mode == TSDF_PROFILE_PHASES) HIP_OK(hipEventRecord((*ev)[0], s));
  // ---- allocate (voxel_tsdf.cu:377-386) + visibility (:388-397) ----
  // k_ingest_dda sweeps the blocks that already exist for visibility beside the DDA; its last
  // workgroup resolves the new keys and appends the blocks it creates to the visible lists
  if (e->rd.pending && e->maxs <= 3 && slice_count == 1 && !keys_out && e->cfg.shard_count <= 1) {
    // the deferred raycast of the previous frame in the same launch (k_render_ingest)
    e->rd.pending = false;
    const tsdf_engine::DeferredRender& r = e->rd;
    const int rgx = (r.P.W + 15) / 16, nray = rgx * ((r.P.nrows + 15) / 16);
    hipLaunchKernelGGL(k_render_ingest, dim3(nray + kVisWorkgroups + tiles), dim3(256), 0, s, Dv, r.P, r.step, r.V,
                       r.rgba, r.normal, rgx, nray, *P, depth, rgb, ht, lt, tiles_x, tiles);
    LAUNCH_OK("k_render_ingest");
    return TSDF_OK;
  }
  {  // a deferred raycast this ingest cannot take up runs first; a TSDF_RENDER_OVERLAP raycast on the
     // render stream keeps overlapping this ingest (it writes nothing the raycast reads; the update joins it)
    int rc = join_render(e, false, false);
    if (rc) return rc;
  }
  if (e->maxs <= 3)
    hipLaunchKernelGGL(k_ingest_dda<1024>, dim3(kVisWorkgroups + tiles), dim3(256), 0, s, Dv, *P, depth,
                       rgb, ht, lt, tiles_x, tiles);
  else
    hipLaunchKernelGGL(k_ingest_dda<2048>, dim3(kVisWorkgroups + tiles), dim3(256), 0, s, Dv, *P, depth,
                       rgb, ht, lt, tiles_x, tiles);
  LAUNCH_OK("k_ingest_dda");
  return TSDF_OK;
}

// Phase 2: fused update (+ carve minimum) on view Dv; the last workgroup carves (kTailResolve) or
// packs a shard's carve candidates into cands_out. (Measured and not kept in round 1: running the
// update of the existing blocks beside the allocation resolver, on a second stream or as a dispatch
// without the AQL barrier bit: the resolver's chain of dependent HBM round trips slows ~2.5x under
// the update's memory load.)
int frame_update(tsdf_engine* e, const EngineDev& Dv, FrameParams P, std::array<hipEvent_t, 5>* ev,
                 void* cands_out = nullptr, int cand_cap = 0) {
  hipStream_t s = e->stream;
  JOIN_RENDER(e);  // the update writes the pool a raycast on the render stream may still read
  const bool all_ev = ev && e->prof_mode == TSDF_PROFILE_PHASES;
  if (all_ev) HIP_OK(hipEventRecord((*ev)[1], s));
  P.tail = cands_out ? kTailPack : kTailResolve;
  P.slot = reinterpret_cast<ShardRec*>(cands_out);
  P.slot_cap = cand_cap;
  // ---- update (voxel_tsdf.cu:474-481) + space carving (:483-488) ----
  auto kfn = P.pack_pixels ? k_integrate_t<false, false> : k_integrate_t<false, true>;
  if (ev && e->prof_mode == TSDF_PROFILE_KERNEL) {
    // the two events are bound to the kernel's own dispatch packet (its begin / end timestamps,
    // the interval rocprofv3's kernel trace reports): no marker packets enter the stream
    hipExtLaunchKernelGGL(kfn, dim3(e->D.integrate_grid), dim3(kIntegrateThreads), 0, s,
                          (*ev)[2], (*ev)[3], 0, Dv, P, (const FrameArgs*)nullptr);
  } else {
    if (ev) HIP_OK(hipEventRecord((*ev)[2], s));
    hipLaunchKernelGGL(kfn, dim3(e->D.integrate_grid), dim3(kIntegrateThreads), 0, s,
                       Dv, P, (const FrameArgs*)nullptr);
    if (ev) HIP_OK(hipEventRecord((*ev)[3], s));
  }
  LAUNCH_OK("k_integrate");
  if (all_ev && !cands_out) HIP_OK(hipEventRecord((*ev)[4], s));
  return TSDF_OK;
}

// the launch-wide fields of a k_frame's arguments
void finish_args(tsdf_engine* e, PipeArgs& A, const FrameParams& Pu) {
  A.tag = ++e->pipe_tag ? e->pipe_tag : ++e->pipe_tag;  // (0: the flags' initial value)
  A.nint = e->D.integrate_grid_pre;
  A.order = e->frame_order;
  A.range = A.has_alloc ? (uint32_t)((size_t)Pu.W * Pu.H * e->maxs) : 0u;
  if (!A.has_frame) A.tiles = A.tiles_x = 0;
  A.tiles_per_wg = std::max(1, e->env.frame_tiles_per_wg);
  A.tile_wgs = (A.tiles + A.tiles_per_wg - 1) / A.tiles_per_wg;
}

// One k_frame launch (tsdf_fuse.hip): frame A.fid_carve's carving, frame A.fid_alloc's allocation and
// update (camera / pixel records Pu), frame A.fid_new's ingest (Pn) -- the parts A enables.
int launch_frame(tsdf_engine* e, PipeArgs A, const FrameParams& Pu, const FrameParams& Pn,
                 std::array<hipEvent_t, 5>* ev) {
  hipStream_t s = e->stream;
  JOIN_RENDER(e);
  finish_args(e, A, Pu);
  const int nwg = kPipeHead + (A.has_update ? A.nint : 0) + pipe_fresh_wgs(A) +
                  (A.has_frame ? A.tile_wgs + kVisWorkgroups : 0);
  if (e->profiling && A.has_frame) ++e->prof_pipelined;  // (frame launches; not the flush's)
  if (ev && e->prof_mode == TSDF_PROFILE_KERNEL) {
    hipExtLaunchKernelGGL(k_frame, dim3(nwg), dim3(kIntegrateThreads), 0, s, (*ev)[2], (*ev)[3], 0, e->D, Pu, Pn, A);
  } else {
    // (phase events: the launch is the whole frame -- "integrate" spans it, the other phases are empty)
    const bool all_ev = ev && e->prof_mode == TSDF_PROFILE_PHASES;
    if (all_ev) HIP_OK(hipEventRecord((*ev)[0], s));
    if (all_ev) HIP_OK(hipEventRecord((*ev)[1], s));
    if (ev) HIP_OK(hipEventRecord((*ev)[2], s));
    hipLaunchKernelGGL(k_frame, dim3(nwg), dim3(kIntegrateThreads), 0, s, e->D, Pu, Pn, A);
    if (ev) HIP_OK(hipEventRecord((*ev)[3], s));
    if (all_ev) HIP_OK(hipEventRecord((*ev)[4], s));
  }
  LAUNCH_OK("k_frame");
  return TSDF_OK;
}

bool sharded(const tsdf_engine* e) { return e->cfg.shard_count > 1; }
// Frames up to pipe_max_pixels (2^19; TSDF_PIPE_MAX_PIXELS) are pipelined (k_frame). Larger frames take the two launches: their
// ingest (3,600 tiles at 1280x720) no longer fits beside the update in one launch's resident
// workgroups, and the serialised launch is slower (C4, driver-size runs: 13.0-13.3k frames/s
// pipelined against 14.6-14.8k in two launches; at 640x480 21.4k against 19.1k).
bool pipe_frame_size(const tsdf_engine* e, int w, int h) { return (int64_t)w * h <= e->pipe_max_pixels; }

// The k_frame launch that continues the pending frames, with (has_frame) the ingest of a new frame
// fid whose parameters are Pn; the state moves to kPipeCAU (or kPipeAU from kPipeNone).
PipeArgs pipe_step(tsdf_engine* e, bool has_frame, uint32_t fid, const FrameParams& Pn) {
  PipeArgs A{};
  const int ps = e->ps;
  if (ps != tsdf_engine::kPipeNone) {
    A.has_update = 1;
    A.fid_alloc = e->p_fid;
    A.fresh_ready = ps == tsdf_engine::kPipeU;  // p_fid's new blocks were listed by its k_ingest_dda
    A.has_alloc = ps != tsdf_engine::kPipeU;
    A.has_carve = ps == tsdf_engine::kPipeCAU;
    A.fid_carve = e->p_carve;
  }
  if (has_frame) {
    A.has_frame = 1;
    A.fid_new = fid;
    A.tiles_x = (Pn.W + 15) / 16;
    A.tiles = A.tiles_x * ((Pn.H + 15) / 16);
  }
  return A;
}
void pipe_advance(tsdf_engine* e, uint32_t fid, const FrameParams& Pn) {
  if (e->ps == tsdf_engine::kPipeNone) {
    e->ps = tsdf_engine::kPipeAU;
  } else {
    e->p_carve = e->p_fid;
    e->ps = tsdf_engine::kPipeCAU;
  }
  e->p_fid = fid;
  e->p_P = Pn;
}
uint32_t next_fid(tsdf_engine* e) {
  uint32_t fid = e->fid_next++;
  // never 0; after 2^32 - 1 (= 3 mod 6) comes 4: consecutive frames keep distinct parity (frame_view's
  // two-frame lists) and residue mod 3 (its three band views)
  if (fid == 0u) {
    fid = 4u;
    e->fid_next = 5u;
  }
  return fid;
}

// complete the pending frames (pipelined): kPipeU -- the frame's update with its carving in its last
// workgroup (k_integrate); kPipeCAU -- one k_frame for the pending carving, allocation and update,
// then one for that frame's own carving
int flush_pending(tsdf_engine* e) {
  if (e->ps == tsdf_engine::kPipeNone) return TSDF_OK;
  if (sharded(e)) {  // its carvings need every shard's candidates: only the exchange protocol can
    set_error("a pipelined sharded frame is pending: complete it with tsdf_integrate_shard_pipe(frame = "
              "NULL) until *pending == 0");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  const int ps = e->ps;
  e->ps = tsdf_engine::kPipeNone;
  if (ps == tsdf_engine::kPipeU) {
    // a sampled frame's update is timed here (the C5 loop: a raycast after every frame flushes it);
    // (PHASES mode: its allocation ran in the ingest launch before, so event 0 opens at the update)
    std::array<hipEvent_t, 5>* ev = nullptr;
    if (e->p_sampled && e->profiling) {
      int rc = take_events(e, &ev);
      if (rc) return rc;
      if (e->prof_mode == TSDF_PROFILE_PHASES) HIP_OK(hipEventRecord((*ev)[0], e->stream));
    }
    e->p_sampled = false;
    return frame_update(e, frame_view(e->D, e->p_fid), e->p_P, ev);
  }
  PipeArgs A{};
  A.has_carve = ps == tsdf_engine::kPipeCAU;
  A.fid_carve = e->p_carve;
  A.has_alloc = 1;
  A.has_update = 1;
  A.fid_alloc = e->p_fid;
  const FrameParams none{};
  int rc = launch_frame(e, A, e->p_P, none, nullptr);
  if (rc) return rc;
  PipeArgs C{};
  C.has_carve = 1;
  C.fid_carve = e->p_fid;
  return launch_frame(e, C, none, none, nullptr);
}

// The pending unpipelined update (ps == kPipeU) with the view grid of render camera R built in the same
// launch (k_integrate_vg; raycast_impl's deferred C5 path). Events as flush_pending + frame_update.
int update_with_grid(tsdf_engine* e, const FrameParams& R, const ViewGrid& V) {
  hipStream_t s = e->stream;
  std::array<hipEvent_t, 5>* ev = nullptr;
  if (e->p_sampled && e->profiling) {
    int rc = take_events(e, &ev);
    if (rc) return rc;
    if (e->prof_mode == TSDF_PROFILE_PHASES) HIP_OK(hipEventRecord((*ev)[0], s));
  }
  e->p_sampled = false;
  e->ps = tsdf_engine::kPipeNone;
  const EngineDev Dv = frame_view(e->D, e->p_fid);
  FrameParams P = e->p_P;
  P.tail = kTailResolve;
  P.slot = nullptr;
  P.slot_cap = 0;
  const uint32_t vtag = 0x80000000u | (uint32_t)(e->vg_calls & 0x7FFFFFFFu);  // (never a frame id)
  const int nint = e->D.integrate_grid;
  const dim3 grid(nint + kOccWords / 256);
  const bool all_ev = ev && e->prof_mode == TSDF_PROFILE_PHASES;
  if (all_ev) HIP_OK(hipEventRecord((*ev)[1], s));
  if (ev && e->prof_mode == TSDF_PROFILE_KERNEL) {
    hipExtLaunchKernelGGL(k_integrate_vg, grid, dim3(kIntegrateThreads), 0, s, (*ev)[2], (*ev)[3], 0, Dv, P, R, V,
                          vtag, nint);
  } else {
    if (ev) HIP_OK(hipEventRecord((*ev)[2], s));
    hipLaunchKernelGGL(k_integrate_vg, grid, dim3(kIntegrateThreads), 0, s, Dv, P, R, V, vtag, nint);
    if (ev) HIP_OK(hipEventRecord((*ev)[3], s));
  }
  LAUNCH_OK("k_integrate_vg");
  if (all_ev) HIP_OK(hipEventRecord((*ev)[4], s));
  return TSDF_OK;
}

}  // namespace

// One frame (TSDFGrid::Integrate). Pipelined (one volume, <= 3 DDA samples per pixel):
// tsdf_integrate of frame c launches ONE k_frame that carves frame c - 2, allocates and updates frame
// c - 1 and runs frame c's ingest; what remains (c - 1's carving, c's allocation and update) runs in
// the next call's launch, or in flush_pending, which every other entry point (and tsdf_flush /
// tsdf_synchronize) calls first. Stream order and the in-launch flags keep every result identical to
// the unpipelined two launches per frame.
int tsdf_integrate(tsdf_engine* e, const tsdf_frame* f, const tsdf_intrinsics* K,
                   const tsdf_pose* pose, float max_depth) {
  TraceRange trace_("tsdf_integrate");
  if (e && sharded(e)) {
    set_error("tsdf_integrate: a shard of a sharded volume integrates through tsdf_integrate_shard_*");
    return TSDF_ERR_INVALID_ARG;
  }
  if (!e || !f || !K || !pose) {  // (before anything reads the frame: pipe_frame_size below does)
    set_error("tsdf_integrate: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  const bool pipe = e->pipeline && e->maxs <= 3 && pipe_frame_size(e, f->width, f->height);
  if (!pipe) {
    int rc = flush_pending(e);
    if (rc) return rc;
  }
  const uint32_t fid = next_fid(e);
  const EngineDev Dv = frame_view(e->D, fid);
  FrameParams P;
  std::array<hipEvent_t, 5>* ev = nullptr;
  // the first frame after a flush runs k_ingest_dda (its ingest and allocation in one launch)
  const bool ingest_alone = !pipe || e->ps == tsdf_engine::kPipeNone;
  int rc = frame_ingest(e, Dv, f, K, pose, max_depth, 0, 1, &P, &ev, nullptr, 0, ingest_alone, (int)(fid & 1u));
  if (rc) {
    (void)upload_release(e);  // (a failed launch after the upload: the host buffers are still read)
    return rc;
  }
  if (!pipe) {
    rc = frame_update(e, Dv, P, ev);
    const int ru = upload_release(e);
    return rc ? rc : ru;
  }
  if (ingest_alone) {
    // (no k_frame / k_integrate launch to time in this call: the slot is released, and the update,
    // if a flush launches it as k_integrate, takes one then)
    if (ev) --e->ev_used;
    e->p_sampled = ev != nullptr;
    e->ps = tsdf_engine::kPipeU;
    e->p_fid = fid;
    e->p_P = P;
    return upload_release(e);  // (k_ingest_dda read the frame)
  }
  rc = launch_frame(e, pipe_step(e, true, fid, P), e->p_P, P, ev);
  if (rc) {
    (void)upload_release(e);
    return rc;
  }
  pipe_advance(e, fid, P);
  return upload_release(e);  // (the launch's tiles read the frame)
}

int tsdf_flush(tsdf_engine* e) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  return TSDF_OK;
}

// ---------------------------------------------------------------------------------------------
// Sharded frames. Every shard keeps the whole hash index and holds the voxels of its
// own blocks; one frame is three calls around two all-gathers (include/disinfect_tsdf.h).
// ---------------------------------------------------------------------------------------------
int64_t tsdf_shard_slot_bytes(int32_t cap) {
  if (cap < 1) return 0;
  return (int64_t)(cap + 1) * (int64_t)sizeof(ShardRec);
}

int tsdf_integrate_shard_begin(tsdf_engine* e, const tsdf_frame* f, const tsdf_intrinsics* K,
                               const tsdf_pose* pose, float max_depth, int32_t slice_index,
                               int32_t slice_count, void* keys_out, int32_t key_cap) {
  TraceRange trace_("tsdf_integrate_shard_begin");
  if (!e || !sharded(e) || e->shard_phase != 0 || (keys_out && key_cap < 1) ||
      (!keys_out && slice_count != 1)) {
    set_error("tsdf_integrate_shard_begin: invalid argument (a shard engine between frames; a key "
              "slot unless slice_count == 1)");
    return TSDF_ERR_INVALID_ARG;
  }
  ENTER(e);
  FrameParams P;
  std::array<hipEvent_t, 5>* ev = nullptr;
  // split DDA: the last workgroup packs this slice's keys into keys_out; whole-frame DDA (no key
  // exchange): it resolves the allocation right away, like one volume
  int rc = frame_ingest(e, e->D, f, K, pose, max_depth, slice_index, slice_count, &P, &ev, keys_out, key_cap);
  // (a host frame: its upload is complete on return -- the slot itself is released after _update)
  if (e->up_pending >= 0)
    for (int j = 0; j < e->up_nstreams; ++j) HIP_OK(hipEventSynchronize(e->up_done[e->up_pending][j]));
  if (rc) return rc;
  P.tail = kTailResolve;
  P.slot = nullptr;
  P.slot_cap = 0;
  e->shard_P = P;
  e->shard_ev = ev;
  e->shard_keys_packed = keys_out != nullptr;
  e->shard_phase = 1;
  return TSDF_OK;
}

int tsdf_integrate_shard_update(tsdf_engine* e, const void* keys_in, int32_t key_cap, void* cands_out,
                                int32_t cand_cap) {
  TraceRange trace_("tsdf_integrate_shard_update");
  if (!e || e->shard_phase != 1 || (keys_in != nullptr) != e->shard_keys_packed ||
      (keys_in && key_cap < 1) || !cands_out || cand_cap < 1) {
    set_error("tsdf_integrate_shard_update: invalid argument (after tsdf_integrate_shard_begin; the "
              "key inbox iff _begin packed keys; a candidate slot)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  if (keys_in) {  // merge every shard's keys, then the ordered allocation (one workgroup)
    const FrameParams& P = e->shard_P;
    hipLaunchKernelGGL(k_resolve_alloc, dim3(1), dim3(kRT), 0, e->stream, e->D, P,
                       (uint32_t)((size_t)P.W * P.H * e->maxs), 1, reinterpret_cast<const ShardRec*>(keys_in),
                       key_cap, e->cfg.shard_count);
    LAUNCH_OK("k_resolve_alloc");
  }
  int rc = frame_update(e, e->D, e->shard_P, e->shard_ev, cands_out, cand_cap);
  if (rc) return rc;
  e->shard_phase = 2;
  return upload_release(e);  // (a shard's k_integrate reads the raw frame)
}

int tsdf_integrate_shard_end(tsdf_engine* e, const void* cands_in, int32_t cand_cap) {
  TraceRange trace_("tsdf_integrate_shard_end");
  if (!e || e->shard_phase != 2 || !cands_in || cand_cap < 1) {
    set_error("tsdf_integrate_shard_end: invalid argument (after tsdf_integrate_shard_update; the "
              "candidate inbox)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  hipLaunchKernelGGL(k_resolve_delete, dim3(1), dim3(kRT), 0, e->stream, e->D, (const VisRec*)e->D.cand,
                     (const int32_t*)e->D.ncand, 0, reinterpret_cast<const ShardRec*>(cands_in),
                     cand_cap, e->cfg.shard_count);
  LAUNCH_OK("k_resolve_delete");
  e->shard_phase = 0;
  std::array<hipEvent_t, 5>* ev = e->shard_ev;
  if (ev && e->prof_mode == TSDF_PROFILE_PHASES) HIP_OK(hipEventRecord((*ev)[4], e->stream));
  return TSDF_OK;
}

// ---------------------------------------------------------------------------------------------
// Pipelined sharded frames (one exchange per frame): every shard runs the whole frame's
// DDA against its copy of the index (no key exchange: --mode sharded), so only the carve candidates
// cross the shards. Call n launches one k_frame: frame n - 2's carving of every shard's candidates
// (cands_in: the all-gathered slots of call n - 1), frame n - 1's allocation and update (its
// candidates into cands_out, for the exchange after this call), frame n's ingest.
// ---------------------------------------------------------------------------------------------
// tsdf_integrate_shard_pipe, and a group's form (dsts: the update's last workgroup writes the
// candidate slot into the ndst device slots listed at dsts -- a device array; dsts_host: the same
// pointers, for the zeroed headers of the first call -- instead of cands_out)
static int shard_pipe_impl(tsdf_engine* e, const tsdf_frame* f, const tsdf_intrinsics* K, const tsdf_pose* pose,
                           float max_depth, const void* cands_in, void* cands_out, ShardRec* const* dsts,
                           ShardRec* const* dsts_host, int ndst, int32_t cand_cap, int32_t* pending) {
  HIP_OK(hipSetDevice(e->device));
  JOIN_RENDER(e);
  *pending = 0;
  const ShardRec* in = reinterpret_cast<const ShardRec*>(cands_in);
  ShardRec* out = reinterpret_cast<ShardRec*>(cands_out);
  auto shard_args = [&](PipeArgs& A) {
    A.cands_in = A.has_carve ? in : nullptr;
    A.cands_out = A.has_update ? out : nullptr;
    A.cands_dst = A.has_update ? dsts : nullptr;
    A.ndst = ndst;
    A.cand_cap = cand_cap;
    A.nshard = e->cfg.shard_count;
  };
  const FrameParams none{};
  if (!f) {  // one step of completing the pending frames
    const int ps = e->ps;
    if (ps == tsdf_engine::kPipeNone) return TSDF_OK;
    PipeArgs A{};
    if (ps == tsdf_engine::kPipeC) {
      A.has_carve = 1;
      A.fid_carve = e->p_fid;
      shard_args(A);
      int rc = launch_frame(e, A, none, none, nullptr);
      if (rc) return rc;
      e->ps = tsdf_engine::kPipeNone;
      return TSDF_OK;
    }
    A = pipe_step(e, false, 0u, none);
    shard_args(A);
    int rc = launch_frame(e, A, e->p_P, none, nullptr);
    if (rc) return rc;
    e->ps = tsdf_engine::kPipeC;  // (p_fid's carving, after the exchange of its candidates)
    *pending = 1;
    return TSDF_OK;
  }
  if (e->ps == tsdf_engine::kPipeC) {
    set_error("tsdf_integrate_shard_pipe: a flush is in progress (call with frame = NULL until *pending == 0)");
    return TSDF_ERR_INVALID_ARG;
  }
  const uint32_t fid = next_fid(e);
  FrameParams P;
  std::array<hipEvent_t, 5>* ev = nullptr;
  int rc = frame_ingest(e, frame_view(e->D, fid), f, K, pose, max_depth, 0, 1, &P, &ev, nullptr, 0, false,
                        (int)(fid & 1u));
  if (rc) return rc;
  P.pack_pixels = 1;  // every shard packs the whole frame's pixel records (its blocks project anywhere)
  if (e->ps == tsdf_engine::kPipeNone) {  // the first frame: ingest + allocation in one launch
    const EngineDev Dv = frame_view(e->D, fid);
    const int tiles = P.tile_hi - P.tile_lo, tiles_x = (P.W + 15) / 16;
    HIP_OK(hipMemsetAsync(&e->D.ctr->n_pend, 0, sizeof(int32_t), e->stream));  // (its allocation's list)
    hipLaunchKernelGGL(k_ingest_dda<1024>, dim3(kVisWorkgroups + tiles), dim3(256), 0, e->stream, Dv, P, P.depth,
                       P.rgb, P.ht, P.lt, tiles_x, tiles);
    LAUNCH_OK("k_ingest_dda");
    if (dsts_host) {  // (no candidates from this call)
      for (int d = 0; d < ndst; ++d) HIP_OK(hipMemsetAsync(dsts_host[d], 0, sizeof(ShardRec), e->stream));
    } else {
      HIP_OK(hipMemsetAsync(out, 0, sizeof(ShardRec), e->stream));
    }
    if (ev) --e->ev_used;
    e->ps = tsdf_engine::kPipeU;
    e->p_fid = fid;
    e->p_P = P;
    return upload_release(e);
  }
  PipeArgs A = pipe_step(e, true, fid, P);
  shard_args(A);
  rc = launch_frame(e, A, e->p_P, P, ev);
  if (rc) return rc;
  pipe_advance(e, fid, P);
  return upload_release(e);
}

// the group's entry (csrc/tsdf_group.hip, declared in csrc/tsdf_internal.h): tsdf_integrate_shard_pipe
// with the candidate slot written into the ndst slots at dsts_dev (device array) instead of an
// outgoing slot
int tsdf_integrate_shard_pipe_fanout(tsdf_engine* e, const tsdf_frame* f, const tsdf_intrinsics* K,
                                     const tsdf_pose* pose, float max_depth, const void* cands_in,
                                     void* const* dsts_dev, void* const* dsts_host, int ndst, int32_t cand_cap,
                                     int32_t* pending) {
  TraceRange trace_("tsdf_integrate_shard_pipe_fanout");
  if (!e || !sharded(e) || e->shard_phase != 0 || !cands_in || !dsts_dev || !dsts_host || ndst < 1 ||
      cand_cap < 1 || !pending || (f && (!K || !pose)) || e->maxs > 3) {
    set_error("tsdf_integrate_shard_pipe_fanout: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  ShardRec* self = reinterpret_cast<ShardRec*>(dsts_host[e->cfg.shard_index % ndst]);
  return shard_pipe_impl(e, f, K, pose, max_depth, cands_in, self, reinterpret_cast<ShardRec* const*>(dsts_dev),
                         reinterpret_cast<ShardRec* const*>(dsts_host), ndst, cand_cap, pending);
}

int tsdf_integrate_shard_pipe(tsdf_engine* e, const tsdf_frame* f, const tsdf_intrinsics* K,
                              const tsdf_pose* pose, float max_depth, const void* cands_in, void* cands_out,
                              int32_t cand_cap, int32_t* pending) {
  TraceRange trace_("tsdf_integrate_shard_pipe");
  if (!e || !sharded(e) || e->shard_phase != 0 || !cands_in || !cands_out || cand_cap < 1 || !pending ||
      (f && (!K || !pose)) || e->maxs > 3) {
    set_error("tsdf_integrate_shard_pipe: invalid argument (a shard engine between frames, both slots, "
              "<= 3 DDA samples per pixel)");
    return TSDF_ERR_INVALID_ARG;
  }
  return shard_pipe_impl(e, f, K, pose, max_depth, cands_in, cands_out, nullptr, nullptr, 0, cand_cap, pending);
}

int tsdf_integrate_shard_abort(tsdf_engine* e) {
  TraceRange trace_("tsdf_integrate_shard_abort");
  if (!e || !sharded(e)) {
    set_error("tsdf_integrate_shard_abort: not a shard engine");
    return TSDF_ERR_INVALID_ARG;
  }
  if (e->shard_phase == 0 && e->ps == tsdf_engine::kPipeNone) return TSDF_OK;  // nothing pending
  HIP_OK(hipSetDevice(e->device));
  // (not ENTER: a pending pipelined sharded frame cannot be flushed without the exchange protocol --
  // it is dropped here with the rest of the frame's state)
  JOIN_RENDER(e);
  e->shard_phase = 0;
  e->shard_ev = nullptr;
  e->ps = tsdf_engine::kPipeNone;
  hipLaunchKernelGGL(k_shard_abort, dim3(1), dim3(256), 0, e->stream, e->D);
  LAUNCH_OK("k_shard_abort");
  if (int rc = upload_release(e)) return rc;
  return TSDF_OK;
}

int tsdf_stream_wait(tsdf_engine* e, void* stream) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  hipStream_t other = reinterpret_cast<hipStream_t>(stream);
  if (other == e->stream) return TSDF_OK;
  HIP_OK(hipSetDevice(e->device));
  int rc = join_render(e, true);
  if (rc) return rc;
  if (!e->order_ev) HIP_OK(hipEventCreateWithFlags(&e->order_ev, hipEventDisableTiming));
  HIP_OK(hipEventRecord(e->order_ev, other));
  HIP_OK(hipStreamWaitEvent(e->stream, e->order_ev, 0));
  return TSDF_OK;
}

int tsdf_stream_signal(tsdf_engine* e, void* stream) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  hipStream_t other = reinterpret_cast<hipStream_t>(stream);
  if (other == e->stream) return TSDF_OK;
  HIP_OK(hipSetDevice(e->device));
  JOIN_RENDER(e);
  if (!e->order_ev) HIP_OK(hipEventCreateWithFlags(&e->order_ev, hipEventDisableTiming));
  HIP_OK(hipEventRecord(e->order_ev, e->stream));
  HIP_OK(hipStreamWaitEvent(other, e->order_ev, 0));
  return TSDF_OK;
}

int tsdf_get_stream(tsdf_engine* e, void** stream) {
  if (!e || !stream) return TSDF_ERR_INVALID_ARG;
  *stream = reinterpret_cast<void*>(e->stream);
  return TSDF_OK;
}

namespace {

// The view grid of one raycast of camera P (tsdf_kernels.h ViewGrid). Its cube reaches every voxel
// a ray can read: positions up to max_step * step_size / voxel grid units from the camera centre
// (|direction| = 1 up to rounding), plus the binary search, the +-1 gradient neighbours and the
// rounding to the nearest voxel (2.5 voxels). n = 0 (hash lookups) when the cube would exceed
// kViewMaxN cells per axis, the brick bitmap `lds_words` of LDS, or the pool a cell's index bits.
// The cube's shape for a camera: ok = false when a view grid does not apply (hash lookups)
struct ViewShape {
  bool ok = false;
  int n = 0, nb = 0, ns = 0, nbw = 0, nw = 0, half = 0;
  int64_t cells = 0;  // brick-major (view_cell)
};
void view_shape(const tsdf_engine* e, const FrameParams& P, float step_size, int lds_words, ViewShape* out) {
  ViewShape& S = *out;
  S = ViewShape{};
  const double max_step = std::ceil((double)P.max_depth / (double)step_size);
  const double reach = max_step * (double)step_size / (double)P.voxel * (1.0 + 1e-5) + 2.5;
  if (!(reach < 1e6)) return;
  S.half = (int)std::ceil(reach / kBlockLen) + 1;
  S.n = 2 * S.half + 1;
  S.nb = (S.n + 3) / 4;
  S.ns = (S.nb + 3) / 4;
  S.nbw = (S.nb * S.nb * S.nb + 31) / 32;
  S.nw = S.nbw + (S.ns * S.ns * S.ns + 31) / 32;
  S.cells = (int64_t)S.nb * S.nb * S.nb * 64;
  S.ok = S.n <= kViewMaxN && S.nw <= lds_words && e->D.nblocks <= (1 << kViewIdxBits);
}
// whether view_grid_for(P) would clear or reallocate the grid's cells (a deferred raycast reading the
// previous grid must run first): the same shape and the same two conditions view_grid_for acts on
bool view_grid_resets(const tsdf_engine* e, const FrameParams& P, float step_size, int lds_words) {
  ViewShape S;
  view_shape(e, P, step_size, lds_words, &S);
  return S.ok && (S.cells > e->vg_cap || e->vg_gen == kViewGenMax);
}

int view_grid_for(tsdf_engine* e, const FrameParams& P, float step_size, int lds_words, ViewGrid* V) {
  *V = ViewGrid{};
  V->flags = e->vg_flags;
  V->bits = e->vg_bits;
  ViewShape S;
  view_shape(e, P, step_size, lds_words, &S);
  if (!S.ok) return TSDF_OK;
  const int n = S.n, nb = S.nb, ns = S.ns, nbw = S.nbw, nw = S.nw, half = S.half;
  const int64_t cells = S.cells;
  if (cells > e->vg_cap) {
    if (e->vg_cell) HIP_OK(hipFree(e->vg_cell));
    e->vg_cell = nullptr;
    e->vg_cap = 0;
    HIP_OK(hipMalloc(&e->vg_cell, (size_t)cells * 4));
    HIP_OK(hipMemsetAsync(e->vg_cell, 0, (size_t)cells * 4, e->stream));
    e->vg_cap = cells;
    e->vg_gen = 0;
  }
  if (e->vg_gen == kViewGenMax) {  // generations exhausted: stale cells must not match gen 1 again
    HIP_OK(hipMemsetAsync(e->vg_cell, 0, (size_t)e->vg_cap * 4, e->stream));
    e->vg_gen = 0;
  }
  e->vg_gen += 1;
  e->vg_calls += 1;
  V->cell = e->vg_cell;
  V->n = n;
  V->nb = nb;
  V->ns = ns;
  V->nbw = nbw;
  V->nw = nw;
  V->half = half;
  V->gen = e->vg_gen;
  return TSDF_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Graph-captured frame loop (BASELINE config C5): the whole per-frame sequence -- argument upload,
// k_ingest_dda, k_resolve_alloc, k_integrate, k_resolve_delete and (optionally) k_raycast -- is one
// hipGraph launch. The graph's first node copies a FrameArgs block (cameras, frame and output
// pointers) from a pinned host slot, so one instantiated graph serves every frame; kSlots graphs
// with their own slots let the host fill frame i+1 while frame i runs.
// ---------------------------------------------------------------------------------------------
#ifndef TSDF_GRAPH_DONE_FLAGS
#define TSDF_GRAPH_DONE_FLAGS hipEventDisableTiming
#endif
constexpr unsigned kGraphDoneFlags = TSDF_GRAPH_DONE_FLAGS;
struct tsdf_graph {
  static constexpr int kSlots = 4;
  static constexpr int kSegs = 3;  // a shard's frame: begin / update / end around the exchanges
  tsdf_engine* e = nullptr;
  int W = 0, H = 0, RW = 0, RH = 0;
  bool shard = false;     // a shard engine's graph (tsdf_graph_create_shard)
  bool pipe = false;      // pipelined frames: each launch is one k_frame_g (no render camera)
  bool defer = false;     // render-deferring graph (tsdf_graph_create_deferred): each launch renders the
                          // previous frame's camera beside its ingest (k_render_ingest_g)
  int slice_index = 0, slice_count = 1;
  int cur = -1;           // a shard's frame in flight: its slot
  hipStream_t cap = nullptr;  // capture stream (the engine stream may be a legacy default stream)
  FrameArgs* d_args = nullptr;
  FrameArgs* h_args = nullptr;  // pinned
  hipGraph_t graph[kSlots][kSegs] = {};
  hipGraphExec_t exec[kSlots][kSegs] = {};
  hipEvent_t done[kSlots] = {};
  bool used[kSlots] = {};
  int next = 0;
  // batched graphs (tsdf_graph_create_batch): slot k's graph runs `batch` frames, args entries
  // [k batch, (k + 1) batch); one[k][j] runs entry j alone (a batch launched before it is full)
  static constexpr int kMaxBatch = 32;
  int batch = 1;
  int fill = 0;           // frames of the current slot's batch written, not launched
  hipGraph_t one_g[kSlots][kMaxBatch] = {};
  hipGraphExec_t one[kSlots][kMaxBatch] = {};
};

namespace {

void graph_free(tsdf_graph* g) {
  if (g->e && g->e->gbatch == g) g->e->gbatch = nullptr;
  for (int i = 0; i < tsdf_graph::kSlots; ++i) {
    for (int j = 0; j < tsdf_graph::kSegs; ++j) {
      if (g->exec[i][j]) (void)hipGraphExecDestroy(g->exec[i][j]);
      if (g->graph[i][j]) (void)hipGraphDestroy(g->graph[i][j]);
    }
    for (int j = 0; j < tsdf_graph::kMaxBatch; ++j) {
      if (g->one[i][j]) (void)hipGraphExecDestroy(g->one[i][j]);
      if (g->one_g[i][j]) (void)hipGraphDestroy(g->one_g[i][j]);
    }
    if (g->done[i]) (void)hipEventDestroy(g->done[i]);
  }
  if (g->d_args) (void)hipFree(g->d_args);
  if (g->h_args) (void)hipHostFree(g->h_args);
  if (g->cap) (void)hipStreamDestroy(g->cap);
  delete g;
}

}  // namespace

namespace {
int graph_create(tsdf_engine* e, int width, int height, int render_width, int render_height, bool defer,
                 tsdf_graph** out, int batch = 1) {
  if (e && e->cfg.shard_count > 1) {
    set_error("tsdf_graph_create: a shard's graph frames are tsdf_graph_create_shard / tsdf_graph_shard_*");
    return TSDF_ERR_INVALID_ARG;
  }
  if (!e || !out || width <= 0 || height <= 0 || width > e->cfg.max_width || height > e->cfg.max_height ||
      render_width < 0 || render_height < 0 || (int64_t)render_width * render_height > e->max_pixels ||
      (render_width == 0) != (render_height == 0) || batch < 1 || batch > tsdf_graph::kMaxBatch) {
    set_error("tsdf_graph_create: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  auto* g = new tsdf_graph();
  g->batch = batch;
  g->e = e;
  g->W = width;
  g->H = height;
  g->RW = render_width;
  g->RH = render_height;
  // frames without a render camera pipeline like tsdf_integrate; a render camera needs each frame
  // complete before its raycast, so those graphs keep the two-launch frame
  g->pipe = render_width == 0 && e->pipeline && e->maxs <= 3 && pipe_frame_size(e, width, height);
  g->defer = defer && render_width && e->maxs <= 3;  // (k_render_ingest_g is the 1024-slot ingest)
  auto fail = [&](hipError_t err, const char* what) {
    set_error(what, err);
    graph_free(g);
    return TSDF_ERR_HIP;
  };
  hipError_t err;
  if ((err = hipStreamCreateWithFlags(&g->cap, hipStreamNonBlocking)) != hipSuccess) return fail(err, "graph stream");
  const int nargs = tsdf_graph::kSlots * batch;
  if ((err = hipMalloc(&g->d_args, sizeof(FrameArgs) * nargs)) != hipSuccess) return fail(err, "graph args");
  if ((err = hipHostMalloc(&g->h_args, sizeof(FrameArgs) * nargs)) != hipSuccess)
    return fail(err, "graph host args");
  std::memset(g->h_args, 0, sizeof(FrameArgs) * nargs);
  const int tiles = ((width + 15) / 16) * ((height + 15) / 16);
  // the engine's queued work must be done before the capture stream records anything
  if ((err = hipStreamSynchronize(e->stream)) != hipSuccess) return fail(err, "graph sync");
  // the nodes of one frame (args entry A)
  auto frame_nodes = [&](const FrameArgs* A) {
    if (g->pipe) {  // one k_frame per frame, its grid sized for the largest launch (steady state)
      const int tpw = std::max(1, e->env.frame_tiles_per_wg);
      const int nwg = kPipeHead + kPipeFreshWG + e->D.integrate_grid_pre + (tiles + tpw - 1) / tpw + kVisWorkgroups;
      hipLaunchKernelGGL(k_frame_g, dim3(nwg), dim3(kIntegrateThreads), 0, g->cap, e->D, A);
    } else {
      const int rgx = (render_width + 15) / 16, nray = rgx * ((render_height + 15) / 16);
      if (g->defer)  // the previous frame's raycast (args->prev; none: its workgroups exit) + this ingest
        hipLaunchKernelGGL(k_render_ingest_g, dim3(nray + kVisWorkgroups + tiles), dim3(256), 0, g->cap, e->D,
                           A, rgx, nray);
      else if (e->maxs <= 3)
        hipLaunchKernelGGL(k_ingest_dda_g<1024>, dim3(kVisWorkgroups + tiles), dim3(256), 0, g->cap, e->D, A);
      else
        hipLaunchKernelGGL(k_ingest_dda_g<2048>, dim3(kVisWorkgroups + tiles), dim3(256), 0, g->cap, e->D, A);
      if (render_width && e->env.fuse_view_grid)  // the render camera's view grid built in the update launch
        hipLaunchKernelGGL(k_integrate_vg_g, dim3(e->D.integrate_grid + kOccWords / 256), dim3(kIntegrateThreads), 0,
                           g->cap, e->D, A, e->D.integrate_grid);
      else
        hipLaunchKernelGGL((k_integrate_t<true, false>), dim3(e->D.integrate_grid), dim3(kIntegrateThreads), 0,
                           g->cap, e->D, FrameParams{}, A);
    }
    if (render_width) {
      if (g->pipe || !e->env.fuse_view_grid)
        hipLaunchKernelGGL(k_view_grid_g, dim3(kOccWords / 256), dim3(256), 0, g->cap, e->D, A);
      hipLaunchKernelGGL(k_view_pack_g, dim3(kViewPackGrid), dim3(256), 0, g->cap, A);
      const dim3 rgrid((render_width + 15) / 16, (render_height + 15) / 16);
      if (!g->defer) hipLaunchKernelGGL(k_raycast_g, rgrid, dim3(256), 0, g->cap, e->D, A);
    }
  };
  // the args upload of entries [a0, a0 + n): one wave reads the pinned slots over the fabric (a kernel
  // node, no DMA engine in the graph), or a memcpy node (A/B)
  auto upload_node = [&](int a0, int n) {
    if (e->env.graph_memcpy_node)
      (void)hipMemcpyAsync(g->d_args + a0, g->h_args + a0, sizeof(FrameArgs) * n, hipMemcpyHostToDevice, g->cap);
    else
      hipLaunchKernelGGL(k_copy_words, dim3(1), dim3(n > 1 ? 256 : 64), 0, g->cap,
                         reinterpret_cast<uint32_t*>(g->d_args + a0), reinterpret_cast<const uint32_t*>(g->h_args + a0),
                         (int)(sizeof(FrameArgs) * n / 4));
  };
  auto capture = [&](hipGraph_t* gr, hipGraphExec_t* ex, int a0, int n) -> hipError_t {
    hipError_t er = hipStreamBeginCapture(g->cap, hipStreamCaptureModeThreadLocal);
    if (er != hipSuccess) return er;
    upload_node(a0, n);
    for (int j = 0; j < n; ++j) frame_nodes(g->d_args + a0 + j);
    if ((er = hipStreamEndCapture(g->cap, gr)) != hipSuccess) return er;
    return hipGraphInstantiate(ex, *gr, nullptr, nullptr, 0);
  };
  for (int k = 0; k < tsdf_graph::kSlots; ++k) {
    if ((err = hipEventCreateWithFlags(&g->done[k], kGraphDoneFlags)) != hipSuccess) return fail(err, "graph event");
    if ((err = capture(&g->graph[k][0], &g->exec[k][0], k * batch, batch)) != hipSuccess)
      return fail(err, "graph capture");
    for (int j = 0; batch > 1 && j < batch; ++j)  // (a batch launched before it is full)
      if ((err = capture(&g->one_g[k][j], &g->one[k][j], k * batch + j, 1)) != hipSuccess)
        return fail(err, "graph capture (single frame)");
  }
  *out = g;
  return TSDF_OK;
}

// launch the frames of g's current batch that were written but not launched (each alone)
int graph_flush_batch(tsdf_graph* g) {
  tsdf_engine* e = g->e;
  if (e->gbatch == g) e->gbatch = nullptr;
  if (g->fill == 0) return TSDF_OK;
  const int k = g->next, n = g->fill;
  g->fill = 0;
  g->next = (k + 1) % tsdf_graph::kSlots;
  for (int j = 0; j < n; ++j) HIP_OK(hipGraphLaunch(g->one[k][j], e->stream));
  HIP_OK(hipEventRecord(g->done[k], e->stream));
  g->used[k] = true;
  return TSDF_OK;
}
}  // namespace

int tsdf_graph_create(tsdf_engine* e, int width, int height, int render_width, int render_height,
                      tsdf_graph** out) {
  return graph_create(e, width, height, render_width, render_height, false, out);
}

int tsdf_graph_create_deferred(tsdf_engine* e, int width, int height, int render_width, int render_height,
                               tsdf_graph** out) {
  return graph_create(e, width, height, render_width, render_height, true, out);
}

int tsdf_graph_create_batch(tsdf_engine* e, int width, int height, int render_width, int render_height,
                            int deferred, int frames_per_launch, tsdf_graph** out) {
  return graph_create(e, width, height, render_width, render_height, deferred != 0, out, frames_per_launch);
}

// A shard's graph frame: three captured segments per args slot -- (0) the args upload + k_ingest_dda_g
// over the slice (its tail packs the slice's keys into keys_out; slice_count 1: it resolves them, no
// key exchange), (1) k_resolve_alloc_g merging the key inbox (split DDA only) + the raw-frame
// k_integrate (its tail packs the carve candidates into cands_out), (2) k_resolve_delete_g of the
// candidate inbox. The caller's exchanges (RCCL all-gathers on the engine stream) run between them:
// stream-ordered collectives of another library cannot be recorded into the engine's graphs.
int tsdf_graph_create_shard(tsdf_engine* e, int width, int height, int slice_index, int slice_count,
                            tsdf_graph** out) {
  if (!e || !out || e->cfg.shard_count < 2 || width <= 0 || height <= 0 || width > e->cfg.max_width ||
      height > e->cfg.max_height || slice_count < 1 || slice_index < 0 || slice_index >= slice_count) {
    set_error("tsdf_graph_create_shard: invalid argument (a shard engine; the slice of its DDA)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  auto* g = new tsdf_graph();
  g->e = e;
  g->W = width;
  g->H = height;
  g->shard = true;
  g->slice_index = slice_index;
  g->slice_count = slice_count;
  auto fail = [&](hipError_t err, const char* what) {
    set_error(what, err);
    graph_free(g);
    return TSDF_ERR_HIP;
  };
  hipError_t err;
  if ((err = hipStreamCreateWithFlags(&g->cap, hipStreamNonBlocking)) != hipSuccess) return fail(err, "graph stream");
  if ((err = hipMalloc(&g->d_args, sizeof(FrameArgs) * tsdf_graph::kSlots)) != hipSuccess) return fail(err, "graph args");
  if ((err = hipHostMalloc(&g->h_args, sizeof(FrameArgs) * tsdf_graph::kSlots)) != hipSuccess)
    return fail(err, "graph host args");
  std::memset(g->h_args, 0, sizeof(FrameArgs) * tsdf_graph::kSlots);
  const int tiles_x = (width + 15) / 16, tiles_y = (height + 15) / 16;
  const int rows = (tiles_y + slice_count - 1) / slice_count;
  const int tiles = (std::min(tiles_y, (slice_index + 1) * rows) - std::min(tiles_y, slice_index * rows)) * tiles_x;
  if ((err = hipStreamSynchronize(e->stream)) != hipSuccess) return fail(err, "graph sync");
  for (int k = 0; k < tsdf_graph::kSlots; ++k) {
    const FrameArgs* A = g->d_args + k;
    if ((err = hipEventCreateWithFlags(&g->done[k], kGraphDoneFlags)) != hipSuccess) return fail(err, "graph event");
    for (int seg = 0; seg < tsdf_graph::kSegs; ++seg) {
      if ((err = hipStreamBeginCapture(g->cap, hipStreamCaptureModeThreadLocal)) != hipSuccess)
        return fail(err, "hipStreamBeginCapture");
      if (seg == 0) {
        hipLaunchKernelGGL(k_copy_words, dim3(1), dim3(64), 0, g->cap, reinterpret_cast<uint32_t*>(g->d_args + k),
                           reinterpret_cast<const uint32_t*>(g->h_args + k), (int)(sizeof(FrameArgs) / 4));
        if (e->maxs <= 3)
          hipLaunchKernelGGL(k_ingest_dda_g<1024>, dim3(kVisWorkgroups + tiles), dim3(256), 0, g->cap, e->D, A);
        else
          hipLaunchKernelGGL(k_ingest_dda_g<2048>, dim3(kVisWorkgroups + tiles), dim3(256), 0, g->cap, e->D, A);
      } else if (seg == 1) {
        if (slice_count > 1)
          hipLaunchKernelGGL(k_resolve_alloc_g, dim3(1), dim3(kRT), 0, g->cap, e->D, A);
        hipLaunchKernelGGL((k_integrate_t<true, true>), dim3(e->D.integrate_grid), dim3(kIntegrateThreads), 0,
                           g->cap, e->D, FrameParams{}, A);
      } else {
        hipLaunchKernelGGL(k_resolve_delete_g, dim3(1), dim3(kRT), 0, g->cap, e->D, A);
      }
      if ((err = hipStreamEndCapture(g->cap, &g->graph[k][seg])) != hipSuccess) return fail(err, "hipStreamEndCapture");
      if ((err = hipGraphInstantiate(&g->exec[k][seg], g->graph[k][seg], nullptr, nullptr, 0)) != hipSuccess)
        return fail(err, "hipGraphInstantiate");
    }
  }
  *out = g;
  return TSDF_OK;
}

int tsdf_graph_shard_begin(tsdf_graph* g, const tsdf_frame* f, const tsdf_intrinsics* K, const tsdf_pose* pose,
                           float max_depth, void* keys_out, const void* keys_in, int32_t key_cap, void* cands_out,
                           const void* cands_in, int32_t cand_cap) {
  TraceRange trace_("tsdf_graph_shard_begin");
  const bool split = g && g->slice_count > 1;
  if (!g || !g->shard || !f || !K || !pose || f->mem_kind != TSDF_MEM_DEVICE || f->width != g->W ||
      f->height != g->H || !f->depth || !f->rgb || (f->ht == nullptr) != (f->lt == nullptr) || !cands_out ||
      !cands_in || cand_cap < 1 || (split && (!keys_out || !keys_in || key_cap < 1))) {
    set_error("tsdf_graph_shard_begin: invalid argument (a shard graph; device frame of its size; the key "
              "slot / inbox of a split DDA and the candidate slot / inbox)");
    return TSDF_ERR_INVALID_ARG;
  }
  tsdf_engine* e = g->e;
  if (e->shard_phase != 0) {
    set_error("tsdf_graph_shard_begin: a sharded frame is pending");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  const int k = g->next;
  g->next = (k + 1) % tsdf_graph::kSlots;
  if (g->used[k]) HIP_OK(hipEventSynchronize(g->done[k]));  // slot k's upload has run
  FrameArgs& a = g->h_args[k];
  a = FrameArgs{};
  a.P = make_params(e, K, f->width, f->height, pose, max_depth);
  FrameParams& P = a.P;
  P.depth = f->depth;
  P.rgb = f->rgb;
  P.ht = f->ht;
  P.lt = f->lt;
  P.pack_pixels = 0;  // a shard's k_integrate reads the raw frame
  const int tiles_x = (f->width + 15) / 16, tiles_y = (f->height + 15) / 16;
  const int rows = (tiles_y + g->slice_count - 1) / g->slice_count;
  P.tile_lo = std::min(tiles_y, g->slice_index * rows) * tiles_x;
  P.tile_hi = std::min(tiles_y, (g->slice_index + 1) * rows) * tiles_x;
  if (split) {
    P.tail = kTailPack;
    P.slot = reinterpret_cast<ShardRec*>(keys_out);
    P.slot_cap = key_cap;
  }
  a.depth = f->depth;
  a.rgb = f->rgb;
  a.ht = f->ht;
  a.lt = f->lt;
  a.range = (uint32_t)((size_t)f->width * f->height * e->maxs);
  a.tiles_x = tiles_x;
  a.tiles = P.tile_hi - P.tile_lo;
  a.keys_out = reinterpret_cast<ShardRec*>(keys_out);
  a.keys_in = reinterpret_cast<const ShardRec*>(keys_in);
  a.key_cap = key_cap;
  a.cands_out = reinterpret_cast<ShardRec*>(cands_out);
  a.cands_in = reinterpret_cast<const ShardRec*>(cands_in);
  a.cand_cap = cand_cap;
  a.nshard = e->cfg.shard_count;
  HIP_OK(hipGraphLaunch(g->exec[k][0], e->stream));
  // the host slot is read by segment 0's upload only (segments 1 and 2 read the device copy, which
  // only segment 0 of the slot's next use rewrites, after them on the stream)
  HIP_OK(hipEventRecord(g->done[k], e->stream));
  g->used[k] = true;
  g->cur = k;
  e->shard_phase = 1;
  return TSDF_OK;
}

int tsdf_graph_shard_update(tsdf_graph* g) {
  TraceRange trace_("tsdf_graph_shard_update");
  if (!g || !g->shard || g->cur < 0 || g->e->shard_phase != 1) {
    set_error("tsdf_graph_shard_update: no graph frame begun");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(g->e->device));
  HIP_OK(hipGraphLaunch(g->exec[g->cur][1], g->e->stream));
  g->e->shard_phase = 2;
  return TSDF_OK;
}

int tsdf_graph_shard_end(tsdf_graph* g) {
  TraceRange trace_("tsdf_graph_shard_end");
  if (!g || !g->shard || g->cur < 0 || g->e->shard_phase != 2) {
    set_error("tsdf_graph_shard_end: no graph frame updated");
    return TSDF_ERR_INVALID_ARG;
  }
  tsdf_engine* e = g->e;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  HIP_OK(hipGraphLaunch(g->exec[g->cur][2], e->stream));
  g->cur = -1;
  e->shard_phase = 0;
  return TSDF_OK;
}

int tsdf_graph_frame(tsdf_graph* g, const tsdf_frame* f, const tsdf_intrinsics* K, const tsdf_pose* pose,
                     float max_depth, const tsdf_intrinsics* render_K, const tsdf_pose* render_pose,
                     uint8_t* rgba, uint8_t* normal) {
  TraceRange trace_("tsdf_graph_frame");
  if (!g || g->shard || !f || !K || !pose || f->mem_kind != TSDF_MEM_DEVICE || f->width != g->W ||
      f->height != g->H || !f->depth || !f->rgb || (f->ht == nullptr) != (f->lt == nullptr) ||
      (g->RW && (!render_K || !render_pose))) {
    set_error("tsdf_graph_frame: invalid argument (device frame of the graph's size)");
    return TSDF_ERR_INVALID_ARG;
  }
  tsdf_engine* e = g->e;
  if (e->shard_phase != 0) {
    set_error("tsdf_graph_frame: a sharded frame is pending");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  // this graph's deferred raycast of the previous frame: rendered by this launch (k_render_ingest_g).
  // It stays pending (a later call launches it) until the graph launch below, so an error return on
  // the way leaves it to the engine's next call instead of dropping its images. (Batched
  // graphs: the previous frame may sit in this batch, not launched yet; nothing else ran since.)
  const FrameArgs* prev = (g->defer && e->rdg.pending && e->rdg.g == g) ? e->rdg.args : nullptr;
  if (g->fill == 0) {
    if (e->gbatch && e->gbatch != g) {
      int rc = graph_flush_batch(e->gbatch);
      if (rc) return rc;
    }
    int rc = join_render(e, false, true, prev != nullptr);  // (not the raycast this launch takes)
    if (!rc && !g->pipe) rc = flush_pending(e);  // (pipelined: the pending frames continue in this launch)
    if (rc) return rc;
  }
  const int k = g->next, j = g->fill;
  if (j == 0 && g->used[k]) HIP_OK(hipEventSynchronize(g->done[k]));  // slot k's last batch has run
  const int ai = k * g->batch + j;  // this frame's args entry
  FrameArgs& a = g->h_args[ai];
  a.P = make_params(e, K, f->width, f->height, pose, max_depth);
  if (g->RW) a.R = make_params(e, render_K, g->RW, g->RH, render_pose, max_depth);
  a.depth = f->depth;
  a.rgb = f->rgb;
  a.ht = f->ht;
  a.lt = f->lt;
  a.rgba = reinterpret_cast<uchar4*>(rgba);
  a.normal = reinterpret_cast<uchar4*>(normal);
  a.step_size = e->cfg.truncation / 2;
  if (g->RW) {
    if (g->fill > 0 && view_grid_resets(e, a.R, a.step_size, kViewGraphBitmapWords)) {
      // the batch's frames read the grid this call resets or reallocates: they run first, and this
      // frame opens the next batch (recomputed from the start)
      int rc = graph_flush_batch(g);
      if (rc) return rc;
      return tsdf_graph_frame(g, f, K, pose, max_depth, render_K, render_pose, rgba, normal);
    }
    if (prev && view_grid_resets(e, a.R, a.step_size, kViewGraphBitmapWords)) {  // (it reads the old grid)
      e->rdg.pending = false;
      hipLaunchKernelGGL(k_raycast_g, dim3((g->RW + 15) / 16, (g->RH + 15) / 16), dim3(256), 0, e->stream, e->D,
                         prev);
      LAUNCH_OK("k_raycast_g");
      prev = nullptr;
    }
    int rc = view_grid_for(e, a.R, a.step_size, kViewGraphBitmapWords, &a.V);
    if (rc) return rc;
    a.vtag = 0x80000000u | (uint32_t)(e->vg_calls & 0x7FFFFFFFu);  // (never a frame id)
  }
  a.prev = prev;
  a.range = (uint32_t)((size_t)f->width * f->height * e->maxs);
  a.tiles_x = (f->width + 15) / 16;
  a.tiles = a.tiles_x * ((f->height + 15) / 16);
  uint32_t fid = 0;
  if (g->pipe) {  // this frame's ingest + the pending frames' carving / allocation / update
    fid = next_fid(e);
    a.P.depth = f->depth;
    a.P.rgb = f->rgb;
    a.P.ht = f->ht;
    a.P.lt = f->lt;
    a.P.pix_off = (fid & 1u) ? (int)e->max_pixels : 0;
    a.Pu = e->p_P;
    a.pipe = pipe_step(e, true, fid, a.P);
    finish_args(e, a.pipe, a.Pu);
    if (e->profiling && a.pipe.has_update) ++e->prof_pipelined;
  }
  if (prev) e->rdg.pending = false;  // rendered by this launch
  g->fill = j + 1;
  e->gbatch = g;
  const bool hash_raycast = g->defer && !a.V.n;  // (no grid: it reads the table the next ingest writes)
  if (g->fill == g->batch) {  // the batch is full: one launch runs its frames
    e->gbatch = nullptr;
    g->fill = 0;
    g->next = (k + 1) % tsdf_graph::kSlots;
    HIP_OK(hipGraphLaunch(g->exec[k][0], e->stream));
    HIP_OK(hipEventRecord(g->done[k], e->stream));
    g->used[k] = true;
  } else if (hash_raycast) {  // it must run after this frame, before the next one's ingest
    int rc = graph_flush_batch(g);
    if (rc) return rc;
  }
  if (g->defer) {
    // a view grid's raycast waits for the next frame's launch; a hash-lookup raycast runs now, after
    // this frame's graph
    if (a.V.n) {
      e->rdg.pending = true;
      e->rdg.g = g;
      e->rdg.args = g->d_args + ai;
      e->rdg.W = g->RW;
      e->rdg.H = g->RH;
    } else {
      hipLaunchKernelGGL(k_raycast_g, dim3((g->RW + 15) / 16, (g->RH + 15) / 16), dim3(256), 0, e->stream, e->D,
                         g->d_args + ai);
      LAUNCH_OK("k_raycast_g");
    }
  }
  if (g->pipe) pipe_advance(e, fid, a.P);
  return TSDF_OK;
}

int tsdf_graph_destroy(tsdf_graph* g) {
  if (!g) return TSDF_ERR_INVALID_ARG;
  (void)hipSetDevice(g->e->device);
  (void)graph_flush_batch(g);
  (void)join_render(g->e);
  (void)hipStreamSynchronize(g->e->stream);
  graph_free(g);
  return TSDF_OK;
}

namespace {

// cv::resize x0.5 + convertTo + mask (k_rgbd_half) of a W x H frame into device rgb_out / depth_out
int rgbd_half(tsdf_engine* e, const uint8_t* rgb, const uint16_t* depth, const uint8_t* mask, int W,
              int H, float depth_factor, uint8_t* rgb_out, float* depth_out, int mem_kind) {
  hipStream_t s = e->stream;
  const size_t np = (size_t)W * H;
  if (mem_kind == TSDF_MEM_HOST) {
    if ((int64_t)np > e->fe_in_cap) {
      (void)hipFree(e->fe_rgb);
      (void)hipFree(e->fe_depth);
      (void)hipFree(e->fe_mask);
      e->fe_rgb = nullptr;
      e->fe_depth = nullptr;
      e->fe_mask = nullptr;
      e->fe_in_cap = 0;
      HIP_OK(dmalloc(&e->fe_rgb, np * 3));
      HIP_OK(dmalloc(&e->fe_depth, np));
      HIP_OK(dmalloc(&e->fe_mask, np));
      e->fe_in_cap = (int64_t)np;
    }
    HIP_OK(hipMemcpyAsync(e->fe_rgb, rgb, np * 3, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(e->fe_depth, depth, np * 2, hipMemcpyHostToDevice, s));
    if (mask) HIP_OK(hipMemcpyAsync(e->fe_mask, mask, np, hipMemcpyHostToDevice, s));
    rgb = e->fe_rgb;
    depth = e->fe_depth;
    mask = mask ? e->fe_mask : nullptr;
  }
  const float alpha = (float)(1. / (double)depth_factor);  // convertTo(CV_32FC1, 1. / factor)
  const int w = W / 2, h = H / 2;
  hipLaunchKernelGGL(k_rgbd_half, dim3((w + 63) / 64, (h + 3) / 4), dim3(256), 0, s, rgb, depth, mask,
                     W, H, alpha, rgb_out, depth_out);
  LAUNCH_OK("k_rgbd_half");
  return TSDF_OK;
}

bool rgbd_args_ok(const uint8_t* rgb, const uint16_t* depth, int W, int H, float depth_factor,
                  int mem_kind) {
  return rgb && depth && W >= 2 && H >= 2 && W % 2 == 0 && H % 2 == 0 && depth_factor > 0.0f &&
         (mem_kind == TSDF_MEM_HOST || mem_kind == TSDF_MEM_DEVICE);
}

int ensure_fe_out(tsdf_engine* e, int64_t npix) {
  if (npix <= e->fe_out_cap) return TSDF_OK;
  (void)hipFree(e->fe_out_rgb);
  (void)hipFree(e->fe_out_depth);
  e->fe_out_rgb = nullptr;
  e->fe_out_depth = nullptr;
  e->fe_out_cap = 0;
  HIP_OK(dmalloc(&e->fe_out_rgb, (size_t)npix * 3));
  HIP_OK(dmalloc(&e->fe_out_depth, (size_t)npix));
  e->fe_out_cap = npix;
  return TSDF_OK;
}

}  // namespace

int tsdf_rgbd_half(tsdf_engine* e, const uint8_t* rgb, const uint16_t* depth, const uint8_t* mask,
                   int width, int height, float depth_factor, uint8_t* rgb_out, float* depth_out,
                   int mem_kind) {
  if (!e || !rgbd_args_ok(rgb, depth, width, height, depth_factor, mem_kind) || !rgb_out || !depth_out) {
    set_error("tsdf_rgbd_half: invalid argument (even width / height, depth_factor > 0)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  JOIN_RENDER(e);
  const int64_t nout = (int64_t)(width / 2) * (height / 2);
  if (mem_kind == TSDF_MEM_DEVICE)
    return rgbd_half(e, rgb, depth, mask, width, height, depth_factor, rgb_out, depth_out, mem_kind);
  int rc = ensure_fe_out(e, nout);
  if (rc) return rc;
  rc = rgbd_half(e, rgb, depth, mask, width, height, depth_factor, e->fe_out_rgb, e->fe_out_depth, mem_kind);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(rgb_out, e->fe_out_rgb, (size_t)nout * 3, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(depth_out, e->fe_out_depth, (size_t)nout * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

int tsdf_feed_rgbd_frame(tsdf_engine* e, const uint8_t* rgb, const uint16_t* depth,
                         const uint8_t* mask, int width, int height, float depth_factor,
                         const tsdf_intrinsics* K, const tsdf_pose* cam_T_world, float max_depth,
                         int mem_kind) {
  TraceRange trace_("tsdf_feed_rgbd_frame");
  if (!e || !rgbd_args_ok(rgb, depth, width, height, depth_factor, mem_kind)) {
    set_error("tsdf_feed_rgbd_frame: invalid argument (even width / height, depth_factor > 0)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  JOIN_RENDER(e);
  const int w = width / 2, h = height / 2;
  int rc = ensure_fe_out(e, (int64_t)w * h);
  if (rc) return rc;
  rc = rgbd_half(e, rgb, depth, mask, width, height, depth_factor, e->fe_out_rgb, e->fe_out_depth, mem_kind);
  if (rc) return rc;
  // TSDFSystem::Integrate without ht / lt (disinfect_slam.cc:66; ones, tsdf_module.cc:29-33)
  tsdf_frame f{};
  f.width = w;
  f.height = h;
  f.rgb = e->fe_out_rgb;
  f.depth = e->fe_out_depth;
  f.ht = nullptr;
  f.lt = nullptr;
  f.mem_kind = TSDF_MEM_DEVICE;
  return tsdf_integrate(e, &f, K, cam_T_world, max_depth);
}


namespace {
int raycast_impl(tsdf_engine* e, const tsdf_intrinsics* K, int W, int H, const tsdf_pose* pose,
                 float max_depth, int row0, int nrows, uint8_t* rgba, uint8_t* normal, int mem_kind,
                 bool deferred = false) {
  if (!e || !K || !pose || W <= 0 || H <= 0 || (int64_t)W * H > e->max_pixels || row0 < 0 || nrows < 1 ||
      row0 + nrows > H || (mem_kind != TSDF_MEM_HOST && mem_kind != TSDF_MEM_DEVICE)) {
    set_error("tsdf_raycast: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  FrameParams P = make_params(e, K, W, H, pose, max_depth);
  P.row0 = row0;
  P.nrows = nrows;
  uchar4* o1 = mem_kind == TSDF_MEM_DEVICE ? reinterpret_cast<uchar4*>(rgba) : (rgba ? e->rc_rgba : nullptr);
  uchar4* o2 = mem_kind == TSDF_MEM_DEVICE ? reinterpret_cast<uchar4*>(normal) : (normal ? e->rc_norm : nullptr);
  const float step = e->cfg.truncation / 2;
  ViewGrid V;
  int rc;
  // The C5 loop (a deferred raycast while the frame's unpipelined update is still pending): that
  // update's launch builds the view grid too (k_integrate_vg), one launch and boundary fewer
  bool fused = false;
  if (deferred && mem_kind == TSDF_MEM_DEVICE && e->ps == tsdf_engine::kPipeU && !sharded(e) &&
      e->p_P.pack_pixels && e->env.fuse_view_grid) {
    JOIN_RENDER(e);  // (a deferred raycast still pending reads the previous grid)
    rc = view_grid_for(e, P, step, kViewGraphBitmapWords, &V);
    if (rc) return rc;
    if (V.n) {
      rc = update_with_grid(e, P, V);
      if (rc) return rc;
      fused = true;
    }
  }
  if (!fused) {
    ENTER(e);
    rc = view_grid_for(e, P, step, kViewBitmapWords, &V);
    if (rc) return rc;
    if (V.n) {
      hipLaunchKernelGGL(k_view_grid, dim3(kOccWords / 256), dim3(256), 0, e->stream, e->D, P, V);
      LAUNCH_OK("k_view_grid");
    }
  }
  if (V.n) {
    hipLaunchKernelGGL(k_view_pack, dim3(kViewPackGrid), dim3(256), 0, e->stream, V);
    LAUNCH_OK("k_view_pack");
  }
  if (deferred && V.n && V.nw <= kViewGraphBitmapWords && mem_kind == TSDF_MEM_DEVICE) {
    // (tsdf_raycast_deferred: the launch waits for the next call, join_render / frame_ingest)
    e->rd.pending = true;
    e->rd.P = P;
    e->rd.V = V;
    e->rd.step = step;
    e->rd.rgba = o1;
    e->rd.normal = o2;
    return TSDF_OK;
  }
  const size_t lds = V.n ? (size_t)V.nw * 4 : 0;
  // With a view grid the raycast reads only the pool, the grid and its bitmaps, none of which the
  // next frame's ingest writes: it runs on the render stream, overlapping that ingest (the next
  // update and every other call join it first). Without a grid it reads the hash table: engine stream.
  const bool overlap = e->render_overlap && V.n;
  hipStream_t rs = overlap ? e->rstream : e->stream;
  if (overlap) {
    HIP_OK(hipEventRecord(e->rs_ready, e->stream));
    HIP_OK(hipStreamWaitEvent(rs, e->rs_ready, 0));
  }
  const dim3 rgrid((W + 15) / 16, (nrows + 15) / 16);
  hipLaunchKernelGGL(k_raycast, rgrid, dim3(256), lds, rs, e->D, P, step, V, o1, o2);
  LAUNCH_OK("k_raycast");
  if (overlap) {
    HIP_OK(hipEventRecord(e->rs_done, rs));
    e->render_pending = true;
  }
  if (mem_kind == TSDF_MEM_HOST) {
    ENTER(e);
    const size_t bytes = (size_t)W * nrows * 4;
    if (rgba) HIP_OK(hipMemcpyAsync(rgba, e->rc_rgba, bytes, hipMemcpyDeviceToHost, e->stream));
    if (normal) HIP_OK(hipMemcpyAsync(normal, e->rc_norm, bytes, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
  }
  return TSDF_OK;
}
}  // namespace

int tsdf_raycast(tsdf_engine* e, const tsdf_intrinsics* K, int W, int H, const tsdf_pose* pose,
                 float max_depth, uint8_t* rgba, uint8_t* normal, int mem_kind) {
  TraceRange trace_("tsdf_raycast");
  return raycast_impl(e, K, W, H, pose, max_depth, 0, H, rgba, normal, mem_kind);
}

int tsdf_raycast_deferred(tsdf_engine* e, const tsdf_intrinsics* K, int W, int H, const tsdf_pose* pose,
                          float max_depth, uint8_t* rgba, uint8_t* normal) {
  TraceRange trace_("tsdf_raycast_deferred");
  return raycast_impl(e, K, W, H, pose, max_depth, 0, H, rgba, normal, TSDF_MEM_DEVICE, true);
}

int tsdf_raycast_rows(tsdf_engine* e, const tsdf_intrinsics* K, int W, int H, const tsdf_pose* pose,
                      float max_depth, int row0, int nrows, uint8_t* rgba, uint8_t* normal, int mem_kind) {
  TraceRange trace_("tsdf_raycast_rows");
  return raycast_impl(e, K, W, H, pose, max_depth, row0, nrows, rgba, normal, mem_kind);
}

int tsdf_query(tsdf_engine* e, const float* bounds, tsdf_voxel* out, int64_t capacity,
               int64_t* count) {
  TraceRange trace_("tsdf_query");
  if (!e || !count) return TSDF_ERR_INVALID_ARG;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  short4 lo = make_short4(0, 0, 0, 0), hi = make_short4(0, 0, 0, 0);
  if (bounds) {  // BoundingCube::Scale<short>(1. / voxel_size_) (voxel_tsdf.cuh:21-26, :429)
    const float scale = (float)(1. / (double)e->cfg.voxel_size);
    lo = make_short4(h_f2s(bounds[0] * scale), h_f2s(bounds[2] * scale), h_f2s(bounds[4] * scale), 0);
    hi = make_short4(h_f2s(bounds[1] * scale), h_f2s(bounds[3] * scale), h_f2s(bounds[5] * scale), 0);
  }
  hipStream_t s = e->stream;
  hipLaunchKernelGGL(k_query_count, dim3(kOccWords / 256), dim3(256), 0, s, e->D, bounds ? 1 : 0,
                     lo, hi);
  hipLaunchKernelGGL(k_vis_emit, dim3(kOccWords / 256), dim3(256), 0, s, e->D, e->q_sel,
                     e->q_count);
  LAUNCH_OK("query select");
  int32_t nsel = 0;
  HIP_OK(hipMemcpyAsync(&nsel, e->q_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  const int64_t nvox = (int64_t)nsel * kBlockVolume;
  *count = nvox;
  if (!out) return TSDF_OK;
  if (capacity < nvox) {
    set_error("tsdf_query: capacity too small");
    return TSDF_ERR_CAPACITY;
  }
  if (nsel == 0) return TSDF_OK;
  if (e->q_out_cap < nvox) {
    if (e->q_out) (void)hipFree(e->q_out);
    e->q_out = nullptr;
    HIP_OK(dmalloc(&e->q_out, (size_t)nvox));
    e->q_out_cap = nvox;
  }
  hipLaunchKernelGGL(k_query_download, dim3(nsel), dim3(kBlockVolume), 0, s, e->D, e->q_sel,
                     e->cfg.voxel_size, e->q_out);
  LAUNCH_OK("k_query_download");
  HIP_OK(hipMemcpyAsync(out, e->q_out, (size_t)nvox * sizeof(float4), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return TSDF_OK;
}

namespace {
// the nsel blocks listed in q_sel as TSDF_BLOCK_RECORD_BYTES records into out (host or device)
int pack_selected(tsdf_engine* e, int32_t nsel, void* out, int mem_kind, const char* what) {
  hipStream_t s = e->stream;
  const size_t bytes = (size_t)nsel * kBlockRecBytes;
  uint8_t* dst = reinterpret_cast<uint8_t*>(out);
  uint8_t* tmp = nullptr;
  if (mem_kind == TSDF_MEM_HOST) {
    HIP_OK(dmalloc(&tmp, bytes));
    dst = tmp;
  }
  hipLaunchKernelGGL(k_render_pack, dim3(nsel), dim3(256), 0, s, e->D, e->q_sel, dst);
  hipError_t err = hipGetLastError();
  if (err == hipSuccess && tmp) err = hipMemcpyAsync(out, tmp, bytes, hipMemcpyDeviceToHost, s);
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  if (tmp) (void)hipFree(tmp);
  if (err != hipSuccess) {
    set_error(what, err);
    return TSDF_ERR_HIP;
  }
  return TSDF_OK;
}
}  // namespace

static_assert(kBlockRecBytes == TSDF_BLOCK_RECORD_BYTES, "render record layout");

int tsdf_reset(tsdf_engine* e) {
  TraceRange trace_("tsdf_reset");
  if (!e) return TSDF_ERR_INVALID_ARG;
  if (e->shard_phase != 0) {
    set_error("tsdf_reset: a sharded frame is pending");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  // a shard's pending pipelined frames need the exchange protocol to complete: reset drops them
  // (init_state below re-initialises every per-frame buffer); one volume's are flushed first
  if (sharded(e)) e->ps = tsdf_engine::kPipeNone;
  ENTER(e);
  if (!init_state(e)) {
    set_error("tsdf_reset: initialisation failed");
    return TSDF_ERR_HIP;
  }
  return TSDF_OK;
}

namespace {
// the render cull of camera P (tsdf_render_blocks): the pixel-centre pyramid of rows [r0, r1) grown
// by one lookup's reach, cut at the marched length
RenderCull render_cull(const tsdf_engine* e, const FrameParams& P, int W, int r0, int r1) {
  // ray_cast_kernel's march (voxel_tsdf.cu:248-250): max_step samples truncation / 2 apart
  const double step = (double)(e->cfg.truncation / 2);
  const double max_step = std::ceil((double)P.max_depth / step);
  RenderCull C{};
  C.a0 = P.icx;
  C.a1 = (float)(W - 1) * P.ifx + P.icx;
  C.b0 = (float)r0 * P.ify + P.icy;  // the rays' own y / z slopes (pixel_ray's float operations)
  C.b1 = (float)(r1 - 1) * P.ify + P.icy;
  C.na0 = std::sqrt(1.0f + C.a0 * C.a0);
  C.na1 = std::sqrt(1.0f + C.a1 * C.a1);
  C.nb0 = std::sqrt(1.0f + C.b0 * C.b0);
  C.nb1 = std::sqrt(1.0f + C.b1 * C.b1);
  // bounding sphere of the voxel centres (3.5 sqrt 3 voxels) + nearest-voxel rounding (sqrt 3 / 2)
  // + the +-1 gradient neighbours = 7.93 voxels; 10 leaves room for float error
  C.reach = 10.0f * e->cfg.voxel_size;
  C.len = (float)(max_step * step) + C.reach;
  return C;
}

}  // namespace

int tsdf_render_blocks(tsdf_engine* e, const tsdf_intrinsics* K, int W, int H,
                       const tsdf_pose* pose, float max_depth, void* out, int64_t capacity,
                       int64_t* count, int mem_kind) {
  TraceRange trace_("tsdf_render_blocks");
  if (!e || !K || !pose || !count || W <= 0 || H <= 0 || !(max_depth > 0) ||
      (mem_kind != TSDF_MEM_HOST && mem_kind != TSDF_MEM_DEVICE)) {
    set_error("tsdf_render_blocks: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  const FrameParams P = make_params(e, K, W, H, pose, max_depth);
  const RenderCull C = render_cull(e, P, W, 0, H);
  hipStream_t s = e->stream;
  hipLaunchKernelGGL(k_render_count, dim3(kOccWords / 256), dim3(256), 0, s, e->D, P, C);
  hipLaunchKernelGGL(k_vis_emit, dim3(kOccWords / 256), dim3(256), 0, s, e->D, e->q_sel,
                     e->q_count);
  LAUNCH_OK("render select");
  int32_t nsel = 0;
  HIP_OK(hipMemcpyAsync(&nsel, e->q_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  *count = nsel;
  if (!out || nsel == 0) return TSDF_OK;
  if (capacity < nsel) {
    set_error("tsdf_render_blocks: capacity too small");
    return TSDF_ERR_CAPACITY;
  }
  return pack_selected(e, nsel, out, mem_kind, "tsdf_render_blocks");
}

namespace {
int ensure_groups(tsdf_engine* e, int n) {
  if (n <= e->g_cap) return TSDF_OK;
  (void)hipFree(e->g_visbits);
  (void)hipFree(e->g_wgcnt);
  (void)hipFree(e->g_sel);
  (void)hipFree(e->g_count);
  e->g_visbits = nullptr;
  e->g_wgcnt = nullptr;
  e->g_sel = nullptr;
  e->g_count = nullptr;
  e->g_cap = 0;
  HIP_OK(dmalloc(&e->g_visbits, (size_t)n * kOccWords));
  HIP_OK(dmalloc(&e->g_wgcnt, (size_t)n * (kOccWords / 256)));
  HIP_OK(dmalloc(&e->g_sel, (size_t)n * e->D.nblocks));
  HIP_OK(dmalloc(&e->g_count, (size_t)n));
  e->g_cap = n;
  return TSDF_OK;
}

// the groups of S: selection, per-group lists (entry order) and their counts (one host round trip);
// then, when out != NULL, the records group by group (TSDF_BLOCK_RECORD_BYTES each) into out
int group_records(tsdf_engine* e, const FrameParams& P, const GroupSel& S, void* out, int64_t capacity,
                  int64_t* counts, int mem_kind, const char* what) {
  int rc = ensure_groups(e, S.ngroups);
  if (rc) return rc;
  hipStream_t s = e->stream;
  hipLaunchKernelGGL(k_group_count, dim3(kOccWords / 256), dim3(256), 0, s, e->D, P, S, e->g_visbits,
                     e->g_wgcnt);
  for (int g = 0; g < S.ngroups; ++g) {
    EngineDev Dg = e->D;
    Dg.visbits = e->g_visbits + (size_t)g * kOccWords;
    Dg.wgcnt = e->g_wgcnt + (size_t)g * (kOccWords / 256);
    hipLaunchKernelGGL(k_vis_emit, dim3(kOccWords / 256), dim3(256), 0, s, Dg, e->g_sel + (size_t)g * e->D.nblocks,
                       e->g_count + g);
  }
  LAUNCH_OK(what);
  std::vector<int32_t> n(S.ngroups);
  HIP_OK(hipMemcpyAsync(n.data(), e->g_count, sizeof(int32_t) * S.ngroups, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  int64_t total = 0;
  for (int g = 0; g < S.ngroups; ++g) {
    counts[g] = n[g];
    total += n[g];
  }
  if (!out || total == 0) return TSDF_OK;
  if (capacity < total) {
    set_error("grouped block records: capacity too small");
    return TSDF_ERR_CAPACITY;
  }
  uint8_t* dst = reinterpret_cast<uint8_t*>(out);
  uint8_t* tmp = nullptr;
  if (mem_kind == TSDF_MEM_HOST) {
    HIP_OK(dmalloc(&tmp, (size_t)total * kBlockRecBytes));
    dst = tmp;
  }
  int64_t off = 0;
  for (int g = 0; g < S.ngroups; ++g) {
    if (n[g])
      hipLaunchKernelGGL(k_render_pack, dim3(n[g]), dim3(256), 0, s, e->D, e->g_sel + (size_t)g * e->D.nblocks,
                         dst + (size_t)off * kBlockRecBytes);
    off += n[g];
  }
  hipError_t err = hipGetLastError();
  if (err == hipSuccess && tmp) err = hipMemcpyAsync(out, tmp, (size_t)total * kBlockRecBytes, hipMemcpyDeviceToHost, s);
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  if (tmp) (void)hipFree(tmp);
  if (err != hipSuccess) {
    set_error(what, err);
    return TSDF_ERR_HIP;
  }
  return TSDF_OK;
}
}  // namespace

int tsdf_render_bands(tsdf_engine* e, const tsdf_intrinsics* K, int W, int H, const tsdf_pose* pose,
                      float max_depth, int nbands, const int32_t* rows, void* out, int64_t capacity,
                      int64_t* counts, int mem_kind) {
  TraceRange trace_("tsdf_render_bands");
  bool ok = e && K && pose && counts && rows && W > 0 && H > 0 && max_depth > 0 && nbands >= 1 &&
            nbands <= kMaxGroups && (mem_kind == TSDF_MEM_HOST || mem_kind == TSDF_MEM_DEVICE);
  for (int b = 0; ok && b < nbands; ++b) ok = rows[b] >= 0 && rows[b] < rows[b + 1] && rows[b + 1] <= H;
  if (!ok) {
    set_error("tsdf_render_bands: invalid argument (1..64 bands of increasing rows within the image)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  const FrameParams P = make_params(e, K, W, H, pose, max_depth);
  GroupSel S{};
  S.mode = kGroupBands;
  S.ngroups = nbands;
  S.cull = render_cull(e, P, W, 0, H);
  for (int b = 0; b < nbands; ++b) {
    const RenderCull C = render_cull(e, P, W, rows[b], rows[b + 1]);
    S.b0[b] = C.b0;
    S.b1[b] = C.b1;
    S.nb0[b] = C.nb0;
    S.nb1[b] = C.nb1;
  }
  return group_records(e, P, S, out, capacity, counts, mem_kind, "tsdf_render_bands");
}

int tsdf_pack_halo(tsdf_engine* e, void* out, int64_t capacity, int64_t* counts, int mem_kind) {
  TraceRange trace_("tsdf_pack_halo");
  if (!e || !counts || e->cfg.shard_count < 2 || (mem_kind != TSDF_MEM_HOST && mem_kind != TSDF_MEM_DEVICE)) {
    set_error("tsdf_pack_halo: invalid argument (a shard engine)");
    return TSDF_ERR_INVALID_ARG;
  }
  if (e->shard_phase != 0) {
    set_error("tsdf_pack_halo: a sharded frame is pending");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  FrameParams P{};
  P.shard_index = e->cfg.shard_index;
  P.shard_count = e->cfg.shard_count;
  GroupSel S{};
  S.mode = kGroupHalo;
  S.ngroups = e->cfg.shard_count;
  return group_records(e, P, S, out, capacity, counts, mem_kind, "tsdf_pack_halo");
}

int tsdf_pack_blocks(tsdf_engine* e, const float* bounds, void* out, int64_t capacity,
                     int64_t* count, int mem_kind) {
  TraceRange trace_("tsdf_pack_blocks");
  if (!e || !count || (mem_kind != TSDF_MEM_HOST && mem_kind != TSDF_MEM_DEVICE)) {
    set_error("tsdf_pack_blocks: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  short4 lo = make_short4(0, 0, 0, 0), hi = make_short4(0, 0, 0, 0);
  if (bounds) {  // the Query block selection (voxel_tsdf.cuh:21-26, voxel_tsdf.cu:429)
    const float scale = (float)(1. / (double)e->cfg.voxel_size);
    lo = make_short4(h_f2s(bounds[0] * scale), h_f2s(bounds[2] * scale), h_f2s(bounds[4] * scale), 0);
    hi = make_short4(h_f2s(bounds[1] * scale), h_f2s(bounds[3] * scale), h_f2s(bounds[5] * scale), 0);
  }
  hipStream_t s = e->stream;
  hipLaunchKernelGGL(k_query_count, dim3(kOccWords / 256), dim3(256), 0, s, e->D, bounds ? 1 : 0,
                     lo, hi);
  hipLaunchKernelGGL(k_vis_emit, dim3(kOccWords / 256), dim3(256), 0, s, e->D, e->q_sel,
                     e->q_count);
  LAUNCH_OK("pack select");
  int32_t nsel = 0;
  HIP_OK(hipMemcpyAsync(&nsel, e->q_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  *count = nsel;
  if (!out || nsel == 0) return TSDF_OK;
  if (capacity < nsel) {
    set_error("tsdf_pack_blocks: capacity too small");
    return TSDF_ERR_CAPACITY;
  }
  return pack_selected(e, nsel, out, mem_kind, "tsdf_pack_blocks");
}

int tsdf_import_blocks(tsdf_engine* e, const void* records, int64_t n, int mem_kind, int replace) {
  TraceRange trace_("tsdf_import_blocks");
  if (!e || n < 0 || (n > 0 && !records) ||
      (mem_kind != TSDF_MEM_HOST && mem_kind != TSDF_MEM_DEVICE)) {
    set_error("tsdf_import_blocks: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  if (e->shard_phase != 0) {
    set_error("tsdf_import_blocks: a sharded frame is pending");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  if (replace && !init_state(e, false)) {
    set_error("tsdf_import_blocks: clearing the volume failed");
    return TSDF_ERR_HIP;
  }
  if (n == 0) return TSDF_OK;
  hipStream_t s = e->stream;
  const size_t bytes = (size_t)n * kBlockRecBytes;
  const uint8_t* recs = reinterpret_cast<const uint8_t*>(records);
  uint8_t* tmp = nullptr;
  if (mem_kind == TSDF_MEM_HOST) {
    HIP_OK(dmalloc(&tmp, bytes));
    hipError_t err = hipMemcpyAsync(tmp, records, bytes, hipMemcpyHostToDevice, s);
    if (err != hipSuccess) {
      (void)hipFree(tmp);
      set_error("tsdf_import_blocks upload", err);
      return TSDF_ERR_HIP;
    }
    recs = tmp;
  }
  auto done = [&](int rc) {
    if (tmp) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(tmp);
    }
    return rc;
  };
  // VoxelHashTable::Allocate keeps <= 1 structural change per bucket per launch (voxel_hash.cu:
  // 80-118): resolver launches over the still-missing keys until every record has its block
  for (int64_t base = 0; base < n; base += kNewKeyCap) {
    const int m = (int)std::min<int64_t>(kNewKeyCap, n - base);
    const uint8_t* chunk = recs + (size_t)base * kBlockRecBytes;
    int32_t missing = m;
    for (int round = 0; missing > 0; ++round) {
      if (round == 64) {
        set_error("tsdf_import_blocks: keys still missing after 64 allocation launches");
        return done(TSDF_ERR_HIP);
      }
      hipLaunchKernelGGL(k_import_keys, dim3((m + 255) / 256), dim3(256), 0, s, e->D, chunk, m);
      if (hipGetLastError() != hipSuccess) return done(TSDF_ERR_HIP);
      int rc = launch_resolve_alloc(e, FrameParams{}, (uint32_t)m, 0);
      if (rc) return done(rc);
      // every record whose block exists gets its payload; the rest are counted (one round trip
      // for that count and the status word)
      if (hipMemsetAsync(e->q_count, 0, sizeof(int32_t), s) != hipSuccess) return done(TSDF_ERR_HIP);
      hipLaunchKernelGGL(k_import_payload, dim3((unsigned)m), dim3(256), 0, s, e->D, chunk, e->q_count);
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(e->h_ctr, e->D.ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipMemcpyAsync(&missing, e->q_count, sizeof(int32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return done(TSDF_ERR_HIP);
      if (missing > 0 && (e->h_ctr->status & TSDF_STATUS_POOL_EXHAUSTED)) {
        set_error("tsdf_import_blocks: voxel block pool exhausted");
        return done(TSDF_ERR_OUT_OF_MEMORY);
      }
    }
  }
  return done(TSDF_OK);
}

namespace {
int extract_mesh_impl(tsdf_engine* e, const float* bounds, float missing_tsdf, int min_weight, int own_index,
                      int own_count, float* triangles, int64_t capacity, int64_t* num_triangles, int mem_kind) {
  if (!e || !num_triangles || (mem_kind != TSDF_MEM_HOST && mem_kind != TSDF_MEM_DEVICE) || own_count < 1 ||
      own_count > kMaxShards || own_index < 0 || own_index >= own_count) {
    set_error("tsdf_extract_mesh: invalid argument");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  short4 lo = make_short4(0, 0, 0, 0), hi = make_short4(0, 0, 0, 0);
  if (bounds) {  // the Query block selection (voxel_tsdf.cuh:21-26, voxel_tsdf.cu:429)
    const float scale = (float)(1. / (double)e->cfg.voxel_size);
    lo = make_short4(h_f2s(bounds[0] * scale), h_f2s(bounds[2] * scale), h_f2s(bounds[4] * scale), 0);
    hi = make_short4(h_f2s(bounds[1] * scale), h_f2s(bounds[3] * scale), h_f2s(bounds[5] * scale), 0);
  }
  hipStream_t s = e->stream;
  hipLaunchKernelGGL(k_query_count, dim3(kOccWords / 256), dim3(256), 0, s, e->D, bounds ? 1 : 0,
                     lo, hi);
  hipLaunchKernelGGL(k_vis_emit, dim3(kOccWords / 256), dim3(256), 0, s, e->D, e->q_sel,
                     e->q_count);
  LAUNCH_OK("mesh select");
  // selection, count, scan and (device output) emission enqueued back to back: the kernels read
  // the selected-block count and the triangle total from device memory, and the host reads the
  // total once at the end (a host output needs it first, to size the staging buffer)
  const MeshParams M{e->cfg.voxel_size, missing_tsdf, min_weight, own_index, own_count};
  hipLaunchKernelGGL(k_mesh<false>, dim3(e->mesh_grid), dim3(256), 0, s, e->D, e->q_sel, e->q_count, M,
                     e->m_counts, (const int32_t*)nullptr, (const int64_t*)nullptr, (int64_t)0, e->m_nbr, (float*)nullptr);
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, e->m_counts, e->q_count, e->m_offsets,
                     e->m_total);
  LAUNCH_OK("mesh count");
  const bool dev_out = triangles && mem_kind == TSDF_MEM_DEVICE;
  if (dev_out) {
    hipLaunchKernelGGL(k_mesh<true>, dim3(e->mesh_grid), dim3(256), 0, s, e->D, e->q_sel, e->q_count, M,
                       e->m_counts, (const int32_t*)e->m_offsets, (const int64_t*)e->m_total, capacity, e->m_nbr,
                       reinterpret_cast<float*>(triangles));
    LAUNCH_OK("mesh emit");
  }
  int64_t ntri = 0;
  HIP_OK(hipMemcpyAsync(&ntri, e->m_total, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  *num_triangles = ntri;
  if (!triangles || ntri == 0) return TSDF_OK;
  if (capacity < ntri) {  // (device output: the emit pass wrote nothing)
    set_error("tsdf_extract_mesh: capacity too small");
    return TSDF_ERR_CAPACITY;
  }
  if (dev_out) return TSDF_OK;
  if (e->m_out_cap < ntri) {
    if (e->m_out) (void)hipFree(e->m_out);
    e->m_out = nullptr;
    e->m_out_cap = 0;
    HIP_OK(dmalloc(&e->m_out, (size_t)ntri * 9));
    e->m_out_cap = ntri;
  }
  hipLaunchKernelGGL(k_mesh<true>, dim3(e->mesh_grid), dim3(256), 0, s, e->D, e->q_sel, e->q_count, M,
                     e->m_counts, (const int32_t*)e->m_offsets, (const int64_t*)e->m_total, ntri, e->m_nbr, e->m_out);
  LAUNCH_OK("mesh emit");
  HIP_OK(hipMemcpyAsync(triangles, e->m_out, (size_t)ntri * 9 * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return TSDF_OK;
}
}  // namespace

int tsdf_extract_mesh(tsdf_engine* e, const float* bounds, float missing_tsdf, int min_weight,
                      float* triangles, int64_t capacity, int64_t* num_triangles, int mem_kind) {
  TraceRange trace_("tsdf_extract_mesh");
  return extract_mesh_impl(e, bounds, missing_tsdf, min_weight, 0, 1, triangles, capacity, num_triangles,
                           mem_kind);
}

int tsdf_extract_mesh_owned(tsdf_engine* e, const float* bounds, float missing_tsdf, int min_weight,
                            int shard_index, int shard_count, float* triangles, int64_t capacity,
                            int64_t* num_triangles, int mem_kind) {
  TraceRange trace_("tsdf_extract_mesh_owned");
  return extract_mesh_impl(e, bounds, missing_tsdf, min_weight, shard_index, shard_count, triangles, capacity,
                           num_triangles, mem_kind);
}

int tsdf_get_stats(tsdf_engine* e, tsdf_stats* o, int clear_status) {
  if (!e || !o) return TSDF_ERR_INVALID_ARG;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  int rc = read_counters(e);
  if (rc) return rc;
  const DevCounters& c = *e->h_ctr;
  std::memset(o, 0, sizeof(*o));
  o->frames = (int64_t)c.frames;
  o->free_blocks = c.free_count;
  o->active_blocks = e->D.nblocks - c.free_count;
  o->last_num_visible = c.n_vis;
  o->last_num_alloc = c.last_alloc;
  o->last_num_deleted = c.last_deleted;
  o->last_num_new_keys = c.last_new_keys;
  o->last_num_updated = (int64_t)c.last_updated;
  o->total_visible = (int64_t)c.total_visible;
  o->total_updated = (int64_t)c.total_updated;
  o->total_alloc = (int64_t)c.total_alloc;
  o->total_deleted = (int64_t)c.total_deleted;
  o->status = c.status;
  if (clear_status && c.status) {
    HIP_OK(hipMemsetAsync(&e->D.ctr->status, 0, sizeof(uint32_t), e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
  }
  return TSDF_OK;
}

int tsdf_profile_begin(tsdf_engine* e, int mode, int every) {
  if (!e || (mode != TSDF_PROFILE_PHASES && mode != TSDF_PROFILE_INTEGRATE &&
             mode != TSDF_PROFILE_KERNEL) || every < 1)
    return TSDF_ERR_INVALID_ARG;
  e->prof_mode = mode;
  e->prof_every = every;
  e->prof_calls = 0;
  e->prof_pipelined = 0;
  int rc = read_counters(e);
  if (rc) return rc;
  e->prof_vis0 = e->h_ctr->total_visible;
  e->prof_upd0 = e->h_ctr->total_updated;
  e->prof_ticks0 = e->h_ctr->integrate_ticks;
  e->prof_ing0 = e->h_ctr->ingest_ticks;
  e->prof_ra0 = e->h_ctr->resolve_alloc_ticks;
  e->prof_rd0 = e->h_ctr->resolve_delete_ticks;
  e->ev_used = 0;
  e->profiling = true;
  return TSDF_OK;
}

int tsdf_profile_end(tsdf_engine* e, tsdf_profile* o) {
  if (!e || !o) return TSDF_ERR_INVALID_ARG;
  e->profiling = false;
  int rc = read_counters(e);
  if (rc) return rc;
  std::memset(o, 0, sizeof(*o));
  o->frames = (int64_t)e->ev_used;
  o->calls = e->prof_calls;
  o->pipelined = e->prof_pipelined;
  for (size_t i = 0; i < e->ev_used; ++i) {
    float ms[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < 4; ++k)
      if (e->prof_mode == TSDF_PROFILE_PHASES || k == 2)
        HIP_OK(hipEventElapsedTime(&ms[k], e->events[i][k], e->events[i][k + 1]));
    o->ms_allocate += ms[0];
    o->ms_visible += ms[1];
    o->ms_integrate += ms[2];
    o->ms_carve += ms[3];
  }
  o->sum_visible = (int64_t)(e->h_ctr->total_visible - e->prof_vis0);
  o->sum_updated = (int64_t)(e->h_ctr->total_updated - e->prof_upd0);
  o->ms_integrate_device = (double)(e->h_ctr->integrate_ticks - e->prof_ticks0) * 1e-5;
  o->ms_ingest_device = (double)(e->h_ctr->ingest_ticks - e->prof_ing0) * 1e-5;
  o->ms_resolve_alloc_device = (double)(e->h_ctr->resolve_alloc_ticks - e->prof_ra0) * 1e-5;
  o->ms_resolve_delete_device = (double)(e->h_ctr->resolve_delete_ticks - e->prof_rd0) * 1e-5;
  return TSDF_OK;
}

int tsdf_debug_stamps(tsdf_engine* e, uint64_t* out, int64_t capacity, int* enabled) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  HIP_OK(hipSetDevice(e->device));
  // (no flush of pending pipelined frames: the stamps are those of the launches so far)
#ifdef TSDF_DIAG_STAMPS
  if (enabled) *enabled = 1;
#else
  if (enabled) *enabled = 0;
#endif
  const int64_t n = (int64_t)kDiagKernels * kDiagMaxWg * kDiagStamps;
  if (!out) return TSDF_OK;
  if (capacity < n) {
    set_error("tsdf_debug_stamps: capacity too small");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  HIP_OK(hipMemcpy(out, e->D.dbg, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemset(e->D.dbg, 0, n * sizeof(uint64_t)));
  return TSDF_OK;
}

// ---------------------------------------------------------------------------------------------
// Snapshot / restore (SURVEY.md 5 checkpoint / resume; the reference only dumps GatherValid to a
// file, examples/tsdf/offline.cc:181-187). The whole engine state between frames -- hash table,
// occupancy bitmap, free-block stack, voxel pool (free blocks included: a re-acquired block keeps
// its old colour, voxel_mem.cu:43-51) and counters -- so a restored engine continues a stream bit
// for bit. Layout: header | counters | table | occ | heap | pool.
// ---------------------------------------------------------------------------------------------
namespace {
struct SnapshotHeader {
  char magic[8];  // "TSDFSNAP"
  uint32_t version;
  int32_t nblocks;
  float voxel, truncation;
  int64_t bytes;
  int32_t shard_index, shard_count;
};
constexpr uint32_t kSnapshotVersion = 2;

// A snapshot is accepted only if the state it describes is one the engine could have reached: the
// free stack and the table's pool indices partition the pool, foreign entries only on a shard,
// the occupancy bits are exactly the entries with voxels here, and every bucket's list ends. A
// corrupt or hand-edited one would otherwise send the next frame's kernels out of bounds.
bool snapshot_consistent(const tsdf_engine* e, const uint8_t* p) {
  const int nb = e->D.nblocks;
  DevCounters c;
  std::memcpy(&c, p, sizeof(c));
  p += sizeof(DevCounters);
  const int4* table = reinterpret_cast<const int4*>(p);
  p += (size_t)kNumEntry * 16;
  const uint64_t* occ = reinterpret_cast<const uint64_t*>(p);
  p += (size_t)kOccWords * 8;
  const int32_t* heap = reinterpret_cast<const int32_t*>(p);
  if (c.free_count < 0 || c.free_count > nb) return false;
  std::vector<uint8_t> seen((size_t)nb, 0);
  for (int i = 0; i < c.free_count; ++i) {
    const int32_t b = heap[i];
    if (b < 0 || b >= nb || seen[b]) return false;
    seen[b] = 1;
  }
  int64_t occupied = 0, held = 0;
  for (uint32_t en = 0; en < kNumEntry; ++en) {
    const int32_t idx = table[en].z;
    const bool bit = (occ[en >> 6] >> (en & 63)) & 1ull;
    if (idx == -1) {
      if (bit) return false;
      continue;
    }
    ++occupied;
    if (idx == kForeignIdx) {
      if (e->cfg.shard_count <= 1 || bit) return false;
      continue;
    }
    if (idx < 0 || idx >= nb || seen[idx] || !bit) return false;
    seen[idx] = 1;
    ++held;
  }
  if (held + c.free_count != nb) return false;
  // bucket lists (slot 1's offset chain) end within the occupied entries
  for (uint32_t b = 0; b < kNumBucket; ++b) {
    uint32_t last = 2 * b + 1;
    int16_t off = (int16_t)((uint32_t)table[last].y >> 16);
    for (int64_t steps = 0; off; ++steps) {
      if (steps > occupied) return false;
      last = (uint32_t)(last + (int32_t)off) & kEntryMask;
      off = (int16_t)((uint32_t)table[last].y >> 16);
    }
  }
  return true;
}

int64_t snapshot_bytes(const tsdf_engine* e) {
  return (int64_t)sizeof(SnapshotHeader) + (int64_t)sizeof(DevCounters) + (int64_t)kNumEntry * 16 +
         (int64_t)kOccWords * 8 + (int64_t)e->D.nblocks * 4 + (int64_t)e->D.nblocks * kBlockBytes;
}
}  // namespace

int tsdf_snapshot_bytes(tsdf_engine* e, int64_t* bytes) {
  if (!e || !bytes) return TSDF_ERR_INVALID_ARG;
  *bytes = snapshot_bytes(e);
  return TSDF_OK;
}

int tsdf_snapshot_save(tsdf_engine* e, void* out, int64_t capacity) {
  TraceRange trace_("tsdf_snapshot_save");
  if (!e || !out) return TSDF_ERR_INVALID_ARG;
  if (e->shard_phase != 0) {
    set_error("tsdf_snapshot_save: a sharded frame is pending");
    return TSDF_ERR_INVALID_ARG;
  }
  const int64_t need = snapshot_bytes(e);
  if (capacity < need) {
    set_error("tsdf_snapshot_save: buffer smaller than tsdf_snapshot_bytes");
    return TSDF_ERR_CAPACITY;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  hipStream_t s = e->stream;
  uint8_t* p = static_cast<uint8_t*>(out);
  SnapshotHeader h{};
  std::memcpy(h.magic, "TSDFSNAP", 8);
  h.version = kSnapshotVersion;
  h.nblocks = e->D.nblocks;
  h.voxel = e->cfg.voxel_size;
  h.truncation = e->cfg.truncation;
  h.bytes = need;
  h.shard_index = e->cfg.shard_index;
  h.shard_count = e->cfg.shard_count;
  std::memcpy(p, &h, sizeof(h));
  p += sizeof(h);
  HIP_OK(hipMemcpyAsync(p, e->D.ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, s));
  p += sizeof(DevCounters);
  HIP_OK(hipMemcpyAsync(p, e->D.table, (size_t)kNumEntry * 16, hipMemcpyDeviceToHost, s));
  p += (size_t)kNumEntry * 16;
  HIP_OK(hipMemcpyAsync(p, e->D.occ, (size_t)kOccWords * 8, hipMemcpyDeviceToHost, s));
  p += (size_t)kOccWords * 8;
  HIP_OK(hipMemcpyAsync(p, e->D.heap, (size_t)e->D.nblocks * 4, hipMemcpyDeviceToHost, s));
  p += (size_t)e->D.nblocks * 4;
  HIP_OK(hipMemcpyAsync(p, e->D.pool, (size_t)e->D.nblocks * kBlockBytes, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return TSDF_OK;
}

int tsdf_snapshot_load(tsdf_engine* e, const void* in, int64_t size) {
  TraceRange trace_("tsdf_snapshot_load");
  if (!e || !in || size < (int64_t)sizeof(SnapshotHeader)) return TSDF_ERR_INVALID_ARG;
  SnapshotHeader h;
  std::memcpy(&h, in, sizeof(h));
  if (std::memcmp(h.magic, "TSDFSNAP", 8) != 0 || h.version != kSnapshotVersion || h.nblocks != e->D.nblocks ||
      h.voxel != e->cfg.voxel_size || h.truncation != e->cfg.truncation || h.bytes != snapshot_bytes(e) ||
      size < h.bytes || h.shard_index != e->cfg.shard_index || h.shard_count != e->cfg.shard_count ||
      e->shard_phase != 0) {
    set_error("tsdf_snapshot_load: not a snapshot of an engine with this configuration");
    return TSDF_ERR_INVALID_ARG;
  }
  if (!snapshot_consistent(e, static_cast<const uint8_t*>(in) + sizeof(h))) {
    set_error("tsdf_snapshot_load: inconsistent snapshot (pool indices, free stack, occupancy or "
              "bucket lists)");
    return TSDF_ERR_INVALID_ARG;
  }
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  hipStream_t s = e->stream;
  const uint8_t* p = static_cast<const uint8_t*>(in) + sizeof(h);
  HIP_OK(hipMemcpyAsync(e->D.ctr, p, sizeof(DevCounters), hipMemcpyHostToDevice, s));
  p += sizeof(DevCounters);
  HIP_OK(hipMemcpyAsync(e->D.table, p, (size_t)kNumEntry * 16, hipMemcpyHostToDevice, s));
  p += (size_t)kNumEntry * 16;
  HIP_OK(hipMemcpyAsync(e->D.occ, p, (size_t)kOccWords * 8, hipMemcpyHostToDevice, s));
  p += (size_t)kOccWords * 8;
  HIP_OK(hipMemcpyAsync(e->D.heap, p, (size_t)e->D.nblocks * 4, hipMemcpyHostToDevice, s));
  p += (size_t)e->D.nblocks * 4;
  HIP_OK(hipMemcpyAsync(e->D.pool, p, (size_t)e->D.nblocks * kBlockBytes, hipMemcpyHostToDevice, s));
  // lock words hold older epochs than the restored counter's (launches lock with epoch + 1)
  HIP_OK(hipMemsetAsync(e->D.lock_tag, 0, sizeof(uint32_t) * kNumBucket, s));
  HIP_OK(hipStreamSynchronize(s));
  return TSDF_OK;
}

int tsdf_debug_dump(tsdf_engine* e, int16_t* pos_off, int32_t* idx, int32_t* heap,
                    int32_t* free_count, float* tsdf_out, float* prob, uint8_t* rgbw) {
  if (!e) return TSDF_ERR_INVALID_ARG;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  hipStream_t s = e->stream;
  if (pos_off || idx) {
    short4* dpos = nullptr;
    int32_t* didx = nullptr;
    HIP_OK(dmalloc(&dpos, kNumEntry));
    HIP_OK(dmalloc(&didx, kNumEntry));
    hipLaunchKernelGGL(k_dump_table, dim3(kNumEntry / 256), dim3(256), 0, s, e->D, dpos, didx);
    hipError_t err = hipGetLastError();
    if (err == hipSuccess && pos_off)
      err = hipMemcpyAsync(pos_off, dpos, sizeof(short4) * kNumEntry, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess && idx)
      err = hipMemcpyAsync(idx, didx, sizeof(int32_t) * kNumEntry, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    (void)hipFree(dpos);
    (void)hipFree(didx);
    if (err != hipSuccess) {
      set_error("tsdf_debug_dump table", err);
      return TSDF_ERR_HIP;
    }
  }
  if (heap)
    HIP_OK(hipMemcpyAsync(heap, e->D.heap, sizeof(int32_t) * e->D.nblocks, hipMemcpyDeviceToHost, s));
  if (free_count) {
    int rc = read_counters(e);
    if (rc) return rc;
    *free_count = e->h_ctr->free_count;
  }
  if (tsdf_out || prob || rgbw) {
    const size_t nv = (size_t)e->D.nblocks * kBlockVolume;
    float* dt = nullptr;
    float* dp = nullptr;
    uint32_t* dc = nullptr;
    HIP_OK(dmalloc(&dt, nv));
    HIP_OK(dmalloc(&dp, nv));
    HIP_OK(dmalloc(&dc, nv));
    hipLaunchKernelGGL(k_dump_pool, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, e->D, dt,
                       dp, dc);
    hipError_t err = hipGetLastError();
    if (err == hipSuccess && tsdf_out) err = hipMemcpyAsync(tsdf_out, dt, nv * 4, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess && prob) err = hipMemcpyAsync(prob, dp, nv * 4, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess && rgbw) err = hipMemcpyAsync(rgbw, dc, nv * 4, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    (void)hipFree(dt);
    (void)hipFree(dp);
    (void)hipFree(dc);
    if (err != hipSuccess) {
      set_error("tsdf_debug_dump pool", err);
      return TSDF_ERR_HIP;
    }
  }
  HIP_OK(hipStreamSynchronize(s));
  return TSDF_OK;
}

int tsdf_hash_allocate(tsdf_engine* e, const int16_t* keys, int n) {
  if (!e || n < 0 || (n > 0 && !keys) || n > (int)kNewKeyCap) return TSDF_ERR_INVALID_ARG;
  if (n == 0) return TSDF_OK;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  int rc = ensure_test_cap(e, n);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(e->t_keys, keys, sizeof(int16_t) * 3 * n, hipMemcpyHostToDevice, e->stream));
  hipLaunchKernelGGL(k_keys_to_newset, dim3((n + 255) / 256), dim3(256), 0, e->stream, e->D,
                     e->t_keys, n);
  LAUNCH_OK("k_keys_to_newset");
  rc = launch_resolve_alloc(e, FrameParams{}, (uint32_t)n, 0);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

int tsdf_hash_delete(tsdf_engine* e, const int16_t* keys, int n) {
  if (!e || n < 0 || (n > 0 && !keys)) return TSDF_ERR_INVALID_ARG;
  if (n == 0) return TSDF_OK;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  int rc = ensure_test_cap(e, n);
  if (rc) return rc;
  std::vector<VisRec> recs(n);
  for (int i = 0; i < n; ++i) {
    recs[i].x = keys[3 * i];
    recs[i].y = keys[3 * i + 1];
    recs[i].z = keys[3 * i + 2];
    recs[i].pad = 0;
    recs[i].idx = -1;
    recs[i].entry = -1;
  }
  HIP_OK(hipMemcpyAsync(e->t_recs, recs.data(), sizeof(VisRec) * n, hipMemcpyHostToDevice, e->stream));
  HIP_OK(hipMemcpyAsync(e->t_count, &n, sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  hipLaunchKernelGGL(k_resolve_delete, dim3(1), dim3(kRT), 0, e->stream, e->D, (const VisRec*)e->t_recs,
                     (const int32_t*)e->t_count, 1, (const ShardRec*)nullptr, 0, 0);
  LAUNCH_OK("k_resolve_delete");
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

int tsdf_hash_retrieve(tsdf_engine* e, const int16_t* pts, int n, uint8_t* rgbw, float* tsdf_out,
                       float* prob, int16_t* bpo, int32_t* bidx) {
  if (!e || n < 0 || (n > 0 && !pts)) return TSDF_ERR_INVALID_ARG;
  if (n == 0) return TSDF_OK;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  int rc = ensure_test_cap(e, n);
  if (rc) return rc;
  hipStream_t s = e->stream;
  HIP_OK(hipMemcpyAsync(e->t_keys, pts, sizeof(int16_t) * 3 * n, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_hash_retrieve, dim3((n + 255) / 256), dim3(256), 0, s, e->D, e->t_keys, n,
                     e->t_u32, e->t_f0, e->t_f1, e->t_s4, e->t_i32);
  LAUNCH_OK("k_hash_retrieve");
  if (rgbw) HIP_OK(hipMemcpyAsync(rgbw, e->t_u32, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  if (tsdf_out) HIP_OK(hipMemcpyAsync(tsdf_out, e->t_f0, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  if (prob) HIP_OK(hipMemcpyAsync(prob, e->t_f1, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  if (bpo) HIP_OK(hipMemcpyAsync(bpo, e->t_s4, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
  if (bidx) HIP_OK(hipMemcpyAsync(bidx, e->t_i32, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return TSDF_OK;
}

int tsdf_hash_assign(tsdf_engine* e, const int16_t* pts, int n, const uint8_t* rgbw, int* missing) {
  if (!e || n < 0 || (n > 0 && (!pts || !rgbw))) return TSDF_ERR_INVALID_ARG;
  if (missing) *missing = 0;
  if (n == 0) return TSDF_OK;
  HIP_OK(hipSetDevice(e->device));
  ENTER(e);
  int rc = ensure_test_cap(e, n);
  if (rc) return rc;
  hipStream_t s = e->stream;
  HIP_OK(hipMemcpyAsync(e->t_keys, pts, sizeof(int16_t) * 3 * n, hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(e->t_u32, rgbw, 4 * (size_t)n, hipMemcpyHostToDevice, s));
  HIP_OK(hipMemsetAsync(e->t_count, 0, sizeof(int32_t), s));
  hipLaunchKernelGGL(k_hash_assign, dim3((n + 255) / 256), dim3(256), 0, s, e->D, e->t_keys, n,
                     e->t_u32, e->t_count);
  LAUNCH_OK("k_hash_assign");
  int m = 0;
  HIP_OK(hipMemcpyAsync(&m, e->t_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (missing) *missing = m;
  return TSDF_OK;
}

int tsdf_num_active_blocks(tsdf_engine* e, int32_t* out) {
  if (!e || !out) return TSDF_ERR_INVALID_ARG;
  int rc = read_counters(e);
  if (rc) return rc;
  *out = e->D.nblocks - e->h_ctr->free_count;
  return TSDF_OK;
}

int tsdf_pool_acquire(tsdf_engine* e, int n, int32_t* idx_out) {
  if (!e || n < 0 || (n > 0 && !idx_out)) return TSDF_ERR_INVALID_ARG;
  ENTER(e);
  if (n == 0) return TSDF_OK;
  int rc = ensure_test_cap(e, n);
  if (rc) return rc;
  hipLaunchKernelGGL(k_pool_acquire, dim3(1), dim3(64), 0, e->stream, e->D, n, e->t_i32);
  LAUNCH_OK("k_pool_acquire");
  HIP_OK(hipMemcpyAsync(idx_out, e->t_i32, 4 * (size_t)n, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

int tsdf_pool_release(tsdf_engine* e, const int32_t* idx, int n) {
  if (!e || n < 0 || (n > 0 && !idx)) return TSDF_ERR_INVALID_ARG;
  ENTER(e);
  if (n == 0) return TSDF_OK;
  int rc = ensure_test_cap(e, n);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(e->t_i32, idx, 4 * (size_t)n, hipMemcpyHostToDevice, e->stream));
  hipLaunchKernelGGL(k_pool_release, dim3(1), dim3(64), 0, e->stream, e->D, e->t_i32, n);
  LAUNCH_OK("k_pool_release");
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

int tsdf_pool_set_weight(tsdf_engine* e, int32_t block, uint8_t w) {
  if (!e || block < 0 || block >= e->D.nblocks) return TSDF_ERR_INVALID_ARG;
  ENTER(e);
  hipLaunchKernelGGL(k_pool_weight, dim3(1), dim3(kBlockVolume), 0, e->stream, e->D, block, 1, w,
                     (uint8_t*)nullptr);
  LAUNCH_OK("k_pool_weight");
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

int tsdf_pool_get_weights(tsdf_engine* e, int32_t block, uint8_t* out) {
  if (!e || !out || block < 0 || block >= e->D.nblocks) return TSDF_ERR_INVALID_ARG;
  ENTER(e);
  int rc = ensure_test_cap(e, kBlockVolume);
  if (rc) return rc;
  uint8_t* d = reinterpret_cast<uint8_t*>(e->t_u32);
  hipLaunchKernelGGL(k_pool_weight, dim3(1), dim3(kBlockVolume), 0, e->stream, e->D, block, 0,
                     (uint8_t)0, d);
  LAUNCH_OK("k_pool_weight");
  HIP_OK(hipMemcpyAsync(out, d, kBlockVolume, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return TSDF_OK;
}

}  // extern "C"
