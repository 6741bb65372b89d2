// tsdf_group.hip -- one spatially sharded volume owned by the library (tsdf_group_*; SURVEY.md 8b's
// tsdf_create_sharded, 8e). No reference counterpart: TSDFGrid (utils/tsdf/voxel_tsdf.cu:309-375) is
// single-GPU. The C++ callers of the reference interface (TSDFSystem, modules/tsdf_module.h:35-107;
// DISINFSystem, disinfect_slam/disinfect_slam.cc:13-17) reach a sharded volume through this layer
// (host/voxel_tsdf.h, host/tsdf_module.h) without Python or a collective library.
//
// A group holds n shard engines (shard i on devices[i]; a device may repeat) and runs the pipelined
// sharded frames of tsdf_integrate_shard_pipe with the candidate exchange inside the library: each
// shard's update kernel writes its carve-candidate slot straight into every shard's inbox (device
// stores; peer stores over xGMI between GPUs -- tsdf_integrate_shard_pipe_fanout), so nothing runs
// between the launches. Inboxes are double-buffered by call parity: call c writes parity c & 1 and
// reads what call c - 1 wrote. Ordering: the shards of one device run in one group stream, in shard
// order, so call c of every shard there follows call c - 1 of all of them (the reads after the
// writes and the next writes after the reads); across devices each device's stream waits, before
// call c, for the event every other device recorded after call c - 1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "disinfect_tsdf.h"
#include "tsdf_device.h"
#include "tsdf_internal.h"

using tsdf::ShardRec;

namespace {

constexpr int32_t kGroupCandCap = 16384;  // carve candidates (+ pool-exhausted entries) per shard and frame

int hip_fail(const char* what, hipError_t e) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  tsdf_set_last_error(buf);
  return TSDF_ERR_HIP;
}
#define GHIP(expr)                                \
  do {                                            \
    hipError_t _e = (expr);                       \
    if (_e != hipSuccess) return hip_fail(#expr, _e); \
  } while (0)
#define GRC(expr)            \
  do {                       \
    int _rc = (expr);        \
    if (_rc) return _rc;     \
  } while (0)

int invalid(const char* what) {
  tsdf_set_last_error(what);
  return TSDF_ERR_INVALID_ARG;
}

}  // namespace

struct tsdf_group {
  int n = 0;
  tsdf_config cfg{};
  std::vector<tsdf_engine*> shard;
  std::vector<int> udev;                 // the distinct devices, in order of first use
  std::vector<int> slot;                 // shard -> index in udev
  std::vector<hipStream_t> stream;       // per distinct device: the stream of its shards
  std::vector<hipEvent_t> ev;            // per distinct device: recorded after its shards' call
  std::vector<hipEvent_t> sig;           // per distinct device: tsdf_group_stream_signal's marker
  bool ev_valid = false;
  int32_t cap = kGroupCandCap;
  std::vector<ShardRec*> inbox[2];       // per shard, on its device: n slots of cap + 1 records
  std::vector<void**> dst_dev[2];        // per shard: device array of its slot in every inbox
  std::vector<std::vector<void*>> dst_host[2];
  int64_t calls = 0;
  bool pending = false;                  // frames in the pipeline (tsdf_group_flush completes them)
  std::vector<uint8_t*> stage;           // per distinct device: rgb | depth | ht | lt of one frame
  size_t stage_bytes = 0;
  tsdf_engine* replica = nullptr;        // raycast: the view's blocks of every shard (created on demand)
  std::vector<void*> rec;                // per shard: its render records (on its device)
  std::vector<int64_t> rec_cap;
  void* rec_all = nullptr;               // every shard's records, on udev[0]
  int64_t rec_all_cap = 0;
};

namespace {

void free_group(tsdf_group* g) {
  for (tsdf_engine* e : g->shard)
    if (e) (void)tsdf_destroy(e);
  if (g->replica) (void)tsdf_destroy(g->replica);
  for (int p = 0; p < 2; ++p) {
    for (ShardRec* b : g->inbox[p])
      if (b) (void)hipFree(b);
    for (void** b : g->dst_dev[p])
      if (b) (void)hipFree(b);
  }
  for (uint8_t* b : g->stage)
    if (b) (void)hipFree(b);
  for (void* b : g->rec)
    if (b) (void)hipFree(b);
  if (g->rec_all) (void)hipFree(g->rec_all);
  for (hipEvent_t e : g->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : g->sig)
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t s : g->stream)
    if (s) (void)hipStreamDestroy(s);
  delete g;
}

// one call of every shard (frames[u]: the frame staged on distinct device u, or NULL: a flush step)
int group_call(tsdf_group* g, const std::vector<tsdf_frame>* frames, const tsdf_intrinsics* K,
               const tsdf_pose* pose, float max_depth, int32_t* pending) {
  if (g->n == 1) {  // one shard is one volume: the plain pipelined frames, nothing to exchange
    g->calls += 1;
    if (pending) *pending = 0;
    return frames ? tsdf_integrate(g->shard[0], &(*frames)[0], K, pose, max_depth) : tsdf_flush(g->shard[0]);
  }
  const int par = (int)(g->calls & 1), prv = par ^ 1;
  const int nu = (int)g->udev.size();
  if (nu > 1 && g->ev_valid) {
    for (int u = 0; u < nu; ++u) {
      GHIP(hipSetDevice(g->udev[u]));
      for (int v = 0; v < nu; ++v)
        if (v != u) GHIP(hipStreamWaitEvent(g->stream[u], g->ev[v], 0));
    }
  }
  int32_t pend0 = 0;
  for (int s = 0; s < g->n; ++s) {
    int32_t pend = 0;
    const tsdf_frame* f = frames ? &(*frames)[g->slot[s]] : nullptr;
    GRC(tsdf_integrate_shard_pipe_fanout(g->shard[s], f, K, pose, max_depth, g->inbox[prv][s], g->dst_dev[par][s],
                                         g->dst_host[par][s].data(), g->n, g->cap, &pend));
    if (s == 0) pend0 = pend;
  }
  if (nu > 1) {
    for (int u = 0; u < nu; ++u) {
      GHIP(hipSetDevice(g->udev[u]));
      GHIP(hipEventRecord(g->ev[u], g->stream[u]));
    }
    g->ev_valid = true;
  }
  g->calls += 1;
  if (pending) *pending = pend0;
  return TSDF_OK;
}

int group_flush(tsdf_group* g) {
  if (!g->pending) return TSDF_OK;
  int32_t pend = 1;
  for (int guard = 0; pend && guard < 8; ++guard) GRC(group_call(g, nullptr, nullptr, nullptr, 0.0f, &pend));
  g->pending = false;
  return pend ? invalid("tsdf_group_flush: the pipeline did not drain") : TSDF_OK;
}

}  // namespace

extern "C" {

int tsdf_group_create(const tsdf_config* cfg_in, const int* devices, int n, tsdf_group** out) {
  if (!cfg_in || !devices || !out || n < 1 || n > 64) return invalid("tsdf_group_create: invalid argument");
  *out = nullptr;
  tsdf_group* g = new tsdf_group;
  g->n = n;
  g->cfg = *cfg_in;
  for (int i = 0; i < n; ++i) {
    auto it = std::find(g->udev.begin(), g->udev.end(), devices[i]);
    if (it == g->udev.end()) {
      g->slot.push_back((int)g->udev.size());
      g->udev.push_back(devices[i]);
    } else {
      g->slot.push_back((int)(it - g->udev.begin()));
    }
  }
  auto fail = [&](int rc) {
    free_group(g);
    return rc;
  };
  const int nu = (int)g->udev.size();
  g->stream.assign(nu, nullptr);
  g->ev.assign(nu, nullptr);
  g->sig.assign(nu, nullptr);
  for (int u = 0; u < nu; ++u) {
    hipError_t e = hipSetDevice(g->udev[u]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream[u], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&g->ev[u], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&g->sig[u], hipEventDisableTiming);
    for (int v = 0; v < nu && e == hipSuccess; ++v) {  // peer stores into the other devices' inboxes
      if (v == u) continue;
      e = hipDeviceEnablePeerAccess(g->udev[v], 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        e = hipSuccess;
      }
    }
    if (e != hipSuccess) return fail(hip_fail("tsdf_group_create: device / stream / peer access", e));
  }
  g->shard.assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    tsdf_config c = g->cfg;
    c.shard_index = n > 1 ? i : 0;
    c.shard_count = n;
    c.stream = g->stream[g->slot[i]];
    c.use_stream = 1;
    const int rc = tsdf_create(&c, devices[i], &g->shard[i]);
    if (rc) return fail(rc);
  }
  // inboxes (two parities) on each shard's device, and each shard's destination table: its slot in
  // every inbox
  const size_t slot_recs = (size_t)g->cap + 1;
  for (int p = 0; p < 2; ++p) {
    g->inbox[p].assign(n, nullptr);
    g->dst_dev[p].assign(n, nullptr);
    g->dst_host[p].assign(n, std::vector<void*>(n, nullptr));
    for (int i = 0; i < n; ++i) {
      hipError_t e = hipSetDevice(devices[i]);
      if (e == hipSuccess) e = hipMalloc(&g->inbox[p][i], (size_t)n * slot_recs * sizeof(ShardRec));
      if (e == hipSuccess) e = hipMemset(g->inbox[p][i], 0, (size_t)n * slot_recs * sizeof(ShardRec));
      if (e != hipSuccess) return fail(hip_fail("tsdf_group_create: inbox", e));
    }
    for (int s = 0; s < n; ++s) {
      for (int d = 0; d < n; ++d) g->dst_host[p][s][d] = g->inbox[p][d] + (size_t)s * slot_recs;
      hipError_t e = hipSetDevice(devices[s]);
      if (e == hipSuccess) e = hipMalloc(&g->dst_dev[p][s], (size_t)n * sizeof(void*));
      if (e == hipSuccess)
        e = hipMemcpy(g->dst_dev[p][s], g->dst_host[p][s].data(), (size_t)n * sizeof(void*), hipMemcpyHostToDevice);
      if (e != hipSuccess) return fail(hip_fail("tsdf_group_create: destination table", e));
    }
  }
  // frame staging per distinct device
  const size_t px = (size_t)g->cfg.max_width * g->cfg.max_height;
  g->stage_bytes = px * (3 + 4 + 4 + 4) + 256;
  g->stage.assign(nu, nullptr);
  for (int u = 0; u < nu; ++u) {
    hipError_t e = hipSetDevice(g->udev[u]);
    if (e == hipSuccess) e = hipMalloc(&g->stage[u], g->stage_bytes);
    if (e != hipSuccess) return fail(hip_fail("tsdf_group_create: frame staging", e));
  }
  g->rec.assign(n, nullptr);
  g->rec_cap.assign(n, 0);
  *out = g;
  return TSDF_OK;
}

int tsdf_group_destroy(tsdf_group* g) {
  if (!g) return TSDF_ERR_INVALID_ARG;
  for (size_t u = 0; u < g->udev.size(); ++u) {
    (void)hipSetDevice(g->udev[u]);
    (void)hipStreamSynchronize(g->stream[u]);
  }
  free_group(g);
  return TSDF_OK;
}

int tsdf_group_size(const tsdf_group* g) { return g ? g->n : 0; }

int tsdf_group_integrate(tsdf_group* g, const tsdf_frame* f, const tsdf_intrinsics* K, const tsdf_pose* pose,
                         float max_depth) {
  if (!g || !f || !K || !pose || !f->depth || !f->rgb || (f->ht == nullptr) != (f->lt == nullptr) ||
      f->width < 1 || f->height < 1 || f->width > g->cfg.max_width || f->height > g->cfg.max_height ||
      (f->mem_kind != TSDF_MEM_HOST && f->mem_kind != TSDF_MEM_DEVICE))
    return invalid("tsdf_group_integrate: invalid argument (a frame no larger than the group's maximum)");
  const int nu = (int)g->udev.size();
  const size_t px = (size_t)f->width * f->height;
  std::vector<tsdf_frame> frames(nu);
  for (int u = 0; u < nu; ++u) {
    tsdf_frame& d = frames[u];
    d = *f;
    if (f->mem_kind == TSDF_MEM_DEVICE && u == 0) continue;  // (a device frame lives on the first device)
    // stage: one copy per device, shared by its shards (a host frame, or a device frame's peer copy)
    uint8_t* base = g->stage[u];
    uint8_t* rgb = base;
    float* depth = reinterpret_cast<float*>(base + ((px * 3 + 255) & ~(size_t)255));
    float* ht = depth + px;
    float* lt = ht + px;
    GHIP(hipSetDevice(g->udev[u]));
    hipStream_t s = g->stream[u];
    if (f->mem_kind == TSDF_MEM_HOST) {
      GHIP(hipMemcpyAsync(rgb, f->rgb, px * 3, hipMemcpyHostToDevice, s));
      GHIP(hipMemcpyAsync(depth, f->depth, px * 4, hipMemcpyHostToDevice, s));
      if (f->ht) {
        GHIP(hipMemcpyAsync(ht, f->ht, px * 4, hipMemcpyHostToDevice, s));
        GHIP(hipMemcpyAsync(lt, f->lt, px * 4, hipMemcpyHostToDevice, s));
      }
    } else {
      const int src = g->udev[0];
      GHIP(hipMemcpyPeerAsync(rgb, g->udev[u], f->rgb, src, px * 3, s));
      GHIP(hipMemcpyPeerAsync(depth, g->udev[u], f->depth, src, px * 4, s));
      if (f->ht) {
        GHIP(hipMemcpyPeerAsync(ht, g->udev[u], f->ht, src, px * 4, s));
        GHIP(hipMemcpyPeerAsync(lt, g->udev[u], f->lt, src, px * 4, s));
      }
    }
    d.rgb = rgb;
    d.depth = depth;
    d.ht = f->ht ? ht : nullptr;
    d.lt = f->lt ? lt : nullptr;
    d.mem_kind = TSDF_MEM_DEVICE;
  }
  if (f->mem_kind == TSDF_MEM_HOST) {  // (the caller may reuse its buffers once this returns)
    for (int u = 0; u < nu; ++u) {
      GHIP(hipSetDevice(g->udev[u]));
      GHIP(hipStreamSynchronize(g->stream[u]));
    }
  }
  int32_t pend = 0;
  GRC(group_call(g, &frames, K, pose, max_depth, &pend));
  g->pending = true;
  return TSDF_OK;
}

int tsdf_group_flush(tsdf_group* g) {
  if (!g) return TSDF_ERR_INVALID_ARG;
  return group_flush(g);
}

int tsdf_group_synchronize(tsdf_group* g) {
  if (!g) return TSDF_ERR_INVALID_ARG;
  GRC(group_flush(g));
  for (int s = 0; s < g->n; ++s) GRC(tsdf_synchronize(g->shard[s]));
  return TSDF_OK;
}

int tsdf_group_shard(tsdf_group* g, int index, tsdf_engine** out) {
  if (!g || !out || index < 0 || index >= g->n) return TSDF_ERR_INVALID_ARG;
  GRC(group_flush(g));
  *out = g->shard[index];
  return TSDF_OK;
}

int tsdf_group_get_stats(tsdf_group* g, tsdf_stats* out, int clear_status) {
  if (!g || !out) return TSDF_ERR_INVALID_ARG;
  GRC(group_flush(g));
  tsdf_stats t{};
  for (int s = 0; s < g->n; ++s) {
    tsdf_stats a{};
    GRC(tsdf_get_stats(g->shard[s], &a, clear_status));
    if (s == 0) {  // every shard runs the same frames and finds the same new keys (the index is each one's)
      t.frames = a.frames;
      t.last_num_new_keys = a.last_num_new_keys;
    }
    // the voxels and pool blocks are divided: each shard counts the blocks it holds, acquires and
    // releases, and the visible / updated ones among them
    t.active_blocks += a.active_blocks;
    t.free_blocks += a.free_blocks;
    t.last_num_alloc += a.last_num_alloc;
    t.last_num_deleted += a.last_num_deleted;
    t.total_alloc += a.total_alloc;
    t.total_deleted += a.total_deleted;
    t.last_num_visible += a.last_num_visible;
    t.last_num_updated += a.last_num_updated;
    t.total_visible += a.total_visible;
    t.total_updated += a.total_updated;
    t.status |= a.status;
  }
  *out = t;
  return TSDF_OK;
}

int tsdf_group_query(tsdf_group* g, const float* bounds, tsdf_voxel* out, int64_t capacity, int64_t* count) {
  if (!g || !count) return TSDF_ERR_INVALID_ARG;
  GRC(group_flush(g));
  int64_t total = 0;
  std::vector<int64_t> cnt(g->n, 0);
  for (int s = 0; s < g->n; ++s) {
    GRC(tsdf_query(g->shard[s], bounds, nullptr, 0, &cnt[s]));
    total += cnt[s];
  }
  *count = total;
  if (!out) return TSDF_OK;
  if (capacity < total) return TSDF_ERR_CAPACITY;
  int64_t off = 0;
  for (int s = 0; s < g->n; ++s) {
    int64_t c = 0;
    GRC(tsdf_query(g->shard[s], bounds, out + off, capacity - off, &c));
    off += c;
  }
  return TSDF_OK;
}

int tsdf_group_stream_signal(tsdf_group* g, void* stream) {
  if (!g) return TSDF_ERR_INVALID_ARG;
  const int nu = (int)g->udev.size();
  for (int u = 0; u < nu; ++u) {
    GHIP(hipSetDevice(g->udev[u]));
    GHIP(hipEventRecord(g->sig[u], g->stream[u]));
  }
  GHIP(hipSetDevice(g->udev[0]));
  for (int u = 0; u < nu; ++u) GHIP(hipStreamWaitEvent(static_cast<hipStream_t>(stream), g->sig[u], 0));
  return TSDF_OK;
}

int tsdf_group_raycast(tsdf_group* g, const tsdf_intrinsics* K, int width, int height, const tsdf_pose* pose,
                       float max_depth, uint8_t* rgba, uint8_t* normal, int mem_kind) {
  if (!g || !K || !pose || width < 1 || height < 1 || width > g->cfg.max_width || height > g->cfg.max_height)
    return invalid("tsdf_group_raycast: invalid argument");
  GRC(group_flush(g));
  if (g->n == 1) return tsdf_raycast(g->shard[0], K, width, height, pose, max_depth, rgba, normal, mem_kind);
  // every shard's blocks the view can read (render replicas, tsdf_render_blocks) into one replica
  // engine on the first device, which raycasts exactly what the unsharded volume renders
  int64_t total = 0;
  std::vector<int64_t> cnt(g->n, 0);
  for (int s = 0; s < g->n; ++s) {
    GRC(tsdf_render_blocks(g->shard[s], K, width, height, pose, max_depth, nullptr, 0, &cnt[s], TSDF_MEM_DEVICE));
    total += cnt[s];
  }
  const int d0 = g->udev[0];
  if (!g->replica) {
    tsdf_config c = g->cfg;
    c.shard_index = 0;
    c.shard_count = 1;
    c.stream = g->stream[0];
    c.use_stream = 1;
    GRC(tsdf_create(&c, d0, &g->replica));
  }
  if (total > g->rec_all_cap) {
    GHIP(hipSetDevice(d0));
    if (g->rec_all) GHIP(hipFree(g->rec_all));
    g->rec_all = nullptr;
    g->rec_all_cap = 0;
    GHIP(hipMalloc(&g->rec_all, (size_t)std::max<int64_t>(total, 1) * TSDF_BLOCK_RECORD_BYTES));
    g->rec_all_cap = total;
  }
  int64_t off = 0;
  for (int s = 0; s < g->n; ++s) {
    if (!cnt[s]) continue;
    const int dev = g->udev[g->slot[s]];
    uint8_t* dst = static_cast<uint8_t*>(g->rec_all) + (size_t)off * TSDF_BLOCK_RECORD_BYTES;
    int64_t c = 0;
    if (dev == d0) {  // straight into the gathered buffer
      GRC(tsdf_render_blocks(g->shard[s], K, width, height, pose, max_depth, dst, cnt[s], &c, TSDF_MEM_DEVICE));
    } else {
      if (cnt[s] > g->rec_cap[s]) {
        GHIP(hipSetDevice(dev));
        if (g->rec[s]) GHIP(hipFree(g->rec[s]));
        g->rec[s] = nullptr;
        GHIP(hipMalloc(&g->rec[s], (size_t)cnt[s] * TSDF_BLOCK_RECORD_BYTES));
        g->rec_cap[s] = cnt[s];
      }
      GRC(tsdf_render_blocks(g->shard[s], K, width, height, pose, max_depth, g->rec[s], cnt[s], &c, TSDF_MEM_DEVICE));
      GRC(tsdf_synchronize(g->shard[s]));
      GHIP(hipSetDevice(d0));
      GHIP(hipMemcpyPeerAsync(dst, d0, g->rec[s], dev, (size_t)c * TSDF_BLOCK_RECORD_BYTES, g->stream[0]));
    }
    off += c;
  }
  for (int s = 0; s < g->n; ++s) GRC(tsdf_synchronize(g->shard[s]));
  GRC(tsdf_import_blocks(g->replica, g->rec_all, off, TSDF_MEM_DEVICE, 1));
  return tsdf_raycast(g->replica, K, width, height, pose, max_depth, rgba, normal, mem_kind);
}

}  // extern "C"
