/*
 * tsdf_oracle.c -- CPU restatement of yuzhou42/disinfect-slam's CUDA TSDF engine.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + bench cpu_baseline). See tsdf_oracle.h for the
 * pinning status. Every function cites the reference file:line it restates. Eigen 3.3 expression
 * evaluation orders are reproduced explicitly:
 *   - fixed-size 3-vector sum / dot / squaredNorm: a0 + (a1 + a2)  (redux_novec_unroller split)
 *   - q * v  : uv = 2 (q.vec x v); v + w uv + q.vec x uv           (QuaternionBase::_transformVector)
 *   - host q.inverse(): n2 = (x^2 + z^2) + (y^2 + w^2)               (SSE/NEON predux of a Vector4f)
 * Compile with -ffp-contract=off so no multiply-add is fused.
 */
#include "tsdf_oracle.h"


#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- constants: voxel_mem.cuh:10-20, voxel_hash.cuh:12-25 ---- */
#define BLOCK_LEN_BITS 3
#define BLOCK_LEN 8
#define BLOCK_AREA 64
#define BLOCK_VOLUME 512
#define BLOCK_VOLUME_BITS 9
#define NUM_BUCKET_BITS 21
#define NUM_BUCKET (1 << NUM_BUCKET_BITS)
#define BUCKET_MASK (NUM_BUCKET - 1)
#define NUM_ENTRY_PER_BUCKET 2
#define NUM_ENTRY (1 << (NUM_BUCKET_BITS + 1))
#define ENTRY_MASK (NUM_ENTRY - 1)
#define ENTRY_PER_BUCKET_MASK 1

typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } quat;
typedef struct { quat q; v3 t; } se3;
typedef struct { float fx, fy, cx, cy; } intr;
typedef struct { int16_t x, y, z; } s3;

/* voxel_mem.cuh:73-93 VoxelBlock */
typedef struct { s3 pos; int16_t offset; int32_t idx; } entry;

struct ora_grid {
  float voxel, trunc;
  int nb_bits, nblocks;
  entry* table;
  uint8_t* locks;
  int32_t* heap;
  int32_t free_count;
  float* tsdf;     /* voxels_tsdf_  */
  float* prob;     /* voxels_segm_  */
  uint8_t* rgbw;   /* voxels_rgbw_ (r,g,b,weight) */
  float* range;    /* img_depth_to_range_ */
  int range_cap;
  int32_t* vis;    /* visible_blocks_ entry indices (entry order) */
  ora_stats st;
  int shard_index, shard_count; /* spatial sharding (not in the reference) */
  /* a shard's entries of owned keys its exhausted pool could not give voxels this frame: carved in
   * the same frame (appended to its candidates), so no voxel-less owned entry outlives the frame */
  s3* pend_pos;
  int32_t* pend_entry;
  int64_t n_pend, pend_cap;
};

/* ---------------- float math (utils/cuda/camera.cuh, lie_group.cuh, Eigen 3.3) ------------- */
static v3 v3_cross(v3 a, v3 b) { /* Eigen MatrixBase::cross (OrthoMethods.h) */
  v3 r;
  r.x = a.y * b.z - a.z * b.y;
  r.y = a.z * b.x - a.x * b.z;
  r.z = a.x * b.y - a.y * b.x;
  return r;
}
static float v3_dot(v3 a, v3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
static float v3_norm(v3 a) { return sqrtf(v3_dot(a, a)); }

/* Eigen QuaternionBase::_transformVector (used by lie_group.cuh:30 R_ * vec3) */
static v3 qrot(quat q, v3 v) {
  v3 qv = {q.x, q.y, q.z};
  v3 uv = v3_cross(qv, v);
  uv.x += uv.x; uv.y += uv.y; uv.z += uv.z;
  v3 c = v3_cross(qv, uv);
  v3 r;
  r.x = (v.x + q.w * uv.x) + c.x;
  r.y = (v.y + q.w * uv.y) + c.y;
  r.z = (v.z + q.w * uv.z) + c.z;
  return r;
}
/* lie_group.cuh:30-32 SE3::Apply = R * v + t */
static v3 se3_apply(const se3* T, v3 v) {
  v3 r = qrot(T->q, v);
  r.x = r.x + T->t.x; r.y = r.y + T->t.y; r.z = r.z + T->t.z;
  return r;
}
/* lie_group.cuh:22-24 SE3::Inverse = (R^-1, R^-1 * (-t)), evaluated on the host (voxel_tsdf.cu:382,497).
 * Eigen QuaternionBase::inverse(): conj(q).coeffs() / squaredNorm(); host squaredNorm of the 4
 * coefficients is a Packet4f reduction: (x*x + z*z) + (y*y + w*w). */
static se3 se3_inverse(const se3* T) {
  const quat q = T->q;
  const float n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
  se3 r;
  if (n2 > 0.0f) {
    r.q.x = -q.x / n2; r.q.y = -q.y / n2; r.q.z = -q.z / n2; r.q.w = q.w / n2;
  } else {
    r.q.x = r.q.y = r.q.z = r.q.w = 0.0f;
  }
  v3 nt = {-T->t.x, -T->t.y, -T->t.z};
  r.t = qrot(r.q, nt);
  return r;
}
/* camera.cuh:34-39 CameraIntrinsics::Inverse */
static intr intr_inverse(intr k) {
  intr r;
  r.fx = 1.0f / k.fx;
  r.fy = 1.0f / k.fy;
  r.cx = -k.cx * r.fx;
  r.cy = -k.cy * r.fy;
  return r;
}
/* camera.cuh:47-51 CameraIntrinsics::operator* */
static v3 intr_mul(intr k, v3 v) {
  v3 r;
  r.x = k.fx * v.x + k.cx * v.z;
  r.y = k.fy * v.y + k.cy * v.z;
  r.z = v.z;
  return r;
}

/* float -> integer conversions with GPU (cvt.rzi / v_cvt_i32_f32) semantics: truncate toward
 * zero, saturate, NaN -> 0. Makes the oracle deterministic where C leaves it undefined. */
static int32_t f2i(float f) {
  if (f != f) return 0;
  if (f >= 2147483648.0f) return INT32_MAX;
  if (f <= -2147483648.0f) return INT32_MIN;
  return (int32_t)f;
}
static int16_t f2s(float f) {
  if (f != f) return 0;
  if (f >= 32767.0f) return 32767;
  if (f <= -32768.0f) return -32768;
  return (int16_t)f;
}
static uint8_t f2u8(float f) {
  if (!(f > 0.0f)) return 0; /* NaN and negatives */
  if (f >= 255.0f) return 255;
  return (uint8_t)f;
}

/* ---------------- hash table (voxel_hash.cu) ---------------- */
uint32_t ora_hash(int16_t x, int16_t y, int16_t z) { /* voxel_hash.cu:31-35 */
  return (((uint32_t)(int32_t)x * 73856093u) ^ ((uint32_t)(int32_t)y * 19349669u) ^
          ((uint32_t)(int32_t)z * 83492791u)) & BUCKET_MASK;
}
static int s3_eq(s3 a, s3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static s3 point_to_block(s3 p) { /* voxel_mem.cuh:29-32 (arithmetic shift) */
  s3 r = {(int16_t)(p.x >> BLOCK_LEN_BITS), (int16_t)(p.y >> BLOCK_LEN_BITS),
          (int16_t)(p.z >> BLOCK_LEN_BITS)};
  return r;
}
static s3 block_to_point(s3 b) { /* voxel_mem.cuh:41-44 */
  s3 r = {(int16_t)(b.x << BLOCK_LEN_BITS), (int16_t)(b.y << BLOCK_LEN_BITS),
          (int16_t)(b.z << BLOCK_LEN_BITS)};
  return r;
}
static int offset_to_index(int ox, int oy, int oz) { return ox + oy * BLOCK_LEN + oz * BLOCK_AREA; }

/* voxel_mem.cu:37-52 AquireBlock (weight 0, tsdf -1, prob 0.5). The reference leaves rgb as it
 * is: uninitialised cudaMalloc memory for a never-used block, the previous occupant's colour for a
 * re-used one -- which occupant depends on the racy pool order. That colour is
 * only observable on weight-0 voxels (an update multiplies it by w_old = 0), so it is unspecified
 * in the reference; here and in the engine it is defined as 0, which keeps a sharded volume (other
 * pool indices) voxel-identical to one volume. */
static int32_t pool_acquire(ora_grid* g) {
  const int32_t i = g->free_count;
  if (i < 1) return -1; /* reference: assert(idx >= 1), undefined in release; defined here as a
                           refused acquisition that leaves the counter alone */
  g->free_count = i - 1;
  const int32_t idx = g->heap[i - 1];
  const int64_t base = (int64_t)idx << BLOCK_VOLUME_BITS;
  for (int v = 0; v < BLOCK_VOLUME; ++v) {
    memset(&g->rgbw[(base + v) * 4], 0, 4);
    g->tsdf[base + v] = -1.0f;
    g->prob[base + v] = 0.5f;
  }
  return idx;
}
/* voxel_mem.cu:54-59 ReleaseBlock (no clearing) */
static void pool_release(ora_grid* g, int32_t idx) {
  const int32_t i = g->free_count;
  g->free_count = i + 1;
  g->heap[i] = idx;
}

/* Sharded volume (not in the reference): every shard holds the whole hash index, so
 * the bucket locks and the table layout evolve exactly as in one volume; a block's voxels live only
 * on its owner. Other shards mark its entry ORA_FOREIGN: occupied for Allocate / Delete, missing
 * for every reader. local_idx: the entry has voxels in this grid. */
#define ORA_FOREIGN 0x7FFFFFFF
static int local_idx(int32_t idx) { return idx >= 0 && idx != ORA_FOREIGN; }
static int owns(const ora_grid* g, s3 key) {
  return g->shard_count <= 1 ||
         ora_block_owner(key.x, key.y, key.z, (uint32_t)g->shard_count) == (uint32_t)g->shard_index;
}
/* atomicExch(&bucket_locks_[b], LOCKED) == FREE; the lock word remembers the owner shard + 1 of
 * the key that took it, so a sharded grid can count the losses to another shard's key */
static int lock_take(ora_grid* g, uint32_t b, uint8_t tag, int* cross) {
  if (g->locks[b] == 0) {
    g->locks[b] = tag;
    return 1;
  }
  if (g->locks[b] != tag) *cross = 1;
  return 0;
}
/* the pool block of a new entry of `key`: AquireBlock on its owner, ORA_FOREIGN elsewhere.
 * An exhausted pool drops the insert (returns 0; the lock stays taken) in one volume; a shard
 * keeps the entry (ORA_FOREIGN, no voxels) so every shard's index stays the same. */
static int new_block(ora_grid* g, s3 key, int32_t* idx) {
  if (!owns(g, key)) {
    *idx = ORA_FOREIGN;
    return 1;
  }
  if (g->free_count < 1) {
    g->st.pool_exhausted = 1;
    *idx = ORA_FOREIGN;
    return g->shard_count > 1;
  }
  *idx = pool_acquire(g);
  return 1;
}
/* a shard's owned entry without voxels (pool exhausted): listed for this frame's carving */
static void note_pending(ora_grid* g, s3 key, int32_t idx, uint32_t e) {
  if (g->shard_count <= 1 || idx != ORA_FOREIGN || !owns(g, key)) return;
  if (g->n_pend == g->pend_cap) {
    g->pend_cap = g->pend_cap ? 2 * g->pend_cap : 256;
    g->pend_pos = (s3*)realloc(g->pend_pos, sizeof(s3) * (size_t)g->pend_cap);
    g->pend_entry = (int32_t*)realloc(g->pend_entry, sizeof(int32_t) * (size_t)g->pend_cap);
  }
  g->pend_pos[g->n_pend] = key;
  g->pend_entry[g->n_pend] = (int32_t)e;
  g->n_pend++;
}

/* voxel_hash.cu:58-120 VoxelHashTable::Allocate, executed as one step of a sequential launch. */
static int hash_allocate(ora_grid* g, s3 key) {
  const uint32_t bucket = ora_hash(key.x, key.y, key.z);
  const uint32_t e0 = bucket << 1;
  const uint8_t tag = (uint8_t)(1 + (g->shard_count > 1
                                         ? ora_block_owner(key.x, key.y, key.z, (uint32_t)g->shard_count)
                                         : 0u));
  int cross = 0;
  for (int i = 0; i < NUM_ENTRY_PER_BUCKET; ++i) { /* existence :62-68 */
    const entry* b = &g->table[e0 + i];
    if (s3_eq(b->pos, key) && b->idx >= 0) return 0;
  }
  uint32_t last = e0 + NUM_ENTRY_PER_BUCKET - 1; /* traverse list :70-77 */
  while (g->table[last].offset) {
    last = (uint32_t)(last + (int32_t)g->table[last].offset) & ENTRY_MASK;
    const entry* b = &g->table[last];
    if (s3_eq(b->pos, key) && b->idx >= 0) return 0;
  }
  for (int i = 0; i < NUM_ENTRY_PER_BUCKET; ++i) { /* current bucket :79-91 */
    entry* b = &g->table[e0 + i];
    if (b->idx < 0) {
      if (lock_take(g, bucket, tag, &cross)) {
        int32_t idx;
        if (!new_block(g, key, &idx)) return -2; /* pool exhausted: insert dropped, lock stays taken */
        b->pos = key;
        b->offset = 0;
        b->idx = idx;
        note_pending(g, key, idx, e0 + (uint32_t)i);
        return 1;
      }
      g->st.last_cross_losses += cross;
      return -1;
    }
  }
  last = e0 + NUM_ENTRY_PER_BUCKET - 1; /* traverse list again :93-97 */
  while (g->table[last].offset)
    last = (uint32_t)(last + (int32_t)g->table[last].offset) & ENTRY_MASK;
  const uint32_t bucket_last = last >> 1;
  uint32_t next = last;
  for (int probes = 0; probes < NUM_ENTRY; ++probes) { /* append :99-119 */
    next = (next + 1) & ENTRY_MASK;
    if ((next & ENTRY_PER_BUCKET_MASK) != ENTRY_PER_BUCKET_MASK && g->table[next].idx < 0) {
      const uint32_t bucket_next = next >> 1;
      /* atomicExch(last) == FREE && atomicExch(next) == FREE */
      const int ok = lock_take(g, bucket_last, tag, &cross) && lock_take(g, bucket_next, tag, &cross);
      if (ok) {
        int32_t idx;
        if (!new_block(g, key, &idx)) return -2; /* pool exhausted (see new_block) */
        entry* bl = &g->table[last];
        entry* bn = &g->table[next];
        const uint32_t wrap = next > last ? 0u : (uint32_t)NUM_ENTRY;
        bl->offset = (int16_t)(next + wrap - last);
        bn->pos = key;
        bn->offset = 0;
        bn->idx = idx;
        note_pending(g, key, idx, next);
        return 1;
      }
      g->st.last_cross_losses += cross;
      return -1;
    }
  }
  return -1;
}

/* voxel_hash.cu:122-171 VoxelHashTable::Delete, one step of a sequential launch. */
static int hash_delete(ora_grid* g, s3 key) {
  const uint32_t bucket = ora_hash(key.x, key.y, key.z);
  const uint32_t e0 = bucket << 1;
  int cross = 0; /* (delete locks: the owner tag is irrelevant) */
  { /* slot 0, lock free :126-135 */
    entry* b = &g->table[e0];
    if (s3_eq(b->pos, key) && b->idx >= 0) {
      if (local_idx(b->idx)) pool_release(g, b->idx); /* a shard releases only its own blocks */
      b->offset = 0;
      b->idx = -1;
      return 1;
    }
  }
  uint32_t last = e0 + NUM_ENTRY_PER_BUCKET - 1;
  entry* head = &g->table[last];
  if (s3_eq(head->pos, key) && head->idx >= 0) { /* list head :137-152 */
    if (lock_take(g, bucket, 1, &cross)) {
      const uint32_t nidx = (uint32_t)(last + (int32_t)head->offset) & ENTRY_MASK;
      entry* nx = &g->table[nidx];
      if (local_idx(head->idx)) pool_release(g, head->idx);
      head->pos = nx->pos;
      head->offset = nx->offset ? (int16_t)(head->offset + nx->offset) : 0;
      head->idx = nx->idx;
      nx->offset = 0;
      nx->idx = -1;
      return 1;
    }
    return -1;
  }
  while (g->table[last].offset) { /* generic list :154-170 */
    entry* bl = &g->table[last];
    const uint32_t cur = (uint32_t)(last + (int32_t)bl->offset) & ENTRY_MASK;
    entry* bc = &g->table[cur];
    if (s3_eq(bc->pos, key) && bc->idx >= 0) {
      if (lock_take(g, bucket, 1, &cross)) {
        bl->offset = bc->offset ? (int16_t)(bl->offset + bc->offset) : 0;
        if (local_idx(bc->idx)) pool_release(g, bc->idx);
        bc->offset = 0;
        bc->idx = -1;
        return 1;
      }
      return -1;
    }
    last = cur;
  }
  return 0;
}

/* voxel_hash.cuh:124-161 RetrieveMutable -> entry index or -1 (the 1-entry cache never changes
 * results because the table is read-only during retrieval). */
static int64_t hash_find(const ora_grid* g, s3 block) {
  const uint32_t bucket = ora_hash(block.x, block.y, block.z);
  const uint32_t e0 = bucket << 1;
  for (int i = 0; i < NUM_ENTRY_PER_BUCKET; ++i) {
    const entry* b = &g->table[e0 + i];
    if (s3_eq(b->pos, block) && b->idx >= 0) return e0 + i;
  }
  uint32_t last = e0 + NUM_ENTRY_PER_BUCKET - 1;
  while (g->table[last].offset) {
    last = (uint32_t)(last + (int32_t)g->table[last].offset) & ENTRY_MASK;
    const entry* b = &g->table[last];
    if (s3_eq(b->pos, block) && b->idx >= 0) return last;
  }
  return -1;
}
static int64_t voxel_addr(const ora_grid* g, s3 point, int64_t* entry_out) {
  const s3 block = point_to_block(point);
  const int64_t e = hash_find(g, block);
  if (entry_out) *entry_out = e;
  if (e < 0 || !local_idx(g->table[e].idx)) return -1;
  const int off = offset_to_index(point.x & 7, point.y & 7, point.z & 7);
  return ((int64_t)g->table[e].idx << BLOCK_VOLUME_BITS) + off;
}
/* Retrieve<VoxelTSDF> with default VoxelTSDF() = 1 (voxel_types.cu:9) */
static float retrieve_tsdf(const ora_grid* g, s3 p) {
  const int64_t a = voxel_addr(g, p, NULL);
  return a < 0 ? 1.0f : g->tsdf[a];
}

/* ---------------- visibility (voxel_tsdf.cu:48-80) ---------------- */
typedef struct {
  intr K, Kinv;
  int W, H;
  se3 cTw, wTc;
  float voxel, trunc, max_depth;
} frame_params;

static int voxel_visible(const frame_params* P, s3 pg) {
  v3 pw = {(float)pg.x * P->voxel, (float)pg.y * P->voxel, (float)pg.z * P->voxel};
  v3 pc = se3_apply(&P->cTw, pw);
  v3 ph = intr_mul(P->K, pc);
  const float u = ph.x / ph.z, v = ph.y / ph.z; /* hnormalized */
  return u >= 0 && u <= (float)(P->W - 1) && v >= 0 && v <= (float)(P->H - 1) && ph.z >= 0;
}
static int block_visible(const frame_params* P, s3 block, int full) {
  const s3 pg = block_to_point(block);
  int vis = full;
  for (int i = 0; i < 8; ++i) {
    s3 c = {(int16_t)(pg.x + ((i >> 0) & 1) * (BLOCK_LEN - 1)),
            (int16_t)(pg.y + ((i >> 1) & 1) * (BLOCK_LEN - 1)),
            (int16_t)(pg.z + ((i >> 2) & 1) * (BLOCK_LEN - 1))};
    const int v = voxel_visible(P, c);
    if (full) vis &= v; else vis |= v;
  }
  return vis;
}

/* ---------------- public API ---------------- */
ora_grid* ora_create(float voxel_size, float truncation, int num_block_bits) {
  if (num_block_bits < 1 || num_block_bits > 24) return NULL;
  ora_grid* g = (ora_grid*)calloc(1, sizeof(ora_grid));
  g->voxel = voxel_size;
  g->trunc = truncation;
  g->nb_bits = num_block_bits;
  g->nblocks = 1 << num_block_bits;
  g->table = (entry*)calloc(NUM_ENTRY, sizeof(entry)); /* zero position/offset (Appendix A.3b) */
  for (int i = 0; i < NUM_ENTRY; ++i) g->table[i].idx = -1; /* voxel_hash.cu:26-29 */
  g->locks = (uint8_t*)calloc(NUM_BUCKET, 1);
  g->heap = (int32_t*)malloc(sizeof(int32_t) * g->nblocks);
  for (int i = 0; i < g->nblocks; ++i) g->heap[i] = i; /* voxel_mem.cu:6-11 */
  g->free_count = g->nblocks;
  const size_t nv = (size_t)g->nblocks * BLOCK_VOLUME;
  g->tsdf = (float*)calloc(nv, sizeof(float));
  g->prob = (float*)calloc(nv, sizeof(float));
  g->rgbw = (uint8_t*)calloc(nv, 4);
  g->vis = (int32_t*)malloc(sizeof(int32_t) * NUM_ENTRY);
  if (!g->table || !g->locks || !g->heap || !g->tsdf || !g->prob || !g->rgbw || !g->vis) {
    ora_destroy(g);
    return NULL;
  }
  return g;
}

void ora_destroy(ora_grid* g) {
  if (!g) return;
  free(g->table); free(g->locks); free(g->heap); free(g->tsdf); free(g->prob); free(g->rgbw);
  free(g->range); free(g->vis); free(g->pend_pos); free(g->pend_entry);
  free(g);
}

static void make_params(const ora_grid* g, frame_params* P, const float K[4], int W, int H,
                        const float q[4], const float t[3], float max_depth) {
  P->K.fx = K[0]; P->K.fy = K[1]; P->K.cx = K[2]; P->K.cy = K[3];
  P->Kinv = intr_inverse(P->K); /* camera.cuh:65 CameraParams ctor */
  P->W = W; P->H = H;
  P->cTw.q.x = q[0]; P->cTw.q.y = q[1]; P->cTw.q.z = q[2]; P->cTw.q.w = q[3];
  P->cTw.t.x = t[0]; P->cTw.t.y = t[1]; P->cTw.t.z = t[2];
  P->wTc = se3_inverse(&P->cTw);
  P->voxel = g->voxel; P->trunc = g->trunc; P->max_depth = max_depth;
}

/* owner of block b among shard_count GPUs: hash of the 4^3-block brick; must match
 * tsdf_block_owner / brick_owner in the engine */
uint32_t ora_block_owner(int16_t x, int16_t y, int16_t z, uint32_t shards) {
  uint32_t h = ((uint32_t)(int32_t)(x >> 2) * 0x9E3779B1u) ^ ((uint32_t)(int32_t)(y >> 2) * 0x85EBCA77u) ^
               ((uint32_t)(int32_t)(z >> 2) * 0xC2B2AE3Du);
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  return shards <= 1 ? 0u : h % shards;
}

void ora_set_shard(ora_grid* g, int index, int count) {
  g->shard_index = index;
  g->shard_count = count;
}

static void ensure_range(ora_grid* g, int W, int H) {
  if (g->range_cap < W * H) {
    free(g->range);
    g->range = (float*)malloc(sizeof(float) * (size_t)W * H);
    g->range_cap = W * H;
  }
}

/* voxel_tsdf.cu:104-147 block_allocate_kernel for one pixel: writes img_depth_to_range_ and hands
 * every DDA sample's block whose 8 corners are all in view (is_block_visible<true>) to `visit`,
 * with its candidate order (pixel raster index, then DDA step): Allocate in one volume, key
 * collection in a sharded frame. */
typedef void (*key_visit)(ora_grid* g, void* ctx, s3 key, uint64_t order);
static void dda_pixel(ora_grid* g, const frame_params* P, const float* depth, int x, int y,
                      key_visit visit, void* ctx) {
  const int idx = y * P->W + x;
  const float d = depth[idx];
  v3 ph = {(float)x, (float)y, 1.0f};
  v3 pc = intr_mul(P->Kinv, ph);
  g->range[idx] = v3_norm(pc);
  if (d == 0 || d > P->max_depth) return;
  v3 pcd = {pc.x * d, pc.y * d, pc.z * d};
  v3 pw = se3_apply(&P->wTc, pcd);
  const float r = g->range[idx];
  v3 dc = {pc.x / r, pc.y / r, pc.z / r};
  v3 dw = qrot(P->wTc.q, dc);
  v3 sw = {pw.x - dw.x * P->trunc, pw.y - dw.y * P->trunc, pw.z - dw.z * P->trunc};
  v3 dg = {dw.x / P->voxel, dw.y / P->voxel, dw.z / P->voxel};
  v3 sg = {sw.x / P->voxel, sw.y / P->voxel, sw.z / P->voxel};
  const float two_trunc = 2 * P->trunc;
  v3 rg = {two_trunc * dg.x, two_trunc * dg.y, two_trunc * dg.z};
  const int step_grid = f2i(ceilf(fmaxf(fmaxf(fabsf(rg.x), fabsf(rg.y)), fabsf(rg.z)) / BLOCK_LEN));
  const float div = fmaxf((float)step_grid, 1);
  v3 st = {rg.x / div, rg.y / div, rg.z / div};
  v3 pos = sg;
  for (int i = 0; i <= step_grid; ++i) {
    s3 p = {f2s(roundf(pos.x)), f2s(roundf(pos.y)), f2s(roundf(pos.z))};
    s3 b = point_to_block(p);
    if (block_visible(P, b, 1)) visit(g, ctx, b, ((uint64_t)idx << 8) | (uint64_t)(i & 0xFF));
    pos.x += st.x; pos.y += st.y; pos.z += st.z;
  }
}
static void visit_allocate(ora_grid* g, void* ctx, s3 key, uint64_t order) {
  const int r2 = hash_allocate(g, key);
  if (r2 != 0) g->st.last_num_candidates++;
  if (r2 > 0) g->st.last_num_alloc++;
}

/* GatherVisible (voxel_tsdf.cu:388-397, 82-102, 456-472: full-table scan, entry order) +
 * UpdateTSDF (:149-205) + the min |tsdf| >= 0.9 test of space_carving_kernel (:207-230), over the
 * blocks this grid holds voxels for. The carve candidates are returned in visible-list (= entry)
 * order as the snapshot gather_visible_blocks_kernel took: positions in *cpos, entries in *cent
 * (malloc'ed, caller frees). */
static int update_and_carve_test(ora_grid* g, const frame_params* Pp, const uint8_t* rgb,
                                 const float* depth, const float* ht, const float* lt, s3** cpos,
                                 int32_t** cent) {
  const frame_params P = *Pp;
  const int W = P.W, H = P.H;
  const float max_depth = P.max_depth;
  int nvis = 0;
  for (int e = 0; e < NUM_ENTRY; ++e) {
    const entry* b = &g->table[e];
    if (!local_idx(b->idx)) continue;
    if (block_visible(&P, b->pos, 0)) g->vis[nvis++] = e;
  }
  g->st.last_num_visible = nvis;

  s3* snap_pos = (s3*)malloc(sizeof(s3) * (nvis ? nvis : 1));
  int32_t* snap_idx = (int32_t*)malloc(sizeof(int32_t) * (nvis ? nvis : 1));
  for (int i = 0; i < nvis; ++i) { /* gather_visible_blocks_kernel copies the entries */
    snap_pos[i] = g->table[g->vis[i]].pos;
    snap_idx[i] = g->table[g->vis[i]].idx;
  }
  const float neg_trunc = -P.trunc;
  int64_t nupd = 0;
  for (int i = 0; i < nvis; ++i) {
    const s3 bp = block_to_point(snap_pos[i]);
    const int64_t base = (int64_t)snap_idx[i] << BLOCK_VOLUME_BITS;
    for (int rz = 0; rz < BLOCK_LEN; ++rz)
      for (int ry = 0; ry < BLOCK_LEN; ++ry)
        for (int rx = 0; rx < BLOCK_LEN; ++rx) {
          const s3 pa = {(int16_t)(bp.x + rx), (int16_t)(bp.y + ry), (int16_t)(bp.z + rz)};
          v3 pw = {(float)pa.x * P.voxel, (float)pa.y * P.voxel, (float)pa.z * P.voxel};
          v3 pc = se3_apply(&P.cTw, pw);
          v3 ph = intr_mul(P.K, pc);
          const int u = f2i(roundf(ph.x / ph.z));
          const int v = f2i(roundf(ph.y / ph.z));
          if (!(u >= 0 && u < W && v >= 0 && v < H)) continue;
          const int img = v * W + u;
          const float d = depth[img];
          if (d == 0 || d > max_depth) continue;
          const float sdf = g->range[img] * (d - ph.z);
          if (!(sdf > neg_trunc)) continue;
          const float tsdf_new = fminf(1, sdf / P.trunc);
          const int64_t a = base + offset_to_index(rx, ry, rz);
          uint8_t* rgbw = &g->rgbw[a * 4];
          const float w_new = (1 - d / max_depth) * 4;
          const float w_old = (float)rgbw[3];
          const float wc = w_old + w_new;
          const float r0 = ((float)rgbw[0] * w_old + (float)rgb[img * 3 + 0] * w_new) / wc;
          const float r1 = ((float)rgbw[1] * w_old + (float)rgb[img * 3 + 1] * w_new) / wc;
          const float r2 = ((float)rgbw[2] * w_old + (float)rgb[img * 3 + 2] * w_new) / wc;
          g->tsdf[a] = (g->tsdf[a] * w_old + tsdf_new * w_new) / wc;
          rgbw[3] = f2u8(fminf(roundf(wc), 40));
          rgbw[0] = f2u8(roundf(r0));
          rgbw[1] = f2u8(roundf(r1));
          rgbw[2] = f2u8(roundf(r2));
          const float p = g->prob[a];
          const float h = ht ? ht[img] : 1.0f;
          const float l = lt ? lt[img] : 1.0f;
          /* CUDA logf / expf restated as the oracle's fixed algorithms (ora_math.c: why) */
          const float pos = ora_expf((w_old * ora_logf(p) + w_new * ora_logf(h)) / wc);
          const float neg = ora_expf((w_old * ora_logf(1 - p) + w_new * ora_logf(l)) / wc);
          g->prob[a] = pos / (pos + neg);
          ++nupd;
        }
  }
  g->st.last_num_updated = nupd;

  /* space_carving_kernel's block minimum (deletes do not touch voxel values, so all minima can be
   * taken before the first Delete) */
  int nc = 0;
  for (int i = 0; i < nvis; ++i) {
    const int64_t base = (int64_t)snap_idx[i] << BLOCK_VOLUME_BITS;
    float mn = fabsf(g->tsdf[base]);
    for (int v = 1; v < BLOCK_VOLUME; ++v) mn = fminf(mn, fabsf(g->tsdf[base + v]));
    if (mn >= 0.9f) {
      snap_pos[nc] = snap_pos[i];
      snap_idx[nc] = g->vis[i];
      ++nc;
    }
  }
  *cpos = snap_pos;
  *cent = snap_idx;
  return nc;
}

int ora_integrate(ora_grid* g, const uint8_t* rgb, const float* depth, const float* ht,
                  const float* lt, int W, int H, const float K[4], const float q[4],
                  const float t[3], float max_depth) {
  if (W <= 0 || H <= 0) return -1;
  if (g->shard_count > 1) return -2; /* a shard integrates through ora_shard_keys/_update/_delete */
  ensure_range(g, W, H);
  frame_params P;
  make_params(g, &P, K, W, H, q, t, max_depth);
  g->st.last_num_alloc = 0;
  g->st.last_num_candidates = 0;
  g->st.last_num_deleted = 0;
  g->st.last_num_updated = 0;
  g->st.last_cross_losses = 0;

  /* ---- Allocate (voxel_tsdf.cu:377-386): sequential raster order, then ResetLocks ---- */
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) dda_pixel(g, &P, depth, x, y, visit_allocate, NULL);
  memset(g->locks, 0, NUM_BUCKET);

  /* ---- GatherVisible + UpdateTSDF + SpaceCarving (voxel_tsdf.cu:388-397, 474-488) ---- */
  s3* cpos;
  int32_t* cent;
  const int nc = update_and_carve_test(g, &P, rgb, depth, ht, lt, &cpos, &cent);
  for (int i = 0; i < nc; ++i) /* deletes in entry order, then ResetLocks */
    if (hash_delete(g, cpos[i]) > 0) g->st.last_num_deleted++;
  memset(g->locks, 0, NUM_BUCKET);
  free(cpos);
  free(cent);
  g->st.frames++;
  return 0;
}

/* ---------------------------------------------------------------------------------------------
 * Sharded frame (not in the reference), the engine's tsdf_integrate_shard_* in three
 * phases around the two exchanges. Every shard keeps the whole hash index, so the union of the
 * shards is the one-volume TSDFGrid::Integrate above, block for block and voxel for voxel:
 *   ora_shard_keys   : the DDA over pixel rows [row_lo, row_hi) -> the fully visible keys missing
 *                      from the index, each once with its smallest candidate order;
 *   ora_shard_update : Allocate of the union of every shard's keys in candidate order (a key's
 *                      first attempt decides it: a lock it lost stays taken for the launch), pool
 *                      blocks only for owned keys; then visibility, update and the carve test of
 *                      the owned blocks -> carve candidates;
 *   ora_shard_delete : Delete of the union of every shard's candidates in entry order.
 * --------------------------------------------------------------------------------------------- */
typedef struct {
  uint64_t* key;   /* packed (x, y, z) | 1 << 48 */
  uint64_t* order;
  int64_t n, cap;
} keylist;
static uint64_t pack_s3(s3 k) {
  return (uint64_t)(uint16_t)k.x | ((uint64_t)(uint16_t)k.y << 16) | ((uint64_t)(uint16_t)k.z << 32) |
         (1ull << 48);
}
static void visit_collect(ora_grid* g, void* ctx, s3 key, uint64_t order) {
  keylist* L = (keylist*)ctx;
  if (hash_find(g, key) >= 0) return; /* already in the index (any shard's) */
  if (L->n == L->cap) {
    L->cap = L->cap ? 2 * L->cap : 4096;
    L->key = (uint64_t*)realloc(L->key, sizeof(uint64_t) * (size_t)L->cap);
    L->order = (uint64_t*)realloc(L->order, sizeof(uint64_t) * (size_t)L->cap);
  }
  L->key[L->n] = pack_s3(key);
  L->order[L->n] = order;
  L->n++;
}
typedef struct { uint64_t a, b; int64_t i; } triple;
static int cmp_triple(const void* x, const void* y) {
  const triple* p = (const triple*)x;
  const triple* q = (const triple*)y;
  if (p->a != q->a) return p->a < q->a ? -1 : 1;
  if (p->b != q->b) return p->b < q->b ? -1 : 1;
  return 0;
}

int64_t ora_shard_keys(ora_grid* g, const float* depth, int W, int H, const float K[4],
                       const float q[4], const float t[3], float max_depth, int row_lo, int row_hi,
                       int16_t* keys_out, uint64_t* orders_out, int64_t capacity) {
  if (W <= 0 || H <= 0) return -1;
  ensure_range(g, W, H);
  frame_params P;
  make_params(g, &P, K, W, H, q, t, max_depth);
  keylist L = {NULL, NULL, 0, 0};
  if (row_lo < 0) row_lo = 0;
  if (row_hi > H) row_hi = H;
  for (int y = row_lo; y < row_hi; ++y)
    for (int x = 0; x < W; ++x) dda_pixel(g, &P, depth, x, y, visit_collect, &L);
  /* unique keys, smallest order each */
  triple* s = (triple*)malloc(sizeof(triple) * (size_t)(L.n ? L.n : 1));
  for (int64_t i = 0; i < L.n; ++i) s[i] = (triple){L.key[i], L.order[i], i};
  qsort(s, (size_t)L.n, sizeof(triple), cmp_triple);
  int64_t n = 0;
  for (int64_t i = 0; i < L.n; ++i) {
    if (i > 0 && s[i].a == s[i - 1].a) continue;
    if (n < capacity) {
      keys_out[3 * n + 0] = (int16_t)(s[i].a & 0xFFFF);
      keys_out[3 * n + 1] = (int16_t)((s[i].a >> 16) & 0xFFFF);
      keys_out[3 * n + 2] = (int16_t)((s[i].a >> 32) & 0xFFFF);
      orders_out[n] = s[i].b;
    }
    ++n;
  }
  free(s);
  free(L.key);
  free(L.order);
  return n;
}

int64_t ora_shard_update(ora_grid* g, const int16_t* keys, const uint64_t* orders, int64_t n,
                         const uint8_t* rgb, const float* depth, const float* ht, const float* lt,
                         int W, int H, const float K[4], const float q[4], const float t[3],
                         float max_depth, int16_t* cand_pos, int32_t* cand_entry, int64_t cand_cap) {
  if (W <= 0 || H <= 0 || n < 0) return -1;
  ensure_range(g, W, H);
  frame_params P;
  make_params(g, &P, K, W, H, q, t, max_depth);
  for (int y = 0; y < H; ++y) /* img_depth_to_range_ of every pixel (block_allocate_kernel :120) */
    for (int x = 0; x < W; ++x) {
      v3 ph = {(float)x, (float)y, 1.0f};
      g->range[y * W + x] = v3_norm(intr_mul(P.Kinv, ph));
    }
  g->st.last_num_alloc = 0;
  g->st.last_num_candidates = 0;
  g->st.last_num_deleted = 0;
  g->st.last_num_updated = 0;
  g->st.last_cross_losses = 0;
  /* ---- Allocate of the union in candidate order, then ResetLocks ---- */
  triple* s = (triple*)malloc(sizeof(triple) * (size_t)(n ? n : 1));
  for (int64_t i = 0; i < n; ++i) s[i] = (triple){orders[i], (uint64_t)i, i};
  qsort(s, (size_t)n, sizeof(triple), cmp_triple);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = s[i].i;
    const s3 key = {keys[3 * k], keys[3 * k + 1], keys[3 * k + 2]};
    visit_allocate(g, NULL, key, orders[k]);
  }
  free(s);
  memset(g->locks, 0, NUM_BUCKET);
  /* ---- visibility, update, carve test of the owned blocks ---- */
  s3* cpos;
  int32_t* cent;
  const int nc = update_and_carve_test(g, &P, rgb, depth, ht, lt, &cpos, &cent);
  for (int i = 0; i < nc && i < cand_cap; ++i) {
    cand_pos[3 * i + 0] = cpos[i].x;
    cand_pos[3 * i + 1] = cpos[i].y;
    cand_pos[3 * i + 2] = cpos[i].z;
    cand_entry[i] = cent[i];
  }
  /* + the owned entries left without voxels by an exhausted pool (carved this frame) */
  int64_t ntot = nc;
  for (int64_t j = 0; j < g->n_pend; ++j, ++ntot)
    if (ntot < cand_cap) {
      cand_pos[3 * ntot + 0] = g->pend_pos[j].x;
      cand_pos[3 * ntot + 1] = g->pend_pos[j].y;
      cand_pos[3 * ntot + 2] = g->pend_pos[j].z;
      cand_entry[ntot] = g->pend_entry[j];
    }
  g->n_pend = 0;
  free(cpos);
  free(cent);
  return ntot;
}

void ora_shard_delete(ora_grid* g, const int16_t* cand_pos, const int32_t* cand_entry, int64_t n) {
  triple* s = (triple*)malloc(sizeof(triple) * (size_t)(n ? n : 1));
  for (int64_t i = 0; i < n; ++i) s[i] = (triple){(uint64_t)(uint32_t)cand_entry[i], 0, i};
  qsort(s, (size_t)n, sizeof(triple), cmp_triple);
  int deleted = 0;
  for (int64_t i = 0; i < n; ++i) { /* Delete in entry order (the union of the visible lists) */
    const int64_t k = s[i].i;
    const s3 key = {cand_pos[3 * k], cand_pos[3 * k + 1], cand_pos[3 * k + 2]};
    const int32_t f0 = g->free_count;
    if (hash_delete(g, key) > 0 && g->free_count > f0) ++deleted; /* owned blocks released */
  }
  memset(g->locks, 0, NUM_BUCKET);
  free(s);
  g->st.last_num_deleted = deleted;
  g->st.frames++;
}

/* voxel_tsdf.cu:232-307 ray_cast_kernel */
void ora_raycast(const ora_grid* g, const float K[4], int W, int H, const float q[4],
                 const float t[3], float max_depth, uint8_t* rgba, uint8_t* normal) {
  frame_params P;
  make_params(g, &P, K, W, H, q, t, max_depth);
  const float step_size = g->trunc / 2; /* voxel_tsdf.cu:497 truncation_ / 2 */
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const int idx = y * W + x;
      uint8_t* o1 = &rgba[idx * 4];
      uint8_t* o2 = &normal[idx * 4];
      v3 ph = {(float)x, (float)y, 1.0f};
      v3 pc = intr_mul(P.Kinv, ph);
      const float n = v3_dot(pc, pc); /* Eigen normalized() */
      v3 dc = pc;
      if (n > 0) { const float s = sqrtf(n); dc.x = pc.x / s; dc.y = pc.y / s; dc.z = pc.z / s; }
      v3 dw = qrot(P.wTc.q, dc);
      v3 sg = {dw.x * step_size / P.voxel, dw.y * step_size / P.voxel, dw.z * step_size / P.voxel};
      const int max_step = f2i(ceilf(max_depth / step_size));
      v3 pos = {P.wTc.t.x / P.voxel, P.wTc.t.y / P.voxel, P.wTc.t.z / P.voxel};
      s3 rp = {f2s(roundf(pos.x)), f2s(roundf(pos.y)), f2s(roundf(pos.z))};
      float prev = retrieve_tsdf(g, rp);
      pos.x += sg.x; pos.y += sg.y; pos.z += sg.z;
      int hit = 0;
      for (int i = 1; i < max_step; ++i) {
        rp.x = f2s(roundf(pos.x)); rp.y = f2s(roundf(pos.y)); rp.z = f2s(roundf(pos.z));
        const float cur = retrieve_tsdf(g, rp);
        if (prev > 0 && cur <= 0 && (double)(prev - cur) <= 1.5) {
          v3 p1 = {pos.x - sg.x, pos.y - sg.y, pos.z - sg.z};
          v3 p2 = pos;
          v3 mid = {(p1.x + p2.x) / 2, (p1.y + p2.y) / 2, (p1.z + p2.z) / 2};
          for (;;) {
            v3 dd = {p1.x - p2.x, p1.y - p2.y, p1.z - p2.z};
            if (!((double)v3_dot(dd, dd) > .1)) break;
            s3 mp = {f2s(roundf(mid.x)), f2s(roundf(mid.y)), f2s(roundf(mid.z))};
            if (retrieve_tsdf(g, mp) < 0) p2 = mid; else p1 = mid;
            mid.x = (p1.x + p2.x) / 2; mid.y = (p1.y + p2.y) / 2; mid.z = (p1.z + p2.z) / 2;
          }
          const s3 fg = {f2s(roundf(mid.x)), f2s(roundf(mid.y)), f2s(roundf(mid.z))};
          const int64_t a = voxel_addr(g, fg, NULL);
          uint8_t c0 = 0, c1 = 0, c2 = 0;
          float prob = 0.0f; /* VoxelSEGM() default 0, VoxelRGBW() default 0 */
          if (a >= 0) {
            c0 = g->rgbw[a * 4 + 0]; c1 = g->rgbw[a * 4 + 1]; c2 = g->rgbw[a * 4 + 2];
            prob = g->prob[a];
          }
          const s3 xp = {(int16_t)(fg.x + 1), fg.y, fg.z}, xn = {(int16_t)(fg.x - 1), fg.y, fg.z};
          const s3 yp = {fg.x, (int16_t)(fg.y + 1), fg.z}, yn = {fg.x, (int16_t)(fg.y - 1), fg.z};
          const s3 zp = {fg.x, fg.y, (int16_t)(fg.z + 1)}, zn = {fg.x, fg.y, (int16_t)(fg.z - 1)};
          v3 nr = {retrieve_tsdf(g, xp) - retrieve_tsdf(g, xn), retrieve_tsdf(g, yp) - retrieve_tsdf(g, yn),
                   retrieve_tsdf(g, zp) - retrieve_tsdf(g, zn)};
          v3 nd = {-dw.x, -dw.y, -dw.z};
          const float diff = fmaxf(v3_dot(nr, nd) / v3_norm(nr), 0);
          const float alpha = (float)((double)fmaxf((float)((double)prob - 0.5), 0) / .5);
          const float oma = 1 - alpha;
          o1[0] = f2u8(alpha * 255 + oma * (float)c0);
          o1[1] = f2u8(oma * (float)c1);
          o1[2] = f2u8(oma * (float)c2);
          o1[3] = 255;
          const float sh = oma * diff * 255;
          o2[0] = f2u8(alpha * 255 + sh);
          o2[1] = f2u8(sh);
          o2[2] = f2u8(sh);
          o2[3] = 255;
          hit = 1;
          break;
        }
        prev = cur;
        pos.x += sg.x; pos.y += sg.y; pos.z += sg.z;
      }
      if (!hit) {
        memset(o1, 0, 4);
        memset(o2, 0, 4);
      }
    }
}

/* voxel_tsdf.cu:14-25 check_bound_kernel, :27-32 check_valid_kernel, :34-46 download_tsdf_kernel,
 * :399-454 GatherValid / GatherVoxels; bounds scaled by voxel_tsdf.cuh:21-26 BoundingCube::Scale */
int64_t ora_query(const ora_grid* g, const float* bounds, float* out, int64_t capacity) {
  int16_t bb[6] = {0, 0, 0, 0, 0, 0};
  if (bounds) {
    const float scale = (float)(1. / (double)g->voxel);
    for (int i = 0; i < 6; ++i) bb[i] = f2s(bounds[i] * scale);
  }
  int64_t nblk = 0;
  for (int pass = 0; pass < 2; ++pass) {
    int64_t k = 0;
    for (int e = 0; e < NUM_ENTRY; ++e) {
      const entry* b = &g->table[e];
      if (!local_idx(b->idx)) continue;
      const s3 vg = block_to_point(b->pos);
      if (bounds) {
        const int inside = vg.x >= bb[0] && vg.y >= bb[2] && vg.z >= bb[4] &&
                           vg.x + BLOCK_LEN - 1 <= bb[1] && vg.y + BLOCK_LEN - 1 <= bb[3] &&
                           vg.z + BLOCK_LEN - 1 <= bb[5];
        if (!inside) continue;
      }
      if (pass == 1) {
        const int64_t base = (int64_t)b->idx << BLOCK_VOLUME_BITS;
        for (int rz = 0; rz < BLOCK_LEN; ++rz)
          for (int ry = 0; ry < BLOCK_LEN; ++ry)
            for (int rx = 0; rx < BLOCK_LEN; ++rx) {
              const int o = offset_to_index(rx, ry, rz);
              float* w = &out[(k * BLOCK_VOLUME + o) * 4];
              const s3 pg = {(int16_t)(vg.x + rx), (int16_t)(vg.y + ry), (int16_t)(vg.z + rz)};
              w[0] = (float)pg.x * g->voxel;
              w[1] = (float)pg.y * g->voxel;
              w[2] = (float)pg.z * g->voxel;
              w[3] = g->tsdf[base + o];
            }
      }
      ++k;
    }
    nblk = k;
    if (!out || capacity < nblk * BLOCK_VOLUME) break;
  }
  return nblk * BLOCK_VOLUME;
}

void ora_get_stats(const ora_grid* g, ora_stats* s) {
  *s = g->st;
  s->active_blocks = g->nblocks - g->free_count;
}

int32_t ora_num_entries(void) { return NUM_ENTRY; }
int32_t ora_num_blocks(const ora_grid* g) { return g->nblocks; }

void ora_dump(const ora_grid* g, int16_t* pos_off, int32_t* idx, int32_t* heap, int32_t* free_count,
              float* tsdf, float* prob, uint8_t* rgbw) {
  if (pos_off || idx)
    for (int e = 0; e < NUM_ENTRY; ++e) {
      if (pos_off) {
        pos_off[e * 4 + 0] = g->table[e].pos.x;
        pos_off[e * 4 + 1] = g->table[e].pos.y;
        pos_off[e * 4 + 2] = g->table[e].pos.z;
        pos_off[e * 4 + 3] = g->table[e].offset;
      }
      if (idx) idx[e] = g->table[e].idx;
    }
  if (heap) memcpy(heap, g->heap, sizeof(int32_t) * g->nblocks);
  if (free_count) *free_count = g->free_count;
  const size_t nv = (size_t)g->nblocks * BLOCK_VOLUME;
  if (tsdf) memcpy(tsdf, g->tsdf, nv * sizeof(float));
  if (prob) memcpy(prob, g->prob, nv * sizeof(float));
  if (rgbw) memcpy(rgbw, g->rgbw, nv * 4);
}

void ora_hash_allocate(ora_grid* g, const int16_t* keys, int n) {
  for (int i = 0; i < n; ++i) {
    s3 k = {keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]};
    hash_allocate(g, k);
  }
  memset(g->locks, 0, NUM_BUCKET); /* VoxelHashTable::ResetLocks */
}

void ora_hash_delete(ora_grid* g, const int16_t* keys, int n) {
  for (int i = 0; i < n; ++i) {
    s3 k = {keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]};
    hash_delete(g, k);
  }
  memset(g->locks, 0, NUM_BUCKET);
}

void ora_hash_retrieve(const ora_grid* g, const int16_t* points, int n, uint8_t* rgbw, float* tsdf,
                       float* prob, int16_t* bpo, int32_t* bidx) {
  for (int i = 0; i < n; ++i) {
    s3 p = {points[3 * i], points[3 * i + 1], points[3 * i + 2]};
    int64_t e;
    const int64_t a = voxel_addr(g, p, &e);
    if (rgbw) {
      for (int c = 0; c < 4; ++c) rgbw[i * 4 + c] = a < 0 ? 0 : g->rgbw[a * 4 + c];
    }
    if (tsdf) tsdf[i] = a < 0 ? 1.0f : g->tsdf[a];
    if (prob) prob[i] = a < 0 ? 0.0f : g->prob[a];
    const s3 blk = point_to_block(p);
    if (bpo) {
      /* cache semantics (voxel_hash.cuh:157-159): miss -> {pos, offset -1, idx -1} */
      bpo[i * 4 + 0] = e < 0 ? blk.x : g->table[e].pos.x;
      bpo[i * 4 + 1] = e < 0 ? blk.y : g->table[e].pos.y;
      bpo[i * 4 + 2] = e < 0 ? blk.z : g->table[e].pos.z;
      bpo[i * 4 + 3] = e < 0 ? -1 : g->table[e].offset;
    }
    if (bidx) bidx[i] = e < 0 ? -1 : g->table[e].idx;
  }
}

int ora_hash_assign(ora_grid* g, const int16_t* points, int n, const uint8_t* rgbw) {
  int missing = 0;
  for (int i = 0; i < n; ++i) {
    s3 p = {points[3 * i], points[3 * i + 1], points[3 * i + 2]};
    const int64_t a = voxel_addr(g, p, NULL);
    if (a < 0) { ++missing; continue; }
    memcpy(&g->rgbw[a * 4], &rgbw[i * 4], 4);
  }
  return missing;
}

int32_t ora_num_active_blocks(const ora_grid* g) { return g->nblocks - g->free_count; }

void ora_pool_acquire(ora_grid* g, int n, int32_t* out) {
  for (int i = 0; i < n; ++i) out[i] = pool_acquire(g);
}
void ora_pool_release(ora_grid* g, const int32_t* idx, int n) {
  for (int i = 0; i < n; ++i) pool_release(g, idx[i]);
}
void ora_pool_set_weight(ora_grid* g, int32_t b, uint8_t w) {
  const int64_t base = (int64_t)b << BLOCK_VOLUME_BITS;
  for (int v = 0; v < BLOCK_VOLUME; ++v) g->rgbw[(base + v) * 4 + 3] = w;
}
void ora_pool_get_weights(const ora_grid* g, int32_t b, uint8_t* out) {
  const int64_t base = (int64_t)b << BLOCK_VOLUME_BITS;
  for (int v = 0; v < BLOCK_VOLUME; ++v) out[v] = g->rgbw[(base + v) * 4 + 3];
}

/* ---------------- marching cubes over the selected blocks ----------------
 * Replaces Query + KrisLibrary SparseTSDFReconstruction::ExtractMesh
 * (examples/ros_camera_driver/ros_offline.cc:258-318; not vendored -> parity unpinned):
 *  - samples: every voxel g of a selected block (GatherValid / GatherVoxels selection, see
 *    ora_query) at (float)g * voxel + voxel / 2 (the caller's +cell/2 offset, :281-283); its value
 *    is its tsdf when its weight >= min_weight, else `missing` (KrisLibrary defaultValue = the
 *    truncation distance, :279-280); grid points outside selected blocks are `missing` too;
 *  - cells: the cube with lower corner c is meshed iff one of its 8 corners lies in a selected
 *    block; it belongs to the block of the first such corner (corner order i = x | y << 1 | z << 2);
 *  - order: blocks in hash-entry order, cells of a block by (z, y, x) of c in [8b - 1, 8b + 7]^3,
 *    triangles in case-table order; vertex on edge (a, b): t = va / (va - vb), p = pa + t (pb - pa)
 *    along the edge's axis. Output: 9 floats per triangle. */
/* the case table: derived by ora_mc_cases.c (not the product's header; tests/test_mc_table.py
 * checks the two are equal) */
const int8_t* ora_mc_tri(void);
const uint8_t* ora_mc_ntri(void);
int ora_mc_edge(int e, int s);

static int block_selected(const ora_grid* g, s3 blk, const int16_t* bb, int64_t* e_out) {
  const int64_t e = hash_find(g, blk);
  if (e_out) *e_out = e;
  if (e < 0 || !local_idx(g->table[e].idx)) return 0;
  if (!bb) return 1;
  const s3 vg = block_to_point(blk);
  return vg.x >= bb[0] && vg.y >= bb[2] && vg.z >= bb[4] && vg.x + BLOCK_LEN - 1 <= bb[1] &&
         vg.y + BLOCK_LEN - 1 <= bb[3] && vg.z + BLOCK_LEN - 1 <= bb[5];
}

int64_t ora_extract_mesh(const ora_grid* g, const float* bounds, float missing, int min_weight,
                         float* out, int64_t capacity) {
  int16_t bbv[6] = {0, 0, 0, 0, 0, 0};
  const int16_t* bb = NULL;
  if (bounds) {
    const float scale = (float)(1. / (double)g->voxel);
    for (int i = 0; i < 6; ++i) bbv[i] = f2s(bounds[i] * scale);
    bb = bbv;
  }
  const float half = 0.5f * g->voxel;
  int64_t n = 0;
  for (int e = 0; e < NUM_ENTRY; ++e) {
    const entry* b = &g->table[e];
    if (!local_idx(b->idx) || !block_selected(g, b->pos, bb, NULL)) continue;
    const s3 base = block_to_point(b->pos);
    for (int lz = -1; lz < BLOCK_LEN; ++lz)
      for (int ly = -1; ly < BLOCK_LEN; ++ly)
        for (int lx = -1; lx < BLOCK_LEN; ++lx) {
          float val[8];
          int owner_found = 0, mine = 0;
          for (int i = 0; i < 8; ++i) {
            const s3 p = {(int16_t)(base.x + lx + (i & 1)), (int16_t)(base.y + ly + ((i >> 1) & 1)),
                          (int16_t)(base.z + lz + ((i >> 2) & 1))};
            const s3 pb = point_to_block(p);
            int64_t pe = -1;
            const int sel = block_selected(g, pb, bb, &pe);
            if (sel && !owner_found) {
              owner_found = 1;
              mine = pe == e;
            }
            val[i] = missing;
            if (sel) {
              const int64_t a = ((int64_t)g->table[pe].idx << BLOCK_VOLUME_BITS) +
                                offset_to_index(p.x & 7, p.y & 7, p.z & 7);
              if ((int)g->rgbw[a * 4 + 3] >= min_weight) val[i] = g->tsdf[a];
            }
          }
          if (!mine) continue;
          int cube = 0;
          for (int i = 0; i < 8; ++i)
            if (val[i] < 0) cube |= 1 << i;
          const int nt = ora_mc_ntri()[cube];
          for (int t = 0; t < nt; ++t) {
            if (out && n < capacity) {
              float* w = &out[n * 9];
              for (int k = 0; k < 3; ++k) {
                const int ed = ora_mc_tri()[cube * 15 + 3 * t + k];
                const int a = ora_mc_edge(ed, 0), bc = ora_mc_edge(ed, 1);
                const int gx = base.x + lx, gy = base.y + ly, gz = base.z + lz;
                float pa[3] = {(float)(gx + (a & 1)) * g->voxel + half,
                               (float)(gy + ((a >> 1) & 1)) * g->voxel + half,
                               (float)(gz + ((a >> 2) & 1)) * g->voxel + half};
                const float pbv[3] = {(float)(gx + (bc & 1)) * g->voxel + half,
                                      (float)(gy + ((bc >> 1) & 1)) * g->voxel + half,
                                      (float)(gz + ((bc >> 2) & 1)) * g->voxel + half};
                const int axis = (a ^ bc) == 1 ? 0 : (a ^ bc) == 2 ? 1 : 2;
                const float tt = val[a] / (val[a] - val[bc]);
                pa[axis] = pa[axis] + tt * (pbv[axis] - pa[axis]);
                w[3 * k + 0] = pa[0];
                w[3 * k + 1] = pa[1];
                w[3 * k + 2] = pa[2];
              }
            }
            ++n;
          }
        }
  }
  return n;
}

/* ---------------------------------------------------------------------------------------------
 * DISINFSystem::feed_rgbd_frame preprocessing (disinfect_slam/disinfect_slam.cc:31-64).
 * OpenCV 4.x cv::resize (modules/imgproc/src/resize.cpp), not vendored here -- parity unpinned
 * beyond this restatement of its published algorithm: with fx = fy = 0.5 and INTER_LINEAR on an
 * even-sized image, resize() switches to INTER_AREA ("interpolation == INTER_LINEAR &&
 * is_area_fast && iscale_x == 2 && iscale_y == 2"), whose fast path (resizeAreaFast_ with
 * ResizeAreaFastVec, fast_mode for 1 / 3 channels) writes (a + b + c + d + 2) >> 2 of each 2x2
 * block per channel for both CV_8U and CV_16U. convertTo(CV_32FC1, alpha) is
 * (float)src * (float)alpha + 0 (cvtScale_, one rounding). The mask loop zeroes depth where the
 * resized mask is 0 (:46-58).
 * --------------------------------------------------------------------------------------------- */
void ora_rgbd_half(const uint8_t* rgb, const uint16_t* depth, const uint8_t* mask, int W, int H,
                   float depth_factor, uint8_t* rgb_out, float* depth_out) {
  const int w = W / 2, h = H / 2;
  const float alpha = (float)(1. / (double)depth_factor);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t i0 = (size_t)(2 * y) * W + 2 * x, i1 = i0 + W;
      for (int c = 0; c < 3; ++c)
        rgb_out[((size_t)y * w + x) * 3 + c] =
            (uint8_t)((rgb[i0 * 3 + c] + rgb[(i0 + 1) * 3 + c] + rgb[i1 * 3 + c] + rgb[(i1 + 1) * 3 + c] + 2) >> 2);
      const int dv = (depth[i0] + depth[i0 + 1] + depth[i1] + depth[i1 + 1] + 2) >> 2;
      float d = (float)(uint16_t)dv * alpha;
      if (mask) {
        const int mv = (mask[i0] + mask[i0 + 1] + mask[i1] + mask[i1 + 1] + 2) >> 2;
        if (mv == 0) d = 0.0f;
      }
      depth_out[(size_t)y * w + x] = d;
    }
}
