// tsdf_device.h -- device-side data layout and float math of the MI355X TSDF engine.
//
// Layout in HBM (one engine = one GPU shard):
//   table    : 2^22 hash entries x 16 B {int16 x, y, z, offset; int32 idx; int32 pad}; the two
//              entries of a bucket share one 32-B segment (reference VoxelBlock is 12 B AoS,
//              voxel_mem.cuh:73-93; NUM_BUCKET 2^21 x 2, voxel_hash.cuh:12-25).
//   lock_tag : 2^21 u32 bucket locks, "locked" == current lock epoch (no per-launch reset pass;
//              reference resets 8 MiB twice per frame, voxel_tsdf.cu:385,487).
//   pool     : 2^bits voxel blocks x 6 KiB, block-major {f32 tsdf[512] | f32 prob[512] |
//              u8x4 rgbw[512]} so one block's state is one contiguous 6 KiB run (reference: three
//              SoA arrays of 2^27 voxels, voxel_mem.cu:13-27). prob is VoxelSEGM::probability
//              (voxel_types.cuh:36-43) itself, updated with the reference's own float chain.
//   occ      : 2^22-bit occupancy bitmap of the table (replaces the full 48 MiB table scans of
//              check_visibility_kernel / check_valid_kernel with a 512 KiB bitmap sweep).
//
// Float math restates utils/cuda/{camera,lie_group}.cuh with Eigen 3.3's evaluation order; the
// library is compiled with -ffp-contract=off and IEEE division / sqrt so results are bit-identical
// to the CPU oracle (oracle/tsdf_oracle.c), the semantic update's logf / expf included (sem_logf /
// sem_expf below restate the oracle's fixed float algorithms, oracle/ora_math.c).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>


namespace tsdf {

constexpr int kBlockLenBits = 3;
constexpr int kBlockLen = 8;
constexpr int kBlockVolume = 512;
constexpr int kBlockVolumeBits = 9;
constexpr int kNumBucketBits = 21;
constexpr uint32_t kNumBucket = 1u << kNumBucketBits;
constexpr uint32_t kBucketMask = kNumBucket - 1;
constexpr uint32_t kNumEntry = kNumBucket * 2;
constexpr uint32_t kEntryMask = kNumEntry - 1;
constexpr uint32_t kOccWords = kNumEntry / 64;
constexpr int kBlockBytes = kBlockVolume * 12;  // 6 KiB per voxel block
constexpr int kProbOffset = kBlockVolume * 4;   // byte offsets inside a block record (probability)
constexpr int kRgbwOffset = kBlockVolume * 8;
constexpr uint32_t kNewKeyCap = 1u << 17;       // unique new blocks per frame
constexpr int kMaxDdaSamples = 6;               // DDA samples per pixel the ingest kernel supports
constexpr int64_t kMaxOrderRange = 8192ll * 1024;  // candidate order space the resolver streams
constexpr int kResolveThreads = 1024;
constexpr int kIntegrateGrid = 2048;  // k_integrate workgroups (persistent grid-stride) at most
// k_integrate workgroup size: 4 waves, two per visible block (1024-thread workgroups measured
// slower: 24.3 against 17.5 us)
constexpr int kIntegrateThreads = 256;
// carve candidates a k_integrate workgroup buffers in LDS before publishing them at its end (more
// are published as they come)
constexpr int kIntegrateCandBuf = 16;

struct f3 {
  float x, y, z;
};
struct quatf {
  float x, y, z, w;
};

// Per-frame constants, passed by value (host computes K^-1 and world_T_cam exactly like the
// reference does on the host: CameraParams ctor camera.cuh:65, SE3::Inverse lie_group.cuh:22).
struct FrameParams {
  float fx, fy, cx, cy;      // intrinsics
  float ifx, ify, icx, icy;  // intrinsics_inv
  quatf cq;                  // cam_T_world
  f3 ct;
  quatf wq;                  // world_T_cam
  f3 wt;
  float voxel, trunc, max_depth;
  float inv_trunc, inv_voxel, inv_max_depth;  // RN(1 / .), host IEEE divides (quot_const)
  int W, H;
  int maxs;                  // DDA samples reserved per pixel in the candidate order space
  int shard_index, shard_count;
  int tile_lo, tile_hi;      // pixel tiles whose DDA this engine runs (a shard's slice, else all)
  int tail;                  // what the last workgroup of a frame kernel does (kTail*)
  int slot_cap;              // kTailPack: records the exchange slot holds
  struct ShardRec* slot;     // kTailPack: this shard's exchange slot (keys / carve candidates)
  int pack_pixels;           // the ingest writes the pixel records (one volume); else k_integrate
                             // gathers the raw frame below (a shard: no whole-frame pass)
  const float* depth;        // the frame (device pointers)
  const uint8_t* rgb;
  const float* ht;           // NULL: ones (tsdf_module.cc:29-33)
  const float* lt;
  int row0, nrows;           // raycast: the rows [row0, row0 + nrows) of the W x H camera it renders
  int pix_off;               // this frame's pixel records: D.pixA + pix_off (one of the two
                             //   buffers: a pipelined frame's are written while the previous frame reads its own)
};
// the last-arriving workgroup of k_ingest_dda / k_integrate: resolve (allocation / carving) or, in a
// shard's frame with an exchange after the kernel, pack the keys / candidates into the slot
constexpr int kTailResolve = 0, kTailPack = 1;

// Sharded volume: every shard keeps the whole hash index, so bucket locks and table
// layout evolve exactly as in one volume; a block's voxels live only on its owner. The other
// shards' entry of it carries kForeignIdx: occupied for Allocate / Delete (idx >= 0), missing for
// every reader (local_idx false).
constexpr int32_t kForeignIdx = 0x7FFFFFFF;
__device__ __host__ __forceinline__ bool local_idx(int32_t idx) { return idx >= 0 && idx != kForeignIdx; }

// one exchanged record of a sharded frame (16 B): a new block key with its candidate order, or a
// carve candidate with its hash entry. A slot is (cap + 1) records, record 0 a header whose `val`
// holds the count; an inbox is shard_count slots, slot s written by shard s.
// one entry of the new-key list: the key and its new-key-set slot (16 B, published with two
// 8-byte agent-scope stores)
struct alignas(16) NkEnt {
  unsigned long long key;
  unsigned long long slot;
};

struct alignas(16) ShardRec {
  int16_t x, y, z, pad;
  uint32_t val;   // candidate order (keys) / hash entry (carve candidates) / count (header)
  uint32_t zero;
};

// one visible block: snapshot of its hash entry (gather_visible_blocks_kernel copies entries)
struct alignas(16) VisRec {
  int16_t x, y, z, pad;
  int32_t idx;
  int32_t entry;
};

struct DevCounters {
  int32_t free_count;     // VoxelMemPool::num_free_blocks_
  uint32_t lock_epoch;    // current lock epoch (one per allocate / delete launch)
  int32_t nk_count;       // unique new keys inserted by the DDA this frame
  int32_t n_fresh;        // blocks acquired by the hash-level test path
  int32_t n_vis;          // visible blocks this frame
  int32_t n_cand;         // carve candidates this frame
  uint32_t status;        // TSDF_STATUS_* bits
  int32_t last_alloc;
  int32_t last_deleted;
  int32_t last_new_keys;
  unsigned long long last_updated;
  unsigned long long total_visible;
  unsigned long long total_updated;
  unsigned long long total_alloc;
  unsigned long long total_deleted;
  unsigned long long frames;
  unsigned long long integrate_ticks;  // sum of k_integrate device durations (100 MHz clock)
  int32_t n_keys_in;      // sharded frames: key records merged from the exchange (last frame)
  int32_t n_pend;         // a shard's owned entries left without voxels (pool exhausted) this frame
  unsigned long long ingest_ticks;          // k_ingest_dda start -> last arrival (100 MHz clock)
  unsigned long long resolve_alloc_ticks;   // resolve_alloc_wg durations
  unsigned long long resolve_delete_ticks;  // resolve_delete_wg durations
};

// ------------------------------------------------------------------------------------------
// float math (bit-exact restatement; see header comment)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {  // Eigen MatrixBase::cross
  f3 r;
  r.x = a.y * b.z - a.z * b.y;
  r.y = a.z * b.x - a.x * b.z;
  r.z = a.x * b.y - a.y * b.x;
  return r;
}
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
__device__ __forceinline__ f3 qrot(quatf q, f3 v) {  // QuaternionBase::_transformVector
  const f3 qv = {q.x, q.y, q.z};
  f3 uv = cross3(qv, v);
  uv.x += uv.x;
  uv.y += uv.y;
  uv.z += uv.z;
  const f3 c = cross3(qv, uv);
  f3 r;
  r.x = (v.x + q.w * uv.x) + c.x;
  r.y = (v.y + q.w * uv.y) + c.y;
  r.z = (v.z + q.w * uv.z) + c.z;
  return r;
}
__device__ __forceinline__ f3 se3_apply(quatf q, f3 t, f3 v) {  // SE3::Apply, lie_group.cuh:30
  f3 r = qrot(q, v);
  r.x = r.x + t.x;
  r.y = r.y + t.y;
  r.z = r.z + t.z;
  return r;
}
// float -> integer conversions with PTX cvt.rzi semantics (truncate, saturate, NaN -> 0), which
// is exactly what v_cvt_i32_f32 / v_cvt_u32_f32 do in hardware.
__device__ __forceinline__ int32_t f2i(float f) {  // cvt.rzi.s32.f32
  int32_t r;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
  return r;
}
// f2s(roundf(f)) in a few operations: for 1/2 <= |f| < 2^22, f + copysign(1/2, f) truncates to
// roundf(f) (the sum is exact, or rounds without reaching the next integer); |f| < 1/2 gives 0 (the
// sum could round up to 1); from 2^15 on the int16 result saturates either way, so no other range
// needs its own form (NaN -> 0 as f2s). Written as selects on the converted value: the ternary on
// the float operand compiled to three exec-masked branches per call, and the raycast rounds three
// coordinates per march step. tests/test_gpu_numerics.py checks it on every float.
__device__ __forceinline__ int16_t round_s16(float f) {
  const int r = min(32767, max(-32768, f2i(f + __builtin_copysignf(0.5f, f))));
  return (int16_t)(fabsf(f) < 0.5f ? 0 : r);
}

__device__ __forceinline__ int16_t f2s(float f) {  // cvt.rzi.s16.f32
  return (int16_t)min(32767, max(-32768, f2i(f)));
}
__device__ __forceinline__ uint8_t f2u8(float f) {  // cvt.rzi.u8.f32
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(f));
  return (uint8_t)min(r, 255u);
}

// ---- exact quotients without the full IEEE divide sequence (11 VALU ops). Both helpers return
// bit-for-bit what the correctly rounded a / b would give; libtsdf_selfcheck checks them against
// the IEEE divide exhaustively / on adversarial samples (tests/test_gpu_numerics.py). ----

// f2i(roundf(a / b)) -- the integer the reference gets from roundf of the IEEE quotient followed
// by a truncating cvt -- from the reciprocal estimate rb = v_rcp(b) (1 ulp). q = a*rb is within
// 2^-22 |q| of RN(a/b); rounding the two perturbations q (1 +- 2^-20) half away from zero
// (fma with +-1/2, then the truncating cvt) brackets roundf of every value in between, so when
// both land on the same integer it is the answer (the fma rounding error is covered for |q| >= 1/7,
// and below that both give 0). Otherwise -- near k + 1/2, or |b| out of range -- the lane takes
// the IEEE divide. Saturation and NaN -> 0 match cvt.rzi in both paths.
__device__ __forceinline__ int32_t round_quot_i(float a, float b, float rb) {
  const float q = a * rb;
  const float h = __builtin_copysignf(0.5f, q);
  const int32_t i1 = f2i(__builtin_fmaf(q, 1.0f + 0x1p-20f, h));
  const int32_t i2 = f2i(__builtin_fmaf(q, 1.0f - 0x1p-20f, h));
  if (__builtin_expect(i1 == i2 && fabsf(b) < 0x1p100f, 1)) return i1;
  return f2i(roundf(a / b));
}
// f2u8(roundf(a / b)): the saturating u8 cvt of the same rounded quotient
__device__ __forceinline__ uint32_t round_quot_u8(float a, float b, float rb) {
  return (uint32_t)min(255, max(0, round_quot_i(a, b, rb)));
}

// ---- the same helpers on voxel pairs (ext_vector float2 arithmetic: IEEE per element, so results are
// identical to the scalar forms; plain fp32 instructions: the library is built without packed fp32,
// Makefile NOPK); lanes with act == false never take the IEEE fallback (their results are discarded by
// the caller) ----
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f v2(float a, float b) {
  v2f r;
  r.x = a;
  r.y = b;
  return r;
}
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ void round_quot_i2(v2f a, v2f b, v2f rb, bool act0, bool act1,
                                              int32_t& o0, int32_t& o1) {
  const v2f q = a * rb;
  const v2f h = v2(__builtin_copysignf(0.5f, q.x), __builtin_copysignf(0.5f, q.y));
  const v2f f1 = vfma(q, v2(1.0f + 0x1p-20f, 1.0f + 0x1p-20f), h);
  const v2f f2 = vfma(q, v2(1.0f - 0x1p-20f, 1.0f - 0x1p-20f), h);
  o0 = f2i(f1.x);
  o1 = f2i(f1.y);
  if (__builtin_expect(act0 && !(o0 == f2i(f2.x) && fabsf(b.x) < 0x1p100f), 0))
    o0 = f2i(roundf(a.x / b.x));
  if (__builtin_expect(act1 && !(o1 == f2i(f2.y) && fabsf(b.y) < 0x1p100f), 0))
    o1 = f2i(roundf(a.y / b.y));
}

__device__ __forceinline__ v2f quot_const2(v2f a, float b, float rb, bool act0, bool act1) {
  const v2f q = a * rb;
  const v2f r = vfma(-q, v2(b, b), a);
  v2f o = vfma(r, v2(rb, rb), q);
  const float fa0 = fabsf(a.x), fq0 = fabsf(q.x), fa1 = fabsf(a.y), fq1 = fabsf(q.y);
  if (__builtin_expect(act0 && !(fa0 > 0x1p-60f && fa0 < 0x1p60f && fq0 > 0x1p-60f && fq0 < 0x1p60f), 0))
    o.x = a.x / b;
  if (__builtin_expect(act1 && !(fa1 > 0x1p-60f && fa1 < 0x1p60f && fq1 > 0x1p-60f && fq1 < 0x1p60f), 0))
    o.y = a.y / b;
  return o;
}

// f2i(roundf(a / b)) on voxel pairs for a >= 0 and 0 < b < 2^100 (or the NaN of 0 / 0, which
// both paths turn into 0): round_quot_i2 with the half-away offset fixed at +1/2 and no |b| test
__device__ __forceinline__ void round_quot_pos2(v2f a, v2f b, v2f rb, bool act0, bool act1,
                                                int32_t& o0, int32_t& o1) {
  const v2f q = a * rb;
  const v2f f1 = vfma(q, v2(1.0f + 0x1p-20f, 1.0f + 0x1p-20f), v2(0.5f, 0.5f));
  const v2f f2 = vfma(q, v2(1.0f - 0x1p-20f, 1.0f - 0x1p-20f), v2(0.5f, 0.5f));
  o0 = f2i(f1.x);
  o1 = f2i(f1.y);
  if (__builtin_expect(act0 && o0 != f2i(f2.x), 0)) o0 = f2i(roundf(a.x / b.x));
  if (__builtin_expect(act1 && o1 != f2i(f2.y), 0)) o1 = f2i(roundf(a.y / b.y));
}

// RN(a / b) on voxel pairs with y = v_rcp(b): the compiler's IEEE f32 division expansion
// (Newton-refined reciprocal, quotient, two residual corrections) without its v_div_scale /
// v_div_fmas / v_div_fixup range handling, which are identities while |a| and |b| lie in
// [2^-40, 2^40] (every residual is then a normal float or 0); lanes outside that range take the
// IEEE divide. Checked against a / b by libtsdf_selfcheck (tests/test_gpu_numerics.py).
__device__ __forceinline__ v2f div_pair(v2f a, v2f b, v2f y, bool act0, bool act1) {
  const v2f e = vfma(-b, y, v2(1.0f, 1.0f));
  const v2f y1 = vfma(e, y, y);
  const v2f q = a * y1;
  const v2f r = vfma(-b, q, a);
  const v2f q1 = vfma(r, y1, q);
  const v2f r1 = vfma(-b, q1, a);
  v2f o = vfma(r1, y1, q1);
  const float fa0 = fabsf(a.x), fb0 = fabsf(b.x), fa1 = fabsf(a.y), fb1 = fabsf(b.y);
  if (__builtin_expect(act0 && !(fa0 >= 0x1p-40f && fa0 <= 0x1p40f && fb0 >= 0x1p-40f && fb0 <= 0x1p40f), 0))
    o.x = a.x / b.x;
  if (__builtin_expect(act1 && !(fa1 >= 0x1p-40f && fa1 <= 0x1p40f && fb1 >= 0x1p-40f && fb1 <= 0x1p40f), 0))
    o.y = a.y / b.y;
  return o;
}

// div_pair that also takes a == 0 on its fast path (the Newton expansion gives the signed zero
// exactly); the semantic update's numerators are 0 wherever w_old == 0 and ln ht == 0.
__device__ __forceinline__ v2f div_pair0(v2f a, v2f b, v2f y, bool act0, bool act1) {
  const v2f e = vfma(-b, y, v2(1.0f, 1.0f));
  const v2f y1 = vfma(e, y, y);
  const v2f q = a * y1;
  const v2f r = vfma(-b, q, a);
  const v2f q1 = vfma(r, y1, q);
  const v2f r1 = vfma(-b, q1, a);
  v2f o = vfma(r1, y1, q1);
  const float fa0 = fabsf(a.x), fb0 = fabsf(b.x), fa1 = fabsf(a.y), fb1 = fabsf(b.y);
  const bool ok0 = (fa0 == 0.0f || (fa0 >= 0x1p-40f && fa0 <= 0x1p40f)) && fb0 >= 0x1p-40f && fb0 <= 0x1p40f;
  const bool ok1 = (fa1 == 0.0f || (fa1 >= 0x1p-40f && fa1 <= 0x1p40f)) && fb1 >= 0x1p-40f && fb1 <= 0x1p40f;
  if (__builtin_expect(act0 && !ok0, 0)) o.x = a.x / b.x;
  if (__builtin_expect(act1 && !ok1, 0)) o.y = a.y / b.y;
  return o;
}

// ---- logf / expf of the semantic update (voxel_tsdf.cu:196-202). CUDA's own (libdevice, <= 1 /
// 2 ulp) cannot be reproduced here, and the reference's float chain is ill-conditioned near p = 1
// (one ulp of p there moves a later p by up to ~1e-2), so the oracle fixes both functions as
// explicit single-precision algorithms (oracle/ora_math.c, < 0.87 / 0.99 ulp from the correctly
// rounded values over every input) and these are the same operations -- frexp, rint, ldexp, fma and
// + - * with one IEEE rounding each -- so they return the oracle's bits for all 2^32 inputs
// (libtsdf_selfcheck digests, tests/test_gpu_numerics.py). Pairs run as v2f pairs (plain fp32 instructions: the library is built without packed fp32).
constexpr float kSemQ[9] = {0x1.555554p-2f,  -0x1.fffffcp-3f, 0x1.999d5ap-3f,  -0x1.555b4ap-3f, 0x1.23d21ap-3f,
                            -0x1.fcf4c6p-4f, 0x1.dea282p-4f,  -0x1.d635bcp-4f, 0x1.1d8ea4p-4f};
constexpr float kSemE[6] = {0x1p-1f, 0x1.555556p-3f, 0x1.5554eap-5f, 0x1.1110e0p-7f, 0x1.6d4316p-10f,
                            0x1.a124e4p-13f};
constexpr float kSemLn2Hi = 0x1.62e4p-1f;     // 16 significant bits: e * kSemLn2Hi is exact
constexpr float kSemLn2Lo = 0x1.7f7d1cp-20f;
constexpr float kSemInvLn2 = 0x1.715476p+0f;
constexpr float kSemSqrtHalf = 0x1.6a09e6p-1f;

// x = z 2^k with z in [sqrt(1/2), sqrt(2)) for positive finite x: the oracle's frexp + doubling, done
// on the bits (a subnormal x is scaled by 2^24 first, k compensated) -- the same z and k, so the same
// f = z - 1 (exact) and dk = k. Other inputs give garbage, replaced by the callers' special cases.
__device__ __forceinline__ float sem_log_reduce(float x, float& dk) {
  const bool sub = x < 0x1p-126f;
  const uint32_t ix = __float_as_uint(sub ? x * 0x1p24f : x);
  const int32_t k = (int32_t)(ix - 0x3f3504f3u) >> 23;  // 0x3f3504f3 = kSemSqrtHalf
  dk = (float)(sub ? k - 24 : k);
  return __uint_as_float(ix - ((uint32_t)k << 23)) - 1.0f;
}
// log1p(f) - f = f^3 Q(f) - f^2 / 2 and the result, on pairs (the oracle's operations)
__device__ __forceinline__ v2f sem_log_core2(v2f f, v2f dk) {
  v2f q = v2(kSemQ[8], kSemQ[8]);
#pragma unroll
  for (int i = 7; i >= 0; --i) q = vfma(q, f, v2(kSemQ[i], kSemQ[i]));
  const v2f f2 = f * f;
  const v2f hf2 = v2(0.5f, 0.5f) * f2;
  const v2f t = vfma(f2 * f, q, -hf2);
  return vfma(dk, v2(kSemLn2Hi, kSemLn2Hi), vfma(dk, v2(kSemLn2Lo, kSemLn2Lo), t) + f);
}
// logf of x in [0, 1] or NaN (the update's p and 1 - p): 0 -> -inf, NaN -> NaN
__device__ __forceinline__ v2f sem_log_unit2(v2f x) {
  float dk0, dk1;
  const v2f f = v2(sem_log_reduce(x.x, dk0), sem_log_reduce(x.y, dk1));
  const v2f y = sem_log_core2(f, v2(dk0, dk1));
  const float ninf = -__builtin_inff();
  return v2(x.x > 0.0f ? y.x : (x.x == 0.0f ? ninf : x.x), x.y > 0.0f ? y.y : (x.y == 0.0f ? ninf : x.y));
}
// logf of any float: -0 / 0 -> -inf, negative -> NaN, +inf -> +inf, NaN -> NaN
__device__ __forceinline__ float sem_log_special(float x, float y) {
  y = x == __builtin_inff() ? x : y;
  return x > 0.0f ? y : (x == 0.0f ? -__builtin_inff() : __builtin_nanf(""));
}
__device__ __forceinline__ v2f sem_logf2(v2f x) {
  float dk0, dk1;
  const v2f f = v2(sem_log_reduce(x.x, dk0), sem_log_reduce(x.y, dk1));
  const v2f y = sem_log_core2(f, v2(dk0, dk1));
  return v2(sem_log_special(x.x, y.x), sem_log_special(x.y, y.y));
}
__device__ __forceinline__ float sem_logf(float x) { return sem_logf2(v2(x, x)).x; }
// expf: the oracle's thresholds (x > 89 -> inf, x < -104 -> 0) are met by clamping x to
// [-104.5, 89.5] and evaluating (e^89.5 overflows to inf, e^-104 and below round to 0 in ldexp), NaN
// -> NaN
__device__ __forceinline__ v2f sem_expf2(v2f x) {
  const v2f xc = v2(__builtin_amdgcn_fmed3f(x.x, -104.5f, 89.5f), __builtin_amdgcn_fmed3f(x.y, -104.5f, 89.5f));
  const v2f xk = xc * v2(kSemInvLn2, kSemInvLn2);
  const v2f n = v2(__builtin_rintf(xk.x), __builtin_rintf(xk.y));
  v2f r = vfma(-n, v2(kSemLn2Hi, kSemLn2Hi), xc);
  r = vfma(-n, v2(kSemLn2Lo, kSemLn2Lo), r);
  v2f p = v2(kSemE[5], kSemE[5]);
#pragma unroll
  for (int i = 4; i >= 0; --i) p = vfma(p, r, v2(kSemE[i], kSemE[i]));
  const v2f s = vfma(r * r, p, r) + v2(1.0f, 1.0f);
  const float y0 = __builtin_amdgcn_ldexpf(s.x, (int)n.x), y1 = __builtin_amdgcn_ldexpf(s.y, (int)n.y);
  return v2(x.x != x.x ? x.x : y0, x.y != x.y ? x.y : y1);
}
__device__ __forceinline__ float sem_expf(float x) { return sem_expf2(v2(x, x)).x; }

// ---- the semantic update's fast path (k_frame / k_integrate): the same operations without the
// special-value handling, exact where every operand stays in range: p and 1 - p normal, the
// numerators in {0} U [2^-40, 2^40] and wc in [2^-40, 2^40] (div_pair's exact range, zero added: the
// expansion returns the signed zero), P in [2^-40, 2^40] and P + N <= 2^40. A voxel qualifies when its
// pixel does (sem_pixel_fast: ht, lt in [2^-39, 1], so their logs lie in [-27.03, 0], and d <=
// 0.9999 max_depth, so w_new >= 4e-4) and p lies in [2^-39, 1) (sem_voxel_fast). Then both numerators
// are sums of two non-positive terms, each 0 or of magnitude >= 4e-4 * 5.96e-8 (the smallest |ln x| of
// a float x < 1) > 2^-40, and at most 44 * 27.03; wc lies in [4e-4, 44]; the quotients in [-27.03, 0],
// so P and N lie in [e^-27.03, 1] (> 2^-40) and P + N <= 2. Every other voxel is recomputed with
// sem_update_exact.
__device__ __forceinline__ bool sem_pixel_fast(float h, float l, float d, float max_depth) {
  return h >= 0x1p-39f && h <= 1.0f && l >= 0x1p-39f && l <= 1.0f && d <= max_depth * 0.9999f;
}
__device__ __forceinline__ bool sem_voxel_fast(bool pixel_fast, float p) {
  return pixel_fast && p >= 0x1p-39f && p < 1.0f;
}
__device__ __forceinline__ float sem_log_reduce_n(float x, float& dk) {  // x normal, positive
  const uint32_t ix = __float_as_uint(x);
  const int32_t k = (int32_t)(ix - 0x3f3504f3u) >> 23;
  dk = (float)k;
  return __uint_as_float(ix - ((uint32_t)k << 23)) - 1.0f;
}
__device__ __forceinline__ v2f sem_log_fast2(v2f x) {
  float dk0, dk1;
  const v2f f = v2(sem_log_reduce_n(x.x, dk0), sem_log_reduce_n(x.y, dk1));
  return sem_log_core2(f, v2(dk0, dk1));
}
__device__ __forceinline__ v2f sem_exp_fast2(v2f x) {  // x in [-104, 89]
  const v2f xk = x * v2(kSemInvLn2, kSemInvLn2);
  const v2f n = v2(__builtin_rintf(xk.x), __builtin_rintf(xk.y));
  v2f r = vfma(-n, v2(kSemLn2Hi, kSemLn2Hi), x);
  r = vfma(-n, v2(kSemLn2Lo, kSemLn2Lo), r);
  v2f p = v2(kSemE[5], kSemE[5]);
#pragma unroll
  for (int i = 4; i >= 0; --i) p = vfma(p, r, v2(kSemE[i], kSemE[i]));
  const v2f s = vfma(r * r, p, r) + v2(1.0f, 1.0f);
  return v2(__builtin_amdgcn_ldexpf(s.x, (int)n.x), __builtin_amdgcn_ldexpf(s.y, (int)n.y));
}
// div_pair's expansion in two parts: the refined reciprocal y1 of b (shared by every numerator over
// the same b), then RN(a / b) for |a| in {0} U [2^-40, 2^40], |b| in [2^-40, 2^40]
__device__ __forceinline__ v2f div_refine(v2f b, v2f y) { return vfma(vfma(-b, y, v2(1.0f, 1.0f)), y, y); }
__device__ __forceinline__ v2f div_expand(v2f a, v2f b, v2f y1) {
  const v2f q = a * y1;
  const v2f r = vfma(-b, q, a);
  const v2f q1 = vfma(r, y1, q);
  const v2f r1 = vfma(-b, q1, a);
  return vfma(r1, y1, q1);
}
// the whole update with every special case (IEEE divides, sem_logf / sem_expf)
__device__ __forceinline__ float sem_update_exact(float p, float w_old, float w_new, float wc, float lnh,
                                                  float lnl) {
  const float sp = sem_expf((w_old * sem_logf(p) + w_new * lnh) / wc);
  const float sn = sem_expf((w_old * sem_logf(1.0f - p) + w_new * lnl) / wc);
  return sp / (sp + sn);
}

// min(roundf(w), 40) as an integer for 0 <= w < 2^23 (the weight update, voxel_tsdf.cu:188):
// floor(RN(w + pred(1/2))) == roundf(w) on that whole range (pred(1/2) = 0x1.fffffep-2 keeps
// RN(0.49999997 + 1/2) below 1; at every larger w the sum's rounding never crosses an integer
// the exact sum does not reach). Exhaustively checked by tests/test_cpu_lib.py.
__device__ __forceinline__ uint32_t weight_round_cap(float w, uint32_t cap) {
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(w));
  return min(r, cap);
}

// RN(a / b) where the caller only compares the quotient with 0 and with the float c: the
// estimate a * rcp(b) is returned when it provably lies on the same side of 0 and of c as the IEEE
// quotient (distance to c above 2^-20 |q|, |q| and |b| in range), else the IEEE quotient.
__device__ __forceinline__ float quot_for_cmp(float a, float b, float rb, float c) {
  const float q = a * rb;
  const float fq = fabsf(q);
  if (__builtin_expect(fq > 0x1p-100f && fq < 0x1p100f && fabsf(b) < 0x1p100f &&
                           fabsf(q - c) > fq * 0x1p-20f, 1))
    return q;
  return a / b;
}

// RN(a / b) for a frame-constant divisor b with rb = RN(1 / b) computed on the host: Markstein's
// correction q + (a - b q) rb (two fma) is the correctly rounded quotient when no intermediate
// leaves the normal range; |a| or |q| outside [2^-60, 2^60] (incl. 0, inf, NaN) takes the IEEE
// divide.
__device__ __forceinline__ float quot_const(float a, float b, float rb) {
  const float q = a * rb;
  const float fa = fabsf(a), fq = fabsf(q);
  if (__builtin_expect(fa > 0x1p-60f && fa < 0x1p60f && fq > 0x1p-60f && fq < 0x1p60f, 1)) {
    const float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, rb, q);
  }
  return a / b;
}

// 16-B pool-state accesses: plain cached loads and stores. TSDF_STREAM_STORES / _LOADS build
// nontemporal forms for timing studies (measured slower on MI355X: 18.3 / 20.2 us against 17.8 us
// for k_integrate at the bench workload).
typedef float v4f __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 pool_ld(const uint8_t* p) {
#if !defined(TSDF_STREAM_LOADS)
  return *reinterpret_cast<const float4*>(p);
#else
  const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
#endif
}
__device__ __forceinline__ uint4 pool_ldu(const uint8_t* p) {
#if !defined(TSDF_STREAM_LOADS)
  return *reinterpret_cast<const uint4*>(p);
#else
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#endif
}
__device__ __forceinline__ void pool_st(uint8_t* p, float4 v) {
#if !defined(TSDF_STREAM_STORES)
  *reinterpret_cast<float4*>(p) = v;
#else
  const v4f t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<v4f*>(p));
#endif
}
__device__ __forceinline__ void pool_stu(uint8_t* p, uint4 v) {
#if !defined(TSDF_STREAM_STORES)
  *reinterpret_cast<uint4*>(p) = v;
#else
  const v4u t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<v4u*>(p));
#endif
}

// voxel_hash.cu:31-35
__device__ __host__ __forceinline__ uint32_t hash_block(int16_t x, int16_t y, int16_t z) {
  return (((uint32_t)(int32_t)x * 73856093u) ^ ((uint32_t)(int32_t)y * 19349669u) ^
          ((uint32_t)(int32_t)z * 83492791u)) & kBucketMask;
}
// shard owner of a block: a 4^3-block brick (16 cm at 5 mm) hashed to a GPU
__device__ __host__ __forceinline__ uint32_t brick_owner(int16_t x, int16_t y, int16_t z,
                                                        uint32_t shards) {
  uint32_t h = ((uint32_t)(int32_t)(x >> 2) * 0x9E3779B1u) ^
               ((uint32_t)(int32_t)(y >> 2) * 0x85EBCA77u) ^
               ((uint32_t)(int32_t)(z >> 2) * 0xC2B2AE3Du);
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  return shards <= 1 ? 0u : h % shards;
}

__device__ __forceinline__ uint64_t pack_key(int16_t x, int16_t y, int16_t z) {
  return (uint64_t)(uint16_t)x | ((uint64_t)(uint16_t)y << 16) | ((uint64_t)(uint16_t)z << 32) |
         (1ull << 48);
}
__device__ __forceinline__ void unpack_key(uint64_t k, int16_t& x, int16_t& y, int16_t& z) {
  x = (int16_t)(k & 0xFFFF);
  y = (int16_t)((k >> 16) & 0xFFFF);
  z = (int16_t)((k >> 32) & 0xFFFF);
}

// hash entry as loaded from the table (int4 = 16 B)
struct Ent {
  int16_t x, y, z, off;
  int32_t idx;
};
__device__ __forceinline__ Ent load_ent(const int4* table, uint32_t e) {
  const int4 v = table[e];
  Ent r;
  r.x = (int16_t)(v.x & 0xFFFF);
  r.y = (int16_t)((uint32_t)v.x >> 16);
  r.z = (int16_t)(v.y & 0xFFFF);
  r.off = (int16_t)((uint32_t)v.y >> 16);
  r.idx = v.z;
  return r;
}
__device__ __forceinline__ void store_ent(int4* table, uint32_t e, int16_t x, int16_t y, int16_t z,
                                          int16_t off, int32_t idx) {
  int4 v;
  v.x = (int32_t)((uint32_t)(uint16_t)x | ((uint32_t)(uint16_t)y << 16));
  v.y = (int32_t)((uint32_t)(uint16_t)z | ((uint32_t)(uint16_t)off << 16));
  v.z = idx;
  v.w = 0;
  table[e] = v;
}
__device__ __forceinline__ void store_off(int4* table, uint32_t e, int16_t off) {
  // the offset is the high half of the second dword
  uint16_t* p = reinterpret_cast<uint16_t*>(&table[e]) + 3;
  *p = (uint16_t)off;
}
__device__ __forceinline__ void store_off_idx(int4* table, uint32_t e, int16_t off, int32_t idx) {
  uint16_t* p = reinterpret_cast<uint16_t*>(&table[e]) + 3;
  *p = (uint16_t)off;
  reinterpret_cast<int32_t*>(&table[e])[2] = idx;
}

// VoxelHashTable::RetrieveMutable lookup (voxel_hash.cuh:124-161): entry index or -1
__device__ __forceinline__ int32_t find_entry(const int4* __restrict__ table, int16_t x, int16_t y,
                                              int16_t z) {
  const uint32_t e0 = hash_block(x, y, z) << 1;
  const Ent a = load_ent(table, e0);
  if (a.x == x && a.y == y && a.z == z && a.idx >= 0) return (int32_t)e0;
  Ent b = load_ent(table, e0 + 1);
  if (b.x == x && b.y == y && b.z == z && b.idx >= 0) return (int32_t)(e0 + 1);
  uint32_t last = e0 + 1;
  while (b.off) {
    last = (uint32_t)(last + (int32_t)b.off) & kEntryMask;
    b = load_ent(table, last);
    if (b.x == x && b.y == y && b.z == z && b.idx >= 0) return (int32_t)last;
  }
  return -1;
}

// the entry of a block this engine holds voxels for, or -1 (missing, or another shard's block)
__device__ __forceinline__ int32_t find_local(const int4* __restrict__ table, int16_t x, int16_t y,
                                              int16_t z) {
  const int32_t e = find_entry(table, x, y, z);
  return (e >= 0 && local_idx(table[e].z)) ? e : -1;
}

// camera.cuh:47-51 and voxel_tsdf.cu:48-57 is_voxel_visible
__device__ __forceinline__ bool voxel_visible(const FrameParams& P, int16_t gx, int16_t gy,
                                              int16_t gz) {
  const f3 pw = {(float)gx * P.voxel, (float)gy * P.voxel, (float)gz * P.voxel};
  const f3 pc = se3_apply(P.cq, P.ct, pw);
  const float hx = P.fx * pc.x + P.cx * pc.z;
  const float hy = P.fy * pc.y + P.cy * pc.z;
  const float hz = pc.z;
  const float rz = __builtin_amdgcn_rcpf(hz);
  const float u = quot_for_cmp(hx, hz, rz, (float)(P.W - 1));
  const float v = quot_for_cmp(hy, hz, rz, (float)(P.H - 1));
  return u >= 0 && u <= (float)(P.W - 1) && v >= 0 && v <= (float)(P.H - 1) && hz >= 0;
}
// voxel_tsdf.cu:59-80 is_block_visible<Full>
template <bool Full>
__device__ __forceinline__ bool block_visible(const FrameParams& P, int16_t bx, int16_t by,
                                              int16_t bz) {
  const int16_t x = (int16_t)(bx << kBlockLenBits), y = (int16_t)(by << kBlockLenBits),
                z = (int16_t)(bz << kBlockLenBits);
  bool vis = Full;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool v = voxel_visible(P, (int16_t)(x + ((i >> 0) & 1) * (kBlockLen - 1)),
                                 (int16_t)(y + ((i >> 1) & 1) * (kBlockLen - 1)),
                                 (int16_t)(z + ((i >> 2) & 1) * (kBlockLen - 1)));
    if (Full)
      vis = vis && v;
    else
      vis = vis || v;
  }
  return vis;
}

// pixel -> normalised camera ray K^-1 [x, y, 1] (camera.cuh:47-51 with intrinsics_inv)
__device__ __forceinline__ f3 pixel_ray(const FrameParams& P, int x, int y) {
  f3 pc;
  pc.x = P.ifx * (float)x + P.icx * 1.0f;
  pc.y = P.ify * (float)y + P.icy * 1.0f;
  pc.z = 1.0f;
  return pc;
}
// the per-pixel terms of tsdf_integrate_kernel's update (voxel_tsdf.cu:174-201), computed once per
// pixel into the pixel records (one volume) or per voxel from the raw frame (a shard): the same
// operations either way, so the results are identical
//   w_new = (1 - d / max_depth) * 4
__device__ __forceinline__ float pixel_w_new(const FrameParams& P, float d) {
  return (1.0f - quot_const(d, P.max_depth, P.inv_max_depth)) * 4.0f;
}
//   logf(ht), logf(lt) (sem_logf)

}  // namespace tsdf
