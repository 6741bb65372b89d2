// Diagnostic (GPU box): latency of one-workgroup sorts of m keys in LDS (s_memrealtime, 100 MHz):
// plain rank counting, rank counting with 16-B reads unrolled 8x, and a one-wave bitonic network.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ void rank_plain(unsigned long long* a, unsigned long long* tmp, int m) {
  const int t = threadIdx.x;
  const unsigned long long x0 = t < m ? a[t] : ~0ull;
  int r0 = 0;
  for (int j = 0; j < m; ++j) r0 += a[j] < x0;
  if (t < m) tmp[r0] = x0;
  __syncthreads();
  if (t < m) a[t] = tmp[t];
  __syncthreads();
}
__device__ __forceinline__ void rank_unrolled(unsigned long long* a, unsigned long long* tmp, int m) {
  const int t = threadIdx.x;
  const unsigned long long x0 = t < m ? a[t] : ~0ull;
  const uint32_t h0 = (uint32_t)(x0 >> 32);
  if (t == 0 && (m & 1)) a[m] = ~0ull;
  __syncthreads();
  const uint4* a4 = reinterpret_cast<const uint4*>(a);
  int r0 = 0;
  const int np = (m + 1) >> 1;
  int j = 0;
  for (; j + 8 <= np; j += 8) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = a4[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) r0 += (v[u].y < h0) + (v[u].w < h0);
  }
  for (; j < np; ++j) {
    const uint4 v = a4[j];
    r0 += (v.y < h0) + (v.w < h0);
  }
  if (t < m) tmp[r0] = x0;
  __syncthreads();
  if (t < m) a[t] = tmp[t];
  __syncthreads();
}
__device__ __forceinline__ void wave_bitonic(unsigned long long* a, int m) {
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    unsigned long long x = l < m ? a[l] : ~0ull;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const unsigned long long y = __shfl_xor(x, j, 64);
        const bool lower = (l & j) == 0, up = (l & k) == 0;
        x = (lower == up) ? (x < y ? x : y) : (x < y ? y : x);
      }
    if (l < m) a[l] = x;
  }
  __syncthreads();
}
__global__ void k(unsigned long long* out, int m, int mode) {
  __shared__ __attribute__((aligned(16))) unsigned long long a[514], tmp[512];
  unsigned long long st[5];
  for (int it = 0; it < 4; ++it) {
    a[threadIdx.x] = (unsigned long long)((threadIdx.x * 2654435761u + it) % 1000003u) << 32;
    a[threadIdx.x + 256] = (unsigned long long)(((threadIdx.x + 256) * 2654435761u + it) % 1000003u) << 32;
    __syncthreads();
    st[it] = __builtin_amdgcn_s_memrealtime();
    if (mode == 0) rank_plain(a, tmp, m);
    else if (mode == 1) rank_unrolled(a, tmp, m);
    else wave_bitonic(a, m);
    st[4] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[it] = st[4] - st[it];
    __syncthreads();
  }
}
int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 64);
  const char* names[3] = {"rank plain", "rank 16B x8", "wave bitonic"};
  for (int mode = 0; mode < 3; ++mode)
    for (int m : {50, 64, 200, 500}) {
      if (mode == 2 && m > 64) continue;
      hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, m, mode);
      unsigned long long h[4];
      (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
      printf("%-13s m=%3d us: %.2f %.2f %.2f %.2f\n", names[mode], m, h[0] * 0.01, h[1] * 0.01, h[2] * 0.01, h[3] * 0.01);
    }
  return 0;
}
