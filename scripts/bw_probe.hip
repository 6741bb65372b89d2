// bw_probe.hip -- diagnostic (not part of the product): the memory-only floor of k_integrate's
// access pattern on this GPU. A resident grid of 256-thread workgroups, two waves per block,
// reads N random 6-KiB pool records (3 x 16 B per lane, as k_integrate does) and writes each
// lane's 48 B back, then reports the HIP-event and in-kernel durations per launch.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe.hip -o build/bw_probe && build/bw_probe [N]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_probe(uint8_t* pool, const int* list, int n, int write,
                                               unsigned long long* ticks) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave >> 1, hf = wave & 1, lane = threadIdx.x & 63;
  const int off = (hf * 256 + lane * 4) * 4;
  if (blockIdx.x == 0 && threadIdx.x == 0) ticks[0] = __builtin_amdgcn_s_memrealtime();
  const int npairs = (n + 1) >> 1;
  for (int pp = blockIdx.x; pp < npairs; pp += gridDim.x) {
    const int b = 2 * pp + pair;
    if (b >= n) continue;
    uint8_t* blk = pool + (size_t)list[b] * 6144;
    float4 a = *reinterpret_cast<const float4*>(blk + off);
    float4 c = *reinterpret_cast<const float4*>(blk + 2048 + off);
    uint4 d = *reinterpret_cast<const uint4*>(blk + 4096 + off);
    a.x += 1.0f; c.y += 1.0f; d.z += 1u;
    if (write) {
      *reinterpret_cast<float4*>(blk + off) = a;
      *reinterpret_cast<float4*>(blk + 2048 + off) = c;
      *reinterpret_cast<uint4*>(blk + 4096 + off) = d;
    } else if (a.x == -12345.f && c.y == 1.f && d.z == 7u) {
      blk[off] = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) ticks[1 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();  // no contended atomic
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 5800;
  const int span = argc > 2 ? atoi(argv[2]) : (1 << 18);  // blocks drawn from [0, span)
  const int nb = 1 << 18;
  uint8_t* pool;
  int* list;
  unsigned long long* ticks;
  CK(hipMalloc(&pool, (size_t)nb * 6144));
  CK(hipMemset(pool, 0, (size_t)nb * 6144));
  CK(hipMalloc(&list, n * sizeof(int)));
  CK(hipMalloc(&ticks, (1 + 65536) * sizeof(unsigned long long)));
  std::vector<int> h(span);
  for (int i = 0; i < span; ++i) h[i] = i;
  std::mt19937 rng(5);
  std::shuffle(h.begin(), h.end(), rng);
  CK(hipMemcpy(list, h.data(), n * sizeof(int), hipMemcpyHostToDevice));
  int per_cu = 0, ncu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_probe, 256, 0));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = per_cu * ncu;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int write = 0; write < 2; ++write) {
    double ev = 0, dev = 0;
    const int iters = 200;
    for (int it = 0; it < iters + 20; ++it) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), 0, 0, pool, list, n, write, ticks);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      std::vector<unsigned long long> t(1 + grid);
      CK(hipMemcpy(t.data(), ticks, (1 + grid) * 8, hipMemcpyDeviceToHost));
      unsigned long long tend = 0;
      for (int i = 1; i <= grid; ++i) tend = t[i] > tend ? t[i] : tend;
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (it >= 20) {
        ev += ms * 1e3;
        dev += (tend - t[0]) * 1e-2;
      }
    }
    ev /= iters;
    dev /= iters;
    const double bytes = (double)n * 6144 * (write ? 2 : 1);
    printf("span=%d n=%d grid=%d write=%d  event %.2f us (%.0f GB/s)  device %.2f us (%.0f GB/s)\n", span, n, grid,
           write, ev, bytes / ev * 1e-3, dev, bytes / dev * 1e-3);
  }
  return 0;
}
