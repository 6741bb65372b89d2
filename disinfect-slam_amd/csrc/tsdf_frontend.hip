// tsdf_frontend.hip -- DISINFSystem::feed_rgbd_frame preprocessing on the GPU
// (disinfect_slam/disinfect_slam.cc:31-64): the x0.5 cv::resize of rgb / depth / mask, the depth
// scale convertTo(CV_32FC1, 1 / depth_factor) and the mask -> depth 0 loop, in one pass.
//
// cv::resize(.., 0.5, 0.5, INTER_LINEAR) on an even-sized image runs OpenCV's fast INTER_AREA
// path (resize.cpp: INTER_LINEAR with integer scale 2 becomes INTER_AREA; ResizeAreaFastVec):
// every output channel is (a + b + c + d + 2) >> 2 of its 2x2 source block, for u8 and u16 alike.
// One thread per output pixel; the two source rows of a pixel pair are read as 4-byte (depth) and
// 2-byte (mask) words, so a wave reads contiguous 256-B / 128-B row segments.
#include "tsdf_kernels.h"

namespace tsdf {

__global__ __launch_bounds__(256) void k_rgbd_half(const uint8_t* __restrict__ rgb,
                                                   const uint16_t* __restrict__ depth,
                                                   const uint8_t* __restrict__ mask, int W, int H,
                                                   float alpha, uint8_t* __restrict__ rgb_out,
                                                   float* __restrict__ depth_out) {
  const int w = W >> 1, h = H >> 1;
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= w || y >= h) return;
  const size_t r0 = (size_t)(2 * y) * W + 2 * x, r1 = r0 + W;
  const uint32_t d0 = *reinterpret_cast<const uint32_t*>(depth + r0);  // 2x aligned: x even
  const uint32_t d1 = *reinterpret_cast<const uint32_t*>(depth + r1);
  const uint32_t dv = ((d0 & 0xFFFFu) + (d0 >> 16) + (d1 & 0xFFFFu) + (d1 >> 16) + 2u) >> 2;
  float d = (float)dv * alpha;  // convertTo: one rounding (cvtScale_ with beta 0)
  if (mask) {
    const uint16_t m0 = *reinterpret_cast<const uint16_t*>(mask + r0);
    const uint16_t m1 = *reinterpret_cast<const uint16_t*>(mask + r1);
    const uint32_t mv = ((m0 & 0xFFu) + (m0 >> 8) + (m1 & 0xFFu) + (m1 >> 8) + 2u) >> 2;
    if (mv == 0u) d = 0.0f;
  }
  const size_t o = (size_t)y * w + x;
  depth_out[o] = d;
  const uint8_t* a = rgb + r0 * 3;
  const uint8_t* b = rgb + r1 * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    rgb_out[o * 3 + c] = (uint8_t)(((uint32_t)a[c] + a[3 + c] + b[c] + b[3 + c] + 2u) >> 2);
}

}  // namespace tsdf
