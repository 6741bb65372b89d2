// bench_main.cc -- the driver bench's timed loop in C++ over the C ABI (no Python, no ctypes): the
// host-side floor of the per-frame enqueue. bench.py writes the frames of its own
// stream and runs this as a child process after its own timed loop:
//   bench_main <dir> <warmup> <steps>
//   <dir>/meta.txt : W H nframes fx fy cx cy voxel trunc max_depth semantic nb_bits
//                    then per frame: qx qy qz qw tx ty tz
//   <dir>/f<i>_{rgb,depth,ht,lt}.bin
// Every frame is uploaded to device memory first (the bench's frames are resident in HBM); then
// warmup frames, a synchronisation, and exactly `steps` frames timed -- tsdf_integrate per frame
// with TSDF_MEM_DEVICE pointers, tsdf_flush (the pipelined last frame), tsdf_synchronize -- on the
// engine's own stream. Prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "disinfect_tsdf.h"

static std::vector<uint8_t> read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + p);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static void check(int rc, const char* what) {
  if (rc != TSDF_OK) throw std::runtime_error(std::string(what) + ": " + tsdf_last_error());
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: bench_main <dir> <warmup> <steps>\n");
    return 2;
  }
  try {
    const std::string dir = argv[1];
    const int warmup = std::atoi(argv[2]), steps = std::atoi(argv[3]);
    std::ifstream meta(dir + "/meta.txt");
    int W, H, n, semantic, nb_bits;
    float fx, fy, cx, cy, voxel, trunc, max_depth;
    meta >> W >> H >> n >> fx >> fy >> cx >> cy >> voxel >> trunc >> max_depth >> semantic >> nb_bits;
    if (n < warmup + steps) throw std::runtime_error("not enough frames");
    std::vector<tsdf_pose> poses(n);
    for (auto& p : poses) meta >> p.qx >> p.qy >> p.qz >> p.qw >> p.tx >> p.ty >> p.tz;
    const size_t px = (size_t)W * H;
    std::vector<tsdf_frame> frames(n);
    std::vector<void*> dev;
    for (int i = 0; i < n; ++i) {
      const std::string p = dir + "/f" + std::to_string(i) + "_";
      const char* names[4] = {"rgb", "depth", "ht", "lt"};
      void* d[4] = {nullptr, nullptr, nullptr, nullptr};
      for (int k = 0; k < (semantic ? 4 : 2); ++k) {
        std::vector<uint8_t> h = read_file(p + names[k] + ".bin");
        if (hipMalloc(&d[k], h.size()) != hipSuccess ||
            hipMemcpy(d[k], h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess)
          throw std::runtime_error("device frame upload");
        dev.push_back(d[k]);
      }
      frames[i] = tsdf_frame{W, H, (const uint8_t*)d[0], (const float*)d[1], (const float*)d[2],
                             (const float*)d[3], TSDF_MEM_DEVICE};
      (void)px;
    }
    tsdf_config cfg;
    tsdf_config_default(&cfg);
    cfg.voxel_size = voxel;
    cfg.truncation = trunc;
    cfg.max_width = W;
    cfg.max_height = H;
    cfg.num_block_bits = nb_bits;
    tsdf_engine* e = nullptr;
    check(tsdf_create(&cfg, 0, &e), "tsdf_create");
    const tsdf_intrinsics K{fx, fy, cx, cy};
    for (int i = 0; i < warmup; ++i) check(tsdf_integrate(e, &frames[i], &K, &poses[i], max_depth), "tsdf_integrate");
    check(tsdf_flush(e), "tsdf_flush");
    check(tsdf_synchronize(e), "tsdf_synchronize");
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int i = warmup; i < warmup + steps; ++i)
      check(tsdf_integrate(e, &frames[i], &K, &poses[i], max_depth), "tsdf_integrate");
    check(tsdf_flush(e), "tsdf_flush");
    const auto t_enq = clk::now();
    check(tsdf_synchronize(e), "tsdf_synchronize");
    const auto t1 = clk::now();
    tsdf_stats st;
    check(tsdf_get_stats(e, &st, 0), "tsdf_get_stats");
    const double el = std::chrono::duration<double>(t1 - t0).count();
    const double enq = std::chrono::duration<double>(t_enq - t0).count();
    std::printf("{\"frames_per_s\": %.1f, \"ms_per_step\": %.5f, \"host_enqueue_us_per_step\": %.2f, "
                "\"steps\": %d, \"warmup\": %d, \"status\": %u, \"active_blocks\": %d}\n",
                steps / el, el / steps * 1e3, enq / steps * 1e6, steps, warmup, st.status, st.active_blocks);
    check(tsdf_destroy(e), "tsdf_destroy");
    for (void* d : dev) (void)hipFree(d);
    return st.status == 0 ? 0 : 1;
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "bench_main: %s\n", ex.what());
    return 1;
  }
}
