// disinfect_main.cc -- drives DISINFSystem (pose_manager + TSDFSystem + GPU feed_rgbd_frame) for
// tests/test_gpu_facade.py. <dir>/meta.txt:
//   W H nframes npose fx fy cx cy voxel trunc max_depth depth_factor nb_bits
//   npose lines "ts qx qy qz qw tx ty tz" (registered poses), then nframes lines "ts has_mask"
// <dir>/f<i>_rgb.bin (W x H x 3 u8), f<i>_depth.bin (W x H u16), f<i>_mask.bin (W x H u8).
// Writes <dir>/out_query.bin (query_tsdf of a huge cube) and out_stats.txt.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "disinfect_slam.h"

using namespace disinfect;

static std::vector<uint8_t> read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + p);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cerr << "usage: disinfect_main <dir>\n";
    return 2;
  }
  const std::string dir = argv[1];
  std::ifstream meta(dir + "/meta.txt");
  int W, H, n, npose, nb_bits;
  float fx, fy, cx, cy, voxel, trunc, max_depth, factor;
  meta >> W >> H >> n >> npose >> fx >> fy >> cx >> cy >> voxel >> trunc >> max_depth >> factor >> nb_bits;
  tsdf_config cfg;
  tsdf_config_default(&cfg);
  cfg.max_width = W / 2;
  cfg.max_height = H / 2;
  cfg.num_block_bits = nb_bits;
  try {
    DISINFSystem sys(voxel, trunc, max_depth, CameraIntrinsics<float>(fx, fy, cx, cy), SE3<float>::Identity(),
                     factor, &cfg, 0);
    for (int i = 0; i < npose; ++i) {
      long long ts;
      float v[7];
      meta >> ts;
      for (float& x : v) meta >> x;
      sys.register_camera_pose(ts, SE3<float>(v[0], v[1], v[2], v[3], v[4], v[5], v[6]));
    }
    for (int i = 0; i < n; ++i) {
      long long ts;
      int has_mask;
      meta >> ts >> has_mask;
      const std::string p = dir + "/f" + std::to_string(i);
      auto rgb = read_file(p + "_rgb.bin");
      auto depth = read_file(p + "_depth.bin");
      std::vector<uint8_t> mask;
      if (has_mask) mask = read_file(p + "_mask.bin");
      Mat m_rgb(H, W, CV_8UC3, rgb.data()), m_depth(H, W, CV_16UC1, depth.data());
      Mat m_mask = has_mask ? Mat(H, W, CV_8UC1, mask.data()) : Mat();
      sys.feed_rgbd_frame(m_rgb, m_depth, ts, m_mask);  // the queue deep-copies the frames
    }
    sys.tsdf().Flush();
    const auto vox = sys.query_tsdf(BoundingCube<float>{-1e4f, 1e4f, -1e4f, 1e4f, -1e4f, 1e4f});
    std::ofstream(dir + "/out_query.bin", std::ios::binary)
        .write(reinterpret_cast<const char*>(vox.data()), vox.size() * sizeof(VoxelSpatialTSDF));
    const tsdf_stats s = sys.tsdf().Stats();
    std::ofstream(dir + "/out_stats.txt") << s.frames << " " << s.active_blocks << " " << s.status << "\n";
  } catch (const std::exception& ex) {
    std::cerr << "disinfect_main: " << ex.what() << "\n";
    return 1;
  }
  return 0;
}
