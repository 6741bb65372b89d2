// facade_main.cc -- drives the C++17 facade (TSDFSystem / TSDFGrid) over the C ABI for the GPU
// tests (tests/test_gpu_facade.py). Frames are raw files written by the test:
//   <dir>/meta.txt : W H nframes fx fy cx cy voxel trunc max_depth semantic nb_bits
//                    then per frame: qx qy qz qw tx ty tz
//   <dir>/f<i>_{rgb,depth,ht,lt}.bin
// Outputs: <dir>/out_query.bin (GatherValid voxels), out_render.bin (RayCast normal of the last
// pose), out_stats.txt. facade_main <dir> <G>: the same through a volume sharded over G shards of
// device 0 (TSDFSystem's group constructor, tsdf_group_*).
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "tsdf_module.h"

using namespace disinfect;

static std::vector<uint8_t> read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + p);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cerr << "usage: facade_main <dir> [shards]\n";
    return 2;
  }
  const std::string dir = argv[1];
  const int shards = argc > 2 ? std::atoi(argv[2]) : 1;
  std::ifstream meta(dir + "/meta.txt");
  int W, H, n, semantic, nb_bits;
  float fx, fy, cx, cy, voxel, trunc, max_depth;
  meta >> W >> H >> n >> fx >> fy >> cx >> cy >> voxel >> trunc >> max_depth >> semantic >> nb_bits;
  std::vector<SE3<float>> poses;
  for (int i = 0; i < n; ++i) {
    float q[4], t[3];
    meta >> q[0] >> q[1] >> q[2] >> q[3] >> t[0] >> t[1] >> t[2];
    poses.emplace_back(q[0], q[1], q[2], q[3], t[0], t[1], t[2]);
  }
  tsdf_config cfg;
  tsdf_config_default(&cfg);
  cfg.voxel_size = voxel;
  cfg.truncation = trunc;
  cfg.max_width = W;
  cfg.max_height = H;
  cfg.num_block_bits = nb_bits;
  const CameraIntrinsics<float> K(fx, fy, cx, cy);
  std::vector<VoxelSpatialTSDF> vox;
  Mat normal;
  tsdf_stats st;
  {
    // extrinsics = identity; the poses are the cam_T_world of the stream
    std::unique_ptr<TSDFSystem> sysp =
        shards > 1 ? std::make_unique<TSDFSystem>(cfg, std::vector<int>(shards, 0), max_depth, K)
                   : std::make_unique<TSDFSystem>(cfg, 0, max_depth, K);
    TSDFSystem& sys = *sysp;
    std::vector<std::vector<uint8_t>> keep;
    for (int i = 0; i < n; ++i) {
      const std::string p = dir + "/f" + std::to_string(i) + "_";
      keep.push_back(read_file(p + "rgb.bin"));
      Mat rgb(H, W, CV_8UC3, keep.back().data());
      keep.push_back(read_file(p + "depth.bin"));
      Mat depth(H, W, CV_32FC1, keep.back().data());
      if (semantic) {
        keep.push_back(read_file(p + "ht.bin"));
        Mat ht(H, W, CV_32FC1, keep.back().data());
        keep.push_back(read_file(p + "lt.bin"));
        Mat lt(H, W, CV_32FC1, keep.back().data());
        sys.Integrate(poses[i], rgb, depth, ht, lt);
      } else {
        sys.Integrate(poses[i], rgb, depth);
      }
    }
    sys.Flush();
    vox = sys.Query(BoundingCube<float>{-100.f, 100.f, -100.f, 100.f, -100.f, 100.f});
    sys.Render(CameraParams(K, H, W), poses.back(), &normal);
    st = sys.Stats();
  }
  std::ofstream(dir + "/out_query.bin", std::ios::binary)
      .write(reinterpret_cast<const char*>(vox.data()), vox.size() * sizeof(VoxelSpatialTSDF));
  std::ofstream(dir + "/out_render.bin", std::ios::binary)
      .write(reinterpret_cast<const char*>(normal.data), normal.total() * 4);
  std::ofstream so(dir + "/out_stats.txt");
  so << st.frames << " " << st.active_blocks << " " << st.last_num_visible << " "
     << st.last_num_updated << " " << st.status << "\n";
  std::printf("facade ok: %zu voxels, %d blocks\n", vox.size(), st.active_blocks);
  return 0;
}
