// offline_main.cc -- examples/tsdf/offline.cc's integration loop without the GUI: replay a log
// directory (offline_log.h) through TSDFGrid, then GatherValid ("Save TSDF", offline.cc:181-187).
//   offline_main <logdir> fx fy cx cy depth_scale voxel trunc nb_bits [decode_only]
// Writes <logdir>/out_query.bin (16-B voxels) and out_stats.txt; decode_only writes the decoded
// frames (f<i>_{rgb,depth,ht,lt}.dec) and poses (poses.txt) instead (tests/test_host_cpu.py).
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>

#include "offline_log.h"

#ifndef OFFLINE_DECODE_ONLY
#include "voxel_tsdf.h"
#endif

using namespace disinfect;

int main(int argc, char** argv) {
  if (argc < 10) {
    std::cerr << "usage: offline_main <logdir> fx fy cx cy depth_scale voxel trunc nb_bits\n";
    return 2;
  }
  const std::string dir = argv[1];
  const CameraIntrinsics<float> K(std::stof(argv[2]), std::stof(argv[3]), std::stof(argv[4]), std::stof(argv[5]));
  const float depth_scale = std::stof(argv[6]), voxel = std::stof(argv[7]), trunc = std::stof(argv[8]);
  const int nb_bits = std::stoi(argv[9]);
  try {
    const auto entries = parse_log_entries(dir);
#ifdef OFFLINE_DECODE_ONLY
    std::ofstream poses(dir + "/poses.txt");
    for (size_t i = 0; i < entries.size(); ++i) {
      Mat rgb, depth, ht, lt;
      get_images_by_id(entries[i].id, depth_scale, &rgb, &depth, &ht, &lt, dir);
      const std::string p = dir + "/f" + std::to_string(i);
      std::ofstream(p + "_rgb.dec", std::ios::binary).write((const char*)rgb.data, rgb.total() * 3);
      std::ofstream(p + "_depth.dec", std::ios::binary).write((const char*)depth.data, depth.total() * 4);
      std::ofstream(p + "_ht.dec", std::ios::binary).write((const char*)ht.data, ht.total() * 4);
      std::ofstream(p + "_lt.dec", std::ios::binary).write((const char*)lt.data, lt.total() * 4);
      const Quaternion<float> q = entries[i].cam_T_world.GetR();
      const float* t = entries[i].cam_T_world.GetT();
      char line[256];
      std::snprintf(line, sizeof line, "%d %.9g %.9g %.9g %.9g %.9g %.9g %.9g\n", entries[i].id, q.x, q.y, q.z,
                    q.w, t[0], t[1], t[2]);
      poses << line;
    }
    (void)K, (void)voxel, (void)trunc, (void)nb_bits;
#else
    tsdf_config cfg;
    tsdf_config_default(&cfg);
    cfg.voxel_size = voxel;
    cfg.truncation = trunc;
    cfg.num_block_bits = nb_bits;
    TSDFGrid tsdf(cfg, 0);
    for (const LogEntry& e : entries) {
      Mat rgb, depth, ht, lt;
      get_images_by_id(e.id, depth_scale, &rgb, &depth, &ht, &lt, dir);
      tsdf.Integrate(rgb, depth, ht, lt, 4, K, e.cam_T_world);  // offline.cc:163-164
    }
    const auto vox = tsdf.GatherValid();
    std::ofstream(dir + "/out_query.bin", std::ios::binary)
        .write(reinterpret_cast<const char*>(vox.data()), vox.size() * sizeof(VoxelSpatialTSDF));
    const tsdf_stats s = tsdf.Stats();
    std::ofstream(dir + "/out_stats.txt") << s.frames << " " << s.active_blocks << " " << s.status << "\n";
#endif
  } catch (const std::exception& ex) {
    std::cerr << "offline_main: " << ex.what() << "\n";
    return 1;
  }
  return 0;
}
