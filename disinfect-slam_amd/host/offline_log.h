// offline_log.h -- the offline replay format of examples/tsdf/offline.cc:26-83 without OpenCV /
// yaml-cpp: <logdir>/trajectory.txt ("id r00 r01 r02 t0 r10 r11 r12 t1 r20 r21 r22 t2" per line,
// cam_T_world as a row-major 3x4) and per id the PNG frames {id}_rgb.png (8-bit colour),
// {id}_depth.png (16-bit, raw sensor units), {id}_ht.png / {id}_no_ht.png (16-bit, probability x
// 65535; absent -> ht = 0, lt = 1 as offline.cc:78-81 does).
#pragma once

#include <string>
#include <vector>

#include "tsdf_types.h"

namespace disinfect {

struct LogEntry {
  int id;
  SE3<float> cam_T_world;
};

// offline.cc:45-63: entries in file order; cam_T_world = extrinsics * SE3(row-major 3x4)
std::vector<LogEntry> parse_log_entries(const std::string& logdir,
                                        const SE3<float>& extrinsics = SE3<float>::Identity());

// PNG decoder (zlib inflate + the five scanline filters), non-interlaced, bit depth 8 or 16:
//   colour types 2 / 6 (RGB / RGBA) -> CV_8UC3 in RGB order (alpha dropped; 16-bit samples >> 8),
//   colour type 0 (grey)            -> CV_8UC1 or CV_16UC1 (IMREAD_UNCHANGED)
// Returns an empty Mat if the file is missing; throws std::runtime_error on a malformed file.
Mat read_png(const std::string& path);

// offline.cc:65-83 get_images_by_id: rgb CV_8UC3 (RGB, i.e. imread + BGR2RGB), depth CV_32FC1
// = raw * (float)(1 / depth_scale), ht / lt CV_32FC1 = raw * (float)(1 / 65535.)
void get_images_by_id(int id, float depth_scale, Mat* img_rgb, Mat* img_depth, Mat* img_ht,
                      Mat* img_lt, const std::string& logdir);

}  // namespace disinfect
