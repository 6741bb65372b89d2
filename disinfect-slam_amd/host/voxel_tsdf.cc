// voxel_tsdf.cc -- TSDFGrid facade over include/disinfect_tsdf.h.
#include "voxel_tsdf.h"

#include <stdexcept>

namespace disinfect {

void check_tsdf(int rc, const char* what) {
  if (rc != TSDF_OK)
    throw std::runtime_error(std::string(what) + ": " + tsdf_error_string(rc) + " (" +
                             tsdf_last_error() + ")");
}

TSDFGrid::TSDFGrid(float voxel_size, float truncation)
    : voxel_size_(voxel_size), truncation_(truncation) {
  tsdf_config cfg;
  tsdf_config_default(&cfg);
  cfg.voxel_size = voxel_size;
  cfg.truncation = truncation;
  check_tsdf(tsdf_create(&cfg, 0, &engine_), "tsdf_create");
}

TSDFGrid::TSDFGrid(const tsdf_config& cfg, int device)
    : voxel_size_(cfg.voxel_size), truncation_(cfg.truncation) {
  check_tsdf(tsdf_create(&cfg, device, &engine_), "tsdf_create");
}

TSDFGrid::TSDFGrid(const tsdf_config& cfg, const std::vector<int>& devices)
    : voxel_size_(cfg.voxel_size), truncation_(cfg.truncation) {
  check_tsdf(tsdf_group_create(&cfg, devices.data(), (int)devices.size(), &group_), "tsdf_group_create");
}

TSDFGrid::~TSDFGrid() {
  if (engine_) tsdf_destroy(engine_);
  if (group_) tsdf_group_destroy(group_);
}

void TSDFGrid::Synchronize() {
  if (group_)
    check_tsdf(tsdf_group_synchronize(group_), "tsdf_group_synchronize");
  else
    check_tsdf(tsdf_synchronize(engine_), "tsdf_synchronize");
}

static tsdf_pose to_pose(const SE3<float>& T) {
  const Quaternion<float> q = T.GetR();
  const float* t = T.GetT();
  return tsdf_pose{q.x, q.y, q.z, q.w, t[0], t[1], t[2]};
}

void TSDFGrid::Integrate(const Mat& img_rgb, const Mat& img_depth, const Mat& img_ht,
                         const Mat& img_lt, float max_depth,
                         const CameraIntrinsics<float>& intrinsics, const SE3<float>& cam_T_world) {
  // voxel_tsdf.cu:350-353 (asserts in the reference)
  if (img_rgb.type() != CV_8UC3 || img_depth.type() != CV_32FC1 || img_rgb.cols != img_depth.cols ||
      img_rgb.rows != img_depth.rows)
    throw std::invalid_argument("TSDFGrid::Integrate: expects CV_8UC3 rgb and CV_32FC1 depth of equal size");
  const bool sem = !img_ht.empty() && !img_lt.empty();
  if (sem && (img_ht.type() != CV_32FC1 || img_lt.type() != CV_32FC1 || img_ht.total() != img_depth.total() ||
              img_lt.total() != img_depth.total()))
    throw std::invalid_argument("TSDFGrid::Integrate: ht / lt must be CV_32FC1 of the depth size");
  tsdf_frame f;
  f.width = img_depth.cols;
  f.height = img_depth.rows;
  f.rgb = img_rgb.ptr<uint8_t>();
  f.depth = img_depth.ptr<float>();
  f.ht = sem ? img_ht.ptr<float>() : nullptr;
  f.lt = sem ? img_lt.ptr<float>() : nullptr;
  f.mem_kind = TSDF_MEM_HOST;
  const tsdf_intrinsics K{intrinsics.fx, intrinsics.fy, intrinsics.cx, intrinsics.cy};
  const tsdf_pose P = to_pose(cam_T_world);
  if (group_)
    check_tsdf(tsdf_group_integrate(group_, &f, &K, &P, max_depth), "tsdf_group_integrate");
  else
    check_tsdf(tsdf_integrate(engine_, &f, &K, &P, max_depth), "tsdf_integrate");
}

void TSDFGrid::FeedRGBD(const Mat& img_rgb, const Mat& img_depth_raw, const Mat& mask, float depth_factor,
                        float max_depth, const CameraIntrinsics<float>& intrinsics,
                        const SE3<float>& cam_T_world) {
  if (img_rgb.type() != CV_8UC3 || img_depth_raw.type() != CV_16UC1 || img_rgb.cols != img_depth_raw.cols ||
      img_rgb.rows != img_depth_raw.rows ||
      (!mask.empty() && (mask.type() != CV_8UC1 || mask.total() != img_depth_raw.total())))
    throw std::invalid_argument("TSDFGrid::FeedRGBD: expects CV_8UC3 rgb, CV_16UC1 depth, CV_8UC1 mask");
  if (group_) throw std::invalid_argument("TSDFGrid::FeedRGBD: not available on a sharded volume");
  const tsdf_intrinsics K{intrinsics.fx, intrinsics.fy, intrinsics.cx, intrinsics.cy};
  const tsdf_pose P = to_pose(cam_T_world);
  check_tsdf(tsdf_feed_rgbd_frame(engine_, img_rgb.ptr<uint8_t>(), img_depth_raw.ptr<uint16_t>(),
                                  mask.empty() ? nullptr : mask.ptr<uint8_t>(), img_depth_raw.cols,
                                  img_depth_raw.rows, depth_factor, &K, &P, max_depth, TSDF_MEM_HOST),
             "tsdf_feed_rgbd_frame");
}

void TSDFGrid::RayCast(float max_depth, const CameraParams& cam, const SE3<float>& cam_T_world,
                       Mat* rgba, Mat* normal) {
  if (rgba && (rgba->rows != cam.img_h || rgba->cols != cam.img_w || rgba->type() != CV_8UC4))
    *rgba = Mat(cam.img_h, cam.img_w, CV_8UC4);
  if (normal && (normal->rows != cam.img_h || normal->cols != cam.img_w || normal->type() != CV_8UC4))
    *normal = Mat(cam.img_h, cam.img_w, CV_8UC4);
  const tsdf_intrinsics K{cam.intrinsics.fx, cam.intrinsics.fy, cam.intrinsics.cx, cam.intrinsics.cy};
  const tsdf_pose P = to_pose(cam_T_world);
  if (group_)
    check_tsdf(tsdf_group_raycast(group_, &K, cam.img_w, cam.img_h, &P, max_depth, rgba ? rgba->data : nullptr,
                                  normal ? normal->data : nullptr, TSDF_MEM_HOST),
               "tsdf_group_raycast");
  else
    check_tsdf(tsdf_raycast(engine_, &K, cam.img_w, cam.img_h, &P, max_depth,
                            rgba ? rgba->data : nullptr, normal ? normal->data : nullptr, TSDF_MEM_HOST),
               "tsdf_raycast");
}

std::vector<VoxelSpatialTSDF> TSDFGrid::Query(const float* bounds) {
  int64_t n = 0;
  auto query = [&](tsdf_voxel* o, int64_t cap) {
    return group_ ? tsdf_group_query(group_, bounds, o, cap, &n) : tsdf_query(engine_, bounds, o, cap, &n);
  };
  check_tsdf(query(nullptr, 0), "tsdf_query");
  std::vector<VoxelSpatialTSDF> out((size_t)n);
  if (n) check_tsdf(query(reinterpret_cast<tsdf_voxel*>(out.data()), n), "tsdf_query");
  return out;
}

std::vector<VoxelSpatialTSDF> TSDFGrid::GatherValid() { return Query(nullptr); }

std::vector<VoxelSpatialTSDF> TSDFGrid::GatherVoxels(const BoundingCube<float>& v) {
  const float b[6] = {v.xmin, v.xmax, v.ymin, v.ymax, v.zmin, v.zmax};
  return Query(b);
}

tsdf_stats TSDFGrid::Stats(bool clear_status) {
  tsdf_stats s;
  if (group_)
    check_tsdf(tsdf_group_get_stats(group_, &s, clear_status ? 1 : 0), "tsdf_group_get_stats");
  else
    check_tsdf(tsdf_get_stats(engine_, &s, clear_status ? 1 : 0), "tsdf_get_stats");
  return s;
}

}  // namespace disinfect
