// voxel_tsdf.h -- TSDFGrid (utils/tsdf/voxel_tsdf.cuh:32-124) on the MI355X engine's C ABI.
#pragma once

#include <string>
#include <vector>

#include "disinfect_tsdf.h"
#include "tsdf_types.h"

namespace disinfect {

class TSDFGrid {
 public:
  // voxel_tsdf.cuh:40 TSDFGrid(voxel_size, truncation); engine sizing defaults to the reference's
  // (2^18 blocks, images up to 1920x1080), overridable through cfg.
  TSDFGrid(float voxel_size, float truncation);
  TSDFGrid(const tsdf_config& cfg, int device = 0);
  // one volume spatially sharded over `devices` (one shard per entry; a device may repeat), the
  // exchange inside the library (tsdf_group_*): same results as one volume. FeedRGBD is not
  // available on a sharded volume (integrate the preprocessed frame).
  TSDFGrid(const tsdf_config& cfg, const std::vector<int>& devices);
  ~TSDFGrid();
  TSDFGrid(const TSDFGrid&) = delete;
  TSDFGrid& operator=(const TSDFGrid&) = delete;

  // voxel_tsdf.cu:347-375: rgb CV_8UC3, depth CV_32FC1 [m], ht / lt CV_32FC1 (empty -> ones)
  void Integrate(const Mat& img_rgb, const Mat& img_depth, const Mat& img_ht, const Mat& img_lt,
                 float max_depth, const CameraIntrinsics<float>& intrinsics,
                 const SE3<float>& cam_T_world);

  // DISINFSystem::feed_rgbd_frame's preprocessing + Integrate on the GPU (disinfect_slam.cc:31-67):
  // full-size rgb CV_8UC3, raw depth CV_16UC1, optional mask CV_8UC1 (empty = none), all of even
  // size; intrinsics are those of the half-size image the volume integrates
  void FeedRGBD(const Mat& img_rgb, const Mat& img_depth_raw, const Mat& mask, float depth_factor,
                float max_depth, const CameraIntrinsics<float>& intrinsics,
                const SE3<float>& cam_T_world);

  // voxel_tsdf.cu:490-506: renders into CV_8UC4 images (either may be null; the reference writes
  // into GL textures, utils/gl/image.h)
  void RayCast(float max_depth, const CameraParams& virtual_cam, const SE3<float>& cam_T_world,
               Mat* tsdf_rgba = nullptr, Mat* tsdf_normal = nullptr);

  std::vector<VoxelSpatialTSDF> GatherValid();                                  // :399-425
  std::vector<VoxelSpatialTSDF> GatherVoxels(const BoundingCube<float>& volumn);  // :427-454

  tsdf_stats Stats(bool clear_status = false);
  tsdf_engine* engine() { return engine_; }  // (NULL for a sharded volume)
  tsdf_group* group() { return group_; }      // (NULL for one engine)
  // block until every integrated frame is in the volume
  void Synchronize();

 private:
  std::vector<VoxelSpatialTSDF> Query(const float* bounds);
  tsdf_engine* engine_ = nullptr;
  tsdf_group* group_ = nullptr;
  float voxel_size_, truncation_;
};

// throws std::runtime_error with the engine's message on a non-zero status
void check_tsdf(int rc, const char* what);

}  // namespace disinfect
