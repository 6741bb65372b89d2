// disinfect_slam.cc -- DISINFSystem's TSDF half (disinfect_slam/disinfect_slam.cc:3-116).
#include "disinfect_slam.h"

namespace disinfect {

static std::shared_ptr<TSDFSystem> make_tsdf(float voxel_size, float truncation, float max_depth,
                                             const CameraIntrinsics<float>& intrinsics,
                                             const SE3<float>& extrinsics, const tsdf_config* cfg,
                                             int device) {
  if (!cfg) return std::make_shared<TSDFSystem>(voxel_size, truncation, max_depth, intrinsics, extrinsics);
  tsdf_config c = *cfg;
  c.voxel_size = voxel_size;
  c.truncation = truncation;
  return std::make_shared<TSDFSystem>(c, device, max_depth, intrinsics, extrinsics);
}

DISINFSystem::DISINFSystem(float voxel_size, float truncation, float max_depth,
                           const CameraIntrinsics<float>& intrinsics, const SE3<float>& extrinsics,
                           float depth_factor, const tsdf_config* engine_cfg, int device)
    : TSDF_(make_tsdf(voxel_size, truncation, max_depth, intrinsics, extrinsics, engine_cfg, device)),
      camera_pose_manager_(std::make_shared<pose_manager>()),
      depthmap_factor_(depth_factor) {}

void DISINFSystem::feed_rgbd_frame(const Mat& img_rgb, const Mat& img_depth, int64_t timestamp,
                                   const Mat& mask) {
  const SE3<float> posecam_P_world = camera_pose_manager_->query_pose(timestamp);
  TSDF_->IntegrateRaw(posecam_P_world, img_rgb, img_depth, mask, depthmap_factor_);
}

void DISINFSystem::register_camera_pose(int64_t timestamp, const SE3<float>& cam_T_world) {
  camera_pose_manager_->register_valid_pose(timestamp, cam_T_world);
}

SE3<float> DISINFSystem::query_camera_pose(int64_t timestamp) {
  return camera_pose_manager_->query_pose(timestamp);
}

std::vector<VoxelSpatialTSDF> DISINFSystem::query_tsdf(const BoundingCube<float>& volumn) {
  return TSDF_->Query(volumn);
}

}  // namespace disinfect
