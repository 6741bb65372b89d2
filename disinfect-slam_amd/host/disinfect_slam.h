// disinfect_slam.h -- DISINFSystem (disinfect_slam/disinfect_slam.h:22-60) reduced to its TSDF
// half: the pose store the SLAM tracker feeds (pose_manager), the sensor-frame entry point
// feed_rgbd_frame and query_tsdf, over TSDFSystem on the MI355X engine. The ORB-SLAM3 tracker,
// the segmentation network and the renderer are outside this engine: a tracker
// registers its poses with register_camera_pose (what feed_stereo / feed_stereo_IMU do after
// TrackStereo, disinfect_slam.cc:69-100).
#pragma once

#include <memory>

#include "pose_manager.h"
#include "tsdf_module.h"

namespace disinfect {

class DISINFSystem {
 public:
  // disinfect_slam.cc:3-24 builds TSDFSystem(0.05, 0.2, 4, intrinsics, extrinsics) from the camera
  // config and reads DepthMapFactor; here the values are passed in (no YAML reader in the engine)
  DISINFSystem(float voxel_size, float truncation, float max_depth,
               const CameraIntrinsics<float>& intrinsics, const SE3<float>& extrinsics,
               float depth_factor, const tsdf_config* engine_cfg = nullptr, int device = 0);

  // disinfect_slam.cc:31-67: pose at `timestamp` [ms], x0.5 resize of rgb / depth / mask, depth
  // scale, mask -> depth 0, integrate (the resize / scale / mask run on the GPU)
  void feed_rgbd_frame(const Mat& img_rgb, const Mat& img_depth, int64_t timestamp, const Mat& mask = {});
  void register_camera_pose(int64_t timestamp, const SE3<float>& cam_T_world);
  SE3<float> query_camera_pose(int64_t timestamp);                              // :108-111
  std::vector<VoxelSpatialTSDF> query_tsdf(const BoundingCube<float>& volumn);  // :113-116
  TSDFSystem& tsdf() { return *TSDF_; }

 private:
  std::shared_ptr<TSDFSystem> TSDF_;
  std::shared_ptr<pose_manager> camera_pose_manager_;
  float depthmap_factor_;
};

}  // namespace disinfect
