// tsdf_module.h -- TSDFSystem (modules/tsdf_module.h:16-107): threaded facade over TSDFGrid.
//
// Same contract as the reference: Integrate() is a non-blocking enqueue (it composes
// cam_T_posecam * posecam_T_world and substitutes all-ones ht / lt maps when they are empty,
// tsdf_module.cc:26-38); one worker thread integrates in order; Integrate, Query and Render are
// mutually exclusive (mtx_read_). Differences: the worker waits on a condition variable instead of
// busy-spinning (tsdf_module.cc:51-75), and the queue deep-copies the frames because Mat views
// may borrow caller memory (the reference keeps shallow ref-counted cv::Mat).
#pragma once

#include <condition_variable>
#include <memory>
#include <mutex>
#include <queue>
#include <thread>

#include "voxel_tsdf.h"

namespace disinfect {

struct TSDFSystemInput {
  SE3<float> cam_T_world;
  Mat img_rgb;
  Mat img_depth;
  Mat img_ht;   // raw frames: the mask
  Mat img_lt;
  float depth_factor = 0.0f;  // > 0: a raw sensor frame (FeedRGBD) with depth in sensor units

  TSDFSystemInput(const SE3<float>& cam_T_world, const Mat& img_rgb, const Mat& img_depth,
                  const Mat& img_ht, const Mat& img_lt, float depth_factor = 0.0f)
      : cam_T_world(cam_T_world), img_rgb(img_rgb), img_depth(img_depth), img_ht(img_ht),
        img_lt(img_lt), depth_factor(depth_factor) {}
};

class TSDFSystem {
 public:
  TSDFSystem(float voxel_size, float truncation, float max_depth,
             const CameraIntrinsics<float>& intrinsics,
             const SE3<float>& extrinsics = SE3<float>::Identity());
  // engine sizing / device selection beyond the reference constructor
  TSDFSystem(const tsdf_config& cfg, int device, float max_depth,
             const CameraIntrinsics<float>& intrinsics,
             const SE3<float>& extrinsics = SE3<float>::Identity());
  // one volume spatially sharded over `devices` (TSDFGrid's group constructor): a C++ caller gets a
  // multi-GPU (or multi-shard) volume without Python or a collective library
  TSDFSystem(const tsdf_config& cfg, const std::vector<int>& devices, float max_depth,
             const CameraIntrinsics<float>& intrinsics,
             const SE3<float>& extrinsics = SE3<float>::Identity());
  ~TSDFSystem();

  void Integrate(const SE3<float>& posecam_T_world, const Mat& img_rgb, const Mat& img_depth,
                 const Mat& img_ht = {}, const Mat& img_lt = {});
  // a raw full-size sensor frame (CV_8UC3 rgb, CV_16UC1 depth, optional CV_8UC1 mask): the GPU
  // runs DISINFSystem::feed_rgbd_frame's resize / depth scale / mask before integrating
  void IntegrateRaw(const SE3<float>& posecam_T_world, const Mat& img_rgb, const Mat& img_depth_raw,
                    const Mat& mask, float depth_factor);
  std::vector<VoxelSpatialTSDF> Query(const BoundingCube<float>& volumn);
  void Render(const CameraParams& virtual_cam, const SE3<float> cam_T_world, Mat* img_normal);

  // block until every queued frame has been integrated (not in the reference; used by tests)
  void Flush();
  tsdf_stats Stats();

 private:
  void Run();
  void Enqueue(std::unique_ptr<TSDFSystemInput> in);
  TSDFGrid tsdf_;
  float max_depth_;
  const CameraIntrinsics<float> intrinsics_;
  const SE3<float> cam_T_posecam_;
  std::mutex mtx_queue_;
  std::condition_variable cv_queue_;
  std::condition_variable cv_idle_;
  std::queue<std::unique_ptr<TSDFSystemInput>> inputs_;
  bool busy_ = false;
  std::mutex mtx_read_;
  bool terminate_ = false;
  std::thread t_;
};

}  // namespace disinfect
