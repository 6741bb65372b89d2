// tsdf_module.cc -- TSDFSystem (modules/tsdf_module.cc:5-75) on the MI355X engine.
#include "tsdf_module.h"

#include <cstdio>

namespace disinfect {

TSDFSystem::TSDFSystem(float voxel_size, float truncation, float max_depth,
                       const CameraIntrinsics<float>& intrinsics, const SE3<float>& extrinsics)
    : tsdf_(voxel_size, truncation),
      max_depth_(max_depth),
      intrinsics_(intrinsics),
      cam_T_posecam_(extrinsics),
      t_(&TSDFSystem::Run, this) {}

TSDFSystem::TSDFSystem(const tsdf_config& cfg, int device, float max_depth,
                       const CameraIntrinsics<float>& intrinsics, const SE3<float>& extrinsics)
    : tsdf_(cfg, device),
      max_depth_(max_depth),
      intrinsics_(intrinsics),
      cam_T_posecam_(extrinsics),
      t_(&TSDFSystem::Run, this) {}

TSDFSystem::TSDFSystem(const tsdf_config& cfg, const std::vector<int>& devices, float max_depth,
                       const CameraIntrinsics<float>& intrinsics, const SE3<float>& extrinsics)
    : tsdf_(cfg, devices),
      max_depth_(max_depth),
      intrinsics_(intrinsics),
      cam_T_posecam_(extrinsics),
      t_(&TSDFSystem::Run, this) {}

TSDFSystem::~TSDFSystem() {
  {
    std::lock_guard<std::mutex> lock(mtx_queue_);
    terminate_ = true;
  }
  cv_queue_.notify_all();
  t_.join();
}

void TSDFSystem::Integrate(const SE3<float>& posecam_T_world, const Mat& img_rgb,
                           const Mat& img_depth, const Mat& img_ht, const Mat& img_lt) {
  std::unique_ptr<TSDFSystemInput> in;
  if (img_ht.empty() || img_lt.empty()) {
    // tsdf_module.cc:29-33 substitutes all-ones maps; the engine reads absent maps as ones
    in = std::make_unique<TSDFSystemInput>(cam_T_posecam_ * posecam_T_world, img_rgb.clone(),
                                           img_depth.clone(), Mat(), Mat());
  } else {
    in = std::make_unique<TSDFSystemInput>(cam_T_posecam_ * posecam_T_world, img_rgb.clone(),
                                           img_depth.clone(), img_ht.clone(), img_lt.clone());
  }
  Enqueue(std::move(in));
}

void TSDFSystem::IntegrateRaw(const SE3<float>& posecam_T_world, const Mat& img_rgb,
                              const Mat& img_depth_raw, const Mat& mask, float depth_factor) {
  if (!(depth_factor > 0.0f)) throw std::invalid_argument("TSDFSystem::IntegrateRaw: depth_factor <= 0");
  Enqueue(std::make_unique<TSDFSystemInput>(cam_T_posecam_ * posecam_T_world, img_rgb.clone(),
                                            img_depth_raw.clone(), mask.empty() ? Mat() : mask.clone(),
                                            Mat(), depth_factor));
}

void TSDFSystem::Enqueue(std::unique_ptr<TSDFSystemInput> in) {
  {
    std::lock_guard<std::mutex> lock(mtx_queue_);
    inputs_.push(std::move(in));
    if (inputs_.size() > 10)  // tsdf_module.cc:62-63
      std::fprintf(stderr, "[TSDF System] Processing cannot catch up (input size: %zu)\n", inputs_.size());
  }
  cv_queue_.notify_one();
}

std::vector<VoxelSpatialTSDF> TSDFSystem::Query(const BoundingCube<float>& volumn) {
  std::lock_guard<std::mutex> lock(mtx_read_);
  return tsdf_.GatherVoxels(volumn);
}

void TSDFSystem::Render(const CameraParams& virtual_cam, const SE3<float> cam_T_world, Mat* img_normal) {
  std::lock_guard<std::mutex> lock(mtx_read_);
  tsdf_.RayCast(max_depth_, virtual_cam, cam_T_world, nullptr, img_normal);
}

void TSDFSystem::Flush() {
  std::unique_lock<std::mutex> lock(mtx_queue_);
  cv_idle_.wait(lock, [&] { return inputs_.empty() && !busy_; });
  std::lock_guard<std::mutex> lr(mtx_read_);
  tsdf_.Synchronize();
}

tsdf_stats TSDFSystem::Stats() {
  std::lock_guard<std::mutex> lock(mtx_read_);
  return tsdf_.Stats();
}

void TSDFSystem::Run() {
  while (true) {
    std::unique_ptr<TSDFSystemInput> input;
    {
      std::unique_lock<std::mutex> lock(mtx_queue_);
      cv_queue_.wait(lock, [&] { return terminate_ || !inputs_.empty(); });
      if (terminate_) return;
      input = std::move(inputs_.front());
      inputs_.pop();
      busy_ = true;
    }
    try {
      std::lock_guard<std::mutex> lock(mtx_read_);
      if (input->depth_factor > 0.0f)
        tsdf_.FeedRGBD(input->img_rgb, input->img_depth, input->img_ht, input->depth_factor, max_depth_,
                       intrinsics_, input->cam_T_world);
      else
        tsdf_.Integrate(input->img_rgb, input->img_depth, input->img_ht, input->img_lt, max_depth_,
                        intrinsics_, input->cam_T_world);
    } catch (const std::exception& ex) {  // never let an engine error kill the worker
      std::fprintf(stderr, "[TSDF System] integrate failed: %s\n", ex.what());
    }
    {
      std::lock_guard<std::mutex> lock(mtx_queue_);
      busy_ = false;
    }
    cv_idle_.notify_all();
  }
}

}  // namespace disinfect
