// pose_manager.h -- timestamped camera poses (utils/rotation_math/pose_manager.{h,cc}): SLAM
// tracking registers cam_T_world at its frame timestamps, the depth stream looks the pose up at
// its own timestamp (DISINFSystem::feed_rgbd_frame, disinfect_slam.cc:36).
#pragma once

#include <cstdint>
#include <mutex>
#include <utility>
#include <vector>

#include "tsdf_types.h"

namespace disinfect {

class pose_manager {
 public:
  // pose_manager.cc:7-14; timestamps are registered in increasing order (SLAM's frame order)
  void register_valid_pose(int64_t timestamp, const SE3<float>& pose);
  // pose_manager.cc:16-43: identity when empty; else the registered pose nearest in time, the
  // earlier one on a tie-free "closer to old" test (new wins at equal distance). A query before
  // the first timestamp returns the first pose (the reference indexes element -1 there).
  SE3<float> query_pose(int64_t timestamp);
  size_t size();

 private:
  // index of the last pose with timestamp <= t (pose_manager.cc:45-66), -1 if none
  int64_t max_lower_idx(int64_t timestamp) const;
  std::vector<std::pair<int64_t, SE3<float>>> timed_pose_vec_;
  std::mutex vec_lock_;
};

}  // namespace disinfect
