// pose_manager.cc -- utils/rotation_math/pose_manager.cc restated (see the header).
#include "pose_manager.h"

#include <algorithm>

namespace disinfect {

void pose_manager::register_valid_pose(int64_t timestamp, const SE3<float>& pose) {
  std::lock_guard<std::mutex> lock(vec_lock_);
  timed_pose_vec_.emplace_back(timestamp, pose);
}

size_t pose_manager::size() {
  std::lock_guard<std::mutex> lock(vec_lock_);
  return timed_pose_vec_.size();
}

int64_t pose_manager::max_lower_idx(int64_t timestamp) const {
  // upper_bound over the (sorted) timestamps == the reference's recursive binary search + linear
  // scan below 42 elements: the last index whose timestamp is <= the query
  auto it = std::upper_bound(timed_pose_vec_.begin(), timed_pose_vec_.end(), timestamp,
                             [](int64_t t, const std::pair<int64_t, SE3<float>>& e) { return t < e.first; });
  return (int64_t)(it - timed_pose_vec_.begin()) - 1;
}

SE3<float> pose_manager::query_pose(int64_t timestamp) {
  std::lock_guard<std::mutex> lock(vec_lock_);
  if (timed_pose_vec_.empty()) return SE3<float>::Identity();
  const int64_t lo = max_lower_idx(timestamp);
  if (lo < 0) return timed_pose_vec_.front().second;
  if (lo == (int64_t)timed_pose_vec_.size() - 1) return timed_pose_vec_[lo].second;
  const int64_t old_ts = timed_pose_vec_[lo].first, new_ts = timed_pose_vec_[lo + 1].first;
  // closest pose (no SLERP, pose_manager.cc:33-41)
  if ((timestamp - old_ts) < (new_ts - timestamp)) return timed_pose_vec_[lo].second;
  return timed_pose_vec_[lo + 1].second;
}

}  // namespace disinfect
