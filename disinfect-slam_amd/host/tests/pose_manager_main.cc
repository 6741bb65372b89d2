// pose_manager_main.cc -- stdin driver of pose_manager for tests/test_host_cpu.py (no GPU):
//   "R <ts> qx qy qz qw tx ty tz"  register_valid_pose
//   "Q <ts>"                        query_pose -> prints "qx qy qz qw tx ty tz" (%.9g)
#include <cstdio>
#include <iostream>
#include <string>

#include "pose_manager.h"

using namespace disinfect;

int main() {
  pose_manager pm;
  std::string op;
  while (std::cin >> op) {
    long long ts;
    std::cin >> ts;
    if (op == "R") {
      float v[7];
      for (float& x : v) std::cin >> x;
      pm.register_valid_pose(ts, SE3<float>(v[0], v[1], v[2], v[3], v[4], v[5], v[6]));
    } else {
      const SE3<float> p = pm.query_pose(ts);
      const Quaternion<float> q = p.GetR();
      const float* t = p.GetT();
      std::printf("%.9g %.9g %.9g %.9g %.9g %.9g %.9g\n", q.x, q.y, q.z, q.w, t[0], t[1], t[2]);
    }
  }
  return 0;
}
