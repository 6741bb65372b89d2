// tsdf_types.h -- value types of the reference TSDF interface, without Eigen / OpenCV / CUDA.
//
//   CameraIntrinsics<T>, CameraParams   utils/cuda/camera.cuh:12-68
//   SE3<T>                              utils/cuda/lie_group.cuh:6-45 (Eigen::Quaternion + t)
//   BoundingCube<T>                     utils/tsdf/voxel_tsdf.cuh:12-27
//   VoxelSpatialTSDF                    utils/tsdf/voxel_types.cuh:48-57
//   Mat                                 the subset of cv::Mat the TSDF API uses (rows, cols, type,
//                                       data, empty, ones); owns or borrows a dense buffer
// SE3 arithmetic keeps host Eigen 3.3's float evaluation order (SSE quaternion product and
// Packet4f squared norm) so poses composed here match poses composed by the reference host code.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

namespace disinfect {

// ---- cv::Mat subset ----
enum : int { CV_8UC3 = 16, CV_8UC4 = 24, CV_32FC1 = 5, CV_16UC1 = 2, CV_8UC1 = 0 };

inline int mat_elem_size(int type) {
  switch (type) {
    case CV_8UC1: return 1;
    case CV_8UC3: return 3;
    case CV_8UC4: return 4;
    case CV_16UC1: return 2;
    case CV_32FC1: return 4;
    default: throw std::invalid_argument("unsupported Mat type");
  }
}

class Mat {
 public:
  Mat() = default;
  Mat(int rows, int cols, int type) : rows(rows), cols(cols), type_(type) {
    owned_ = std::make_shared<std::vector<uint8_t>>((size_t)rows * cols * mat_elem_size(type));
    data = owned_->data();
  }
  // borrow an external buffer (like cv::Mat(rows, cols, type, data)); caller keeps it alive
  Mat(int rows, int cols, int type, void* ext) : rows(rows), cols(cols), type_(type) {
    data = static_cast<uint8_t*>(ext);
  }
  static Mat ones(int rows, int cols, int type) {
    Mat m(rows, cols, type);
    if (type != CV_32FC1) throw std::invalid_argument("Mat::ones: CV_32FC1 only");
    float* p = reinterpret_cast<float*>(m.data);
    for (size_t i = 0; i < m.total(); ++i) p[i] = 1.0f;
    return m;
  }
  Mat clone() const {
    Mat m(rows, cols, type_);
    if (data) std::memcpy(m.data, data, m.total() * mat_elem_size(type_));
    return m;
  }
  int type() const { return type_; }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  size_t total() const { return (size_t)rows * cols; }
  template <typename T>
  T* ptr() const { return reinterpret_cast<T*>(data); }

  int rows = 0;
  int cols = 0;
  uint8_t* data = nullptr;

 private:
  int type_ = CV_8UC1;
  std::shared_ptr<std::vector<uint8_t>> owned_;
};

// ---- camera.cuh ----
template <typename T>
struct CameraIntrinsics {
  T fx, fy, cx, cy;
  CameraIntrinsics(const T& fx, const T& fy, const T& cx, const T& cy) : fx(fx), fy(fy), cx(cx), cy(cy) {}
  CameraIntrinsics<T> Inverse() const {  // camera.cuh:34-39
    const T fx_inv = 1 / fx;
    const T fy_inv = 1 / fy;
    return CameraIntrinsics<T>(fx_inv, fy_inv, -cx * fx_inv, -cy * fy_inv);
  }
};

struct CameraParams {
  CameraIntrinsics<float> intrinsics;
  CameraIntrinsics<float> intrinsics_inv;
  int img_h;
  int img_w;
  CameraParams(const CameraIntrinsics<float>& intrinsics_, int img_h_, int img_w_)
      : intrinsics(intrinsics_), intrinsics_inv(intrinsics_.Inverse()), img_h(img_h_), img_w(img_w_) {}
};

// ---- lie_group.cuh ----
template <typename T>
struct Quaternion {  // coefficients in Eigen order (x, y, z, w)
  T x = 0, y = 0, z = 0, w = 1;
};

template <typename T>
class SE3 {
 public:
  SE3() = default;
  SE3(const Quaternion<T>& rot, const T trans[3]) : R_(rot) { for (int i = 0; i < 3; ++i) t_[i] = trans[i]; }
  SE3(T qx, T qy, T qz, T qw, T tx, T ty, T tz) {
    R_.x = qx; R_.y = qy; R_.z = qz; R_.w = qw;
    t_[0] = tx; t_[1] = ty; t_[2] = tz;
  }
  // 3x4 / 4x4 row-major matrix [R | t] (lie_group.cuh:15-20 via Eigen's Quaternion(Matrix3))
  static SE3<T> FromMatrix(const T* m, int row_stride);
  static SE3<T> Identity() { return SE3<T>(); }

  SE3<T> Inverse() const {  // lie_group.cuh:22-24
    const Quaternion<T> qi = qinv(R_);
    const T nt[3] = {-t_[0], -t_[1], -t_[2]};
    T ti[3];
    rotate(qi, nt, ti);
    return SE3<T>(qi, ti);
  }
  void Apply(const T v[3], T out[3]) const {  // lie_group.cuh:30-32
    rotate(R_, v, out);
    for (int i = 0; i < 3; ++i) out[i] = out[i] + t_[i];
  }
  SE3<T> operator*(const SE3<T>& o) const {  // lie_group.cuh:34-36
    T rt[3];
    rotate(R_, o.t_, rt);
    const T tt[3] = {rt[0] + t_[0], rt[1] + t_[1], rt[2] + t_[2]};
    return SE3<T>(qmul(R_, o.R_), tt);
  }
  Quaternion<T> GetR() const { return R_; }
  const T* GetT() const { return t_; }

  // Eigen QuaternionBase::_transformVector
  static void rotate(const Quaternion<T>& q, const T v[3], T out[3]) {
    T uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    for (int i = 0; i < 3; ++i) uv[i] += uv[i];
    const T c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
    for (int i = 0; i < 3; ++i) out[i] = (v[i] + q.w * uv[i]) + c[i];
  }
  // Eigen inverse(): conj / squaredNorm, squaredNorm as the Packet4f reduction (x2+z2)+(y2+w2)
  static Quaternion<T> qinv(const Quaternion<T>& q) {
    const T n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
    Quaternion<T> r;
    if (n2 > T(0)) {
      r.x = -q.x / n2; r.y = -q.y / n2; r.z = -q.z / n2; r.w = q.w / n2;
    } else {
      r.x = r.y = r.z = r.w = T(0);
    }
    return r;
  }
  // Eigen quat_product<Architecture::SSE, ..., float> lane arithmetic
  static Quaternion<T> qmul(const Quaternion<T>& a, const Quaternion<T>& b) {
    Quaternion<T> r;
    r.x = (a.x * b.w - a.z * b.y) + (a.y * b.z + a.w * b.x);
    r.y = (a.y * b.w - a.x * b.z) + (a.z * b.x + a.w * b.y);
    r.z = (a.z * b.w - a.y * b.x) + (a.x * b.y + a.w * b.z);
    r.w = (a.w * b.w - a.x * b.x) - (a.z * b.z + a.y * b.y);
    return r;
  }

 private:
  Quaternion<T> R_;
  T t_[3] = {0, 0, 0};
};

template <typename T>
SE3<T> SE3<T>::FromMatrix(const T* m, int rs) {  // Eigen quaternionbase_assign_impl<Matrix3>
  auto M = [&](int i, int j) { return m[i * rs + j]; };
  Quaternion<T> q;
  T t = M(0, 0) + (M(1, 1) + M(2, 2));
  if (t > T(0)) {
    t = std::sqrt(t + T(1.0));
    q.w = T(0.5) * t;
    t = T(0.5) / t;
    q.x = (M(2, 1) - M(1, 2)) * t;
    q.y = (M(0, 2) - M(2, 0)) * t;
    q.z = (M(1, 0) - M(0, 1)) * t;
  } else {
    int i = 0;
    if (M(1, 1) > M(0, 0)) i = 1;
    if (M(2, 2) > M(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + T(1.0));
    T c[3];
    c[i] = T(0.5) * t;
    t = T(0.5) / t;
    q.w = (M(k, j) - M(j, k)) * t;
    c[j] = (M(j, i) + M(i, j)) * t;
    c[k] = (M(k, i) + M(i, k)) * t;
    q.x = c[0]; q.y = c[1]; q.z = c[2];
  }
  const T tr[3] = {M(0, 3), M(1, 3), M(2, 3)};
  return SE3<T>(q, tr);
}

// ---- voxel_tsdf.cuh / voxel_types.cuh ----
template <typename T>
struct BoundingCube {
  T xmin, xmax, ymin, ymax, zmin, zmax;
};

struct VoxelSpatialTSDF {  // 16 B, identical layout to tsdf_voxel of the C ABI
  float position[3];
  float tsdf;
};

}  // namespace disinfect
