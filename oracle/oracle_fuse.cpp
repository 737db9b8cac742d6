// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// Restatement of the odometry fusion node: odomHandler's callback
// (src/odom_handler_node.cpp:44-132).  Per synchronized pair (A-LOAM odometry, intensity
// odometry): both poses -> 4x4 (Quaterniond::toRotationMatrix, :65-67, :83-85); the first pair
// initialises prev = current and odom_cur = intensity (:88-95); afterwards
// diff = prev.inverse() * cur for both (:98-99) and odom_cur = odom_cur * (child_frame_id ==
// "/odom_skip" ? aloam_diff : intensity_diff) (:101-107) — "/odom_skip" is what the intensity
// tracker publishes when it skipped a frame (intensity_feature_tracker.cpp:722-730, :861-866);
// prev = current (:109-110); the published pose is Quaterniond(rot_cur) and t_cur (:113-128).
// Matrix4d::inverse() of a rigid transform is restated as [R^T, -R^T t] (Eigen's cofactor
// inverse agrees to the last ulps; the 1e-4 pose tolerance absorbs it); 4x4 products sum k = 0..3
// left to right; Quaterniond(Matrix3d) is Eigen's published trace / largest-diagonal algorithm.
#include <cmath>
#include <cstring>

namespace {

void to_mat(const double* p, double* M) {  // (qx, qy, qz, qw, tx, ty, tz) -> row-major 4x4
  const double x = p[0], y = p[1], z = p[2], w = p[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y,
               tyz = tz * y, tzz = tz * z;
  const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                       txz - twy, tyz + twx, 1 - (txx + tyy)};
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) M[4 * r + c] = R[3 * r + c];
    M[4 * r + 3] = p[4 + r];
  }
  M[12] = M[13] = M[14] = 0;
  M[15] = 1;
}

void inv_rigid(const double* M, double* I) {
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) I[4 * r + c] = M[4 * c + r];
    I[4 * r + 3] = -((M[r] * M[3] + M[4 + r] * M[7]) + M[8 + r] * M[11]);
  }
  I[12] = I[13] = I[14] = 0;
  I[15] = 1;
}

void mul(const double* A, const double* B, double* C) {
  double T[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      T[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
  std::memcpy(C, T, sizeof(T));
}

void to_pose(const double* M, double* out) {  // Quaterniond(Matrix3d) + translation
  auto m = [&](int r, int c) { return M[4 * r + c]; };
  double q[4];  // x, y, z, w
  double t = (m(0, 0) + m(1, 1)) + m(2, 2);
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m(2, 1) - m(1, 2)) * t;
    q[1] = (m(0, 2) - m(2, 0)) * t;
    q[2] = (m(1, 0) - m(0, 1)) * t;
  } else {
    int i = 0;
    if (m(1, 1) > m(0, 0)) i = 1;
    if (m(2, 2) > m(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(((m(i, i) - m(j, j)) - m(k, k)) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m(k, j) - m(j, k)) * t;
    q[j] = (m(j, i) + m(i, j)) * t;
    q[k] = (m(k, i) + m(i, k)) * t;
  }
  for (int e = 0; e < 4; e++) out[e] = q[e];
  out[4] = M[3]; out[5] = M[7]; out[6] = M[11];
}

}  // namespace

extern "C" {

// state[49] = prev A-LOAM 4x4, prev intensity 4x4, odom_cur 4x4, initialised flag.
// n pairs aloam[n][7], intensity[n][7] (q x,y,z,w, t), skip[n] (1 = "/odom_skip") -> fused[n][7].
void oracle_odom_fuse(double* state, const double* aloam, const double* intensity, const int* skip, int n,
                      double* fused) {
  double* pa = state;
  double* pi = state + 16;
  double* cur = state + 32;
  for (int f = 0; f < n; f++) {
    double A[16], I[16];
    to_mat(aloam + 7 * f, A);
    to_mat(intensity + 7 * f, I);
    if (state[48] == 0) {
      std::memcpy(pa, A, sizeof(A));
      std::memcpy(pi, I, sizeof(I));
      std::memcpy(cur, I, sizeof(I));
      state[48] = 1;
    } else {
      double inv[16], di[16], da[16];
      inv_rigid(pi, inv);
      mul(inv, I, di);
      inv_rigid(pa, inv);
      mul(inv, A, da);
      mul(cur, skip[f] ? da : di, cur);
      std::memcpy(pa, A, sizeof(A));
      std::memcpy(pi, I, sizeof(I));
    }
    to_pose(cur, fused + 7 * f);
  }
}

}  // extern "C"
