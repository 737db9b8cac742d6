/*
 * lislam_factors.h — the cost functors of src/lidarFeaturePointsFunction.hpp with the
 * reference's names, constructors, data members, templated operator() and static Create(), so a
 * caller swaps `#include "lidarFeaturePointsFunction.hpp"` for this header and keeps its code.
 *
 *   reference functor (lidarFeaturePointsFunction.hpp)      lislam_eval_factors_raw kind
 *   front_end_residual          :21-58   (3 residuals; q, t)          3
 *   FeatureMatchingResidual     :61-99   (3; q, t)                    3
 *   LidarGroundPlaneNormFactor  :101-141 (1; q)                       4
 *   LidarPlaneFactor            :143-196 (1; q, t)                    1
 *   LidarPlaneNormFactor        :199-240 (1; q, t)                    2
 *   LidarEdgeFactor             :243-293 (3; q, t)                    0
 *
 * operator()<T>(q, t, residual) is the functor's own expression for any scalar T (double, or an
 * automatic-differentiation type with the usual arithmetic, sqrt / acos / sin / abs found by
 * argument-dependent lookup).  Create(...) returns a lislam::CostFunction whose Evaluate()
 * computes the residuals and the Jacobians w.r.t. the raw parameter blocks — what
 * ceres::AutoDiffCostFunction<F, R, 4, 3> returns — on the GPU through lislam_eval_factors_raw.
 * Ceres calls Evaluate() once per residual block per evaluation pass, all at one parameter point:
 * the first call at a new (q, t) evaluates EVERY live Create()d block at that point in one launch
 * (lidarFeaturePointsFunction.hpp:49-54,183-190,282-288 are the per-block functors this batches),
 * and the pass's other calls are served from that result (lislam::FactorLaunches() counts the
 * launches).  lislam::EvaluateBlocks() evaluates a given list of blocks in one launch, and
 * lislam_normal_equations / lislam_pose_solve (lislam.h) reduce and solve them without leaving
 * the device.
 *
 * Create() takes no context (the reference signature has none): the blocks evaluate on the
 * context given to lislam::SetFactorContext().  The reference passes s = 1 at every call site
 * (DISTORTION 0, laserOdometry.cpp:82,556,679; laserMapping.cpp:718): the device path evaluates
 * identity.slerp(1, q) (= +-q, the same rotation) with analytic Jacobians.  With DISTORTION 1
 * (s = the point's relative time in the sweep) LidarEdgeFactor / LidarPlaneFactor interpolate the
 * pose, Identity.slerp(s, q) and s t: Create() then makes a kind 5 / 6 block that the device
 * differentiates with a forward-mode dual number, as ceres::AutoDiffCostFunction does.
 *
 * Host-side C++ only (any C++11 compiler); link liblislam.so.  With Ceres available, define
 * LISLAM_WITH_CERES before including this header and lislam::CostFunction derives from
 * ceres::CostFunction, so Create()'s result goes straight into Problem::AddResidualBlock.
 */
#ifndef LISLAM_FACTORS_H_
#define LISLAM_FACTORS_H_

#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <mutex>
#include <utility>
#include <vector>

#include "lislam.h"

#ifdef LISLAM_WITH_CERES
#include <ceres/ceres.h>
#endif

namespace lislam {

/* The 3-vector the functors store (Eigen::Vector3d's accessors); constructible from any type with
 * x(), y(), z() (Eigen::Vector3d included). */
struct Vector3d {
  double v[3];
  Vector3d() : v{0.0, 0.0, 0.0} {}
  Vector3d(double x_, double y_, double z_) : v{x_, y_, z_} {}
  template <class V, class = decltype(std::declval<const V&>().x() + std::declval<const V&>().z())>
  Vector3d(const V& o) : v{double(o.x()), double(o.y()), double(o.z())} {}
  double x() const { return v[0]; }
  double y() const { return v[1]; }
  double z() const { return v[2]; }
  Vector3d operator-(const Vector3d& o) const { return Vector3d(v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]); }
  Vector3d cross(const Vector3d& o) const {
    return Vector3d(v[1] * o.v[2] - v[2] * o.v[1], v[2] * o.v[0] - v[0] * o.v[2], v[0] * o.v[1] - v[1] * o.v[0]);
  }
  void normalize() {  // Eigen: divide by the norm unless it is zero
    const double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    if (sq > 0.0) {
      const double r = std::sqrt(sq);
      v[0] /= r; v[1] /= r; v[2] /= r;
    }
  }
};

namespace detail {
/* Eigen's Quaternion * Vector3 (_transformVector) for quaternion coefficients (x, y, z, w):
 * uv = 2 (u x c); c + w uv + u x uv. */
template <typename T>
inline void rotate(const T& qx, const T& qy, const T& qz, const T& qw, const T* c, T* out) {
  T uv[3] = {qy * c[2] - qz * c[1], qz * c[0] - qx * c[2], qx * c[1] - qy * c[0]};
  uv[0] = uv[0] + uv[0]; uv[1] = uv[1] + uv[1]; uv[2] = uv[2] + uv[2];
  out[0] = (c[0] + qw * uv[0]) + (qy * uv[2] - qz * uv[1]);
  out[1] = (c[1] + qw * uv[1]) + (qz * uv[0] - qx * uv[2]);
  out[2] = (c[2] + qw * uv[2]) + (qx * uv[1] - qy * uv[0]);
}
/* Eigen's QuaternionBase::slerp(s, other) from the identity, in coefficient order (x, y, z, w). */
template <typename T>
inline void slerp_from_identity(const T& s, const T* q, T* out) {
  using std::abs;
  using std::acos;
  using std::sin;
  const T one = T(1) - T(std::numeric_limits<double>::epsilon());
  const T d = q[3];  // identity . q
  const T absD = abs(d);
  T scale0, scale1;
  if (absD >= one) {
    scale0 = T(1) - s;
    scale1 = s;
  } else {
    const T theta = acos(absD);
    const T sinTheta = sin(theta);
    scale0 = sin((T(1) - s) * theta) / sinTheta;
    scale1 = sin(s * theta) / sinTheta;
  }
  if (d < T(0)) scale1 = -scale1;
  out[0] = scale1 * q[0];
  out[1] = scale1 * q[1];
  out[2] = scale1 * q[2];
  out[3] = scale0 + scale1 * q[3];
}
inline lislam_ctx*& factor_context() {
  static lislam_ctx* ctx = nullptr;
  return ctx;
}
}  // namespace detail

/* The context Create()d blocks evaluate on (one per process / GPU, as the reference runs one
 * Ceres problem per node). */
inline void SetFactorContext(lislam_ctx* ctx) { detail::factor_context() = ctx; }

/* ceres::CostFunction's evaluation surface: Evaluate(parameters, residuals, jacobians) with
 * jacobians[i] row-major num_residuals x parameter_block_sizes()[i] (or null). */
#ifdef LISLAM_WITH_CERES
class CostFunction : public ceres::CostFunction {
 protected:
  void init(int residuals, const std::vector<int32_t>& blocks) {
    set_num_residuals(residuals);
    *mutable_parameter_block_sizes() = blocks;
  }
};
#else
class CostFunction {
 public:
  virtual ~CostFunction() {}
  virtual bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const = 0;
  int num_residuals() const { return num_residuals_; }
  const std::vector<int32_t>& parameter_block_sizes() const { return blocks_; }

 protected:
  void init(int residuals, const std::vector<int32_t>& blocks) {
    num_residuals_ = residuals;
    blocks_ = blocks;
  }

 private:
  int num_residuals_ = 0;
  std::vector<int32_t> blocks_;
};
#endif

class DeviceCostFunction;

namespace detail {
/* One batched evaluation: the blocks of one group (one Ceres problem) at one parameter point. */
struct FactorBatch {
  unsigned long long group = 0;  // the group whose blocks the launch held (0: none yet)
  unsigned long long generation = 0;
  double cq[4] = {0, 0, 0, 0}, ct[3] = {0, 0, 0};  // the parameter values it was evaluated at
  std::vector<int32_t> index;  // registry slot -> row of this batch's outputs, -1 = not in it
  std::vector<double> res, jq, jt;  // [rows][3], [rows][3][4], [rows][3][3]
  unsigned long long used = 0;      // LRU stamp
};
/* Every live DeviceCostFunction, packed as lislam_eval_factors_raw records, and the batches of the
 * parameter points they were last evaluated at.  Blocks are grouped by problem, not by the
 * parameter-block pointers Evaluate sees: Ceres' evaluator points each block's state into its own
 * x / candidate-x vectors, so those pointers change between evaluations of one problem.  A block
 * with no group joins the group of the first batch that serves it (its values matched); a miss
 * launches the block's whole group (plus every block with no group yet) at the new values, into the
 * least recently used batch.  So a problem's pass is one launch, and two live problems at different
 * poses do not evict each other.  One per process (the blocks evaluate on the one
 * SetFactorContext() context); the mutex serializes Ceres' evaluation threads. */
struct FactorRegistry {
  std::mutex mu;
  std::vector<DeviceCostFunction*> blocks;  // slot i = blocks[i]
  std::vector<int32_t> kinds;
  std::vector<double> recs;                  // [n][12]
  std::vector<unsigned long long> group;     // per slot: its problem's group (0: not evaluated yet)
  unsigned long long generation = 0;         // bumped by every Create() / destruction
  unsigned long long next_group = 0;
  static constexpr int kBatches = 4;
  FactorBatch batch[kBatches];
  unsigned long long clock = 0;
  long long launches = 0;
};
inline FactorRegistry& factor_registry() {
  static FactorRegistry r;
  return r;
}
}  // namespace detail

/* lislam_eval_factors_raw launches made by DeviceCostFunction::Evaluate so far. */
inline long long FactorLaunches() {
  detail::FactorRegistry& g = detail::factor_registry();
  std::lock_guard<std::mutex> lock(g.mu);
  return g.launches;
}

/* One residual block evaluated on the GPU: the functor's data packed as a
 * lislam_eval_factors_raw record (kind, 12 doubles), registered for the batched evaluation. */
class DeviceCostFunction : public CostFunction {
 public:
  DeviceCostFunction(int kind, int residuals, const double* rec12) : kind_(kind), residuals_(residuals) {
    for (int k = 0; k < 12; k++) rec_[k] = rec12[k];
    init(residuals, kind == 4 ? std::vector<int32_t>{4} : std::vector<int32_t>{4, 3});
    detail::FactorRegistry& g = detail::factor_registry();
    std::lock_guard<std::mutex> lock(g.mu);
    slot_ = g.blocks.size();
    g.blocks.push_back(this);
    g.kinds.push_back(kind);
    g.recs.insert(g.recs.end(), rec_, rec_ + 12);
    g.group.push_back(0);
    g.generation++;
  }
  ~DeviceCostFunction() override {
    detail::FactorRegistry& g = detail::factor_registry();
    std::lock_guard<std::mutex> lock(g.mu);
    const size_t last = g.blocks.size() - 1;
    if (slot_ != last) {  // the last block moves into this slot
      DeviceCostFunction* m = g.blocks[last];
      g.blocks[slot_] = m;
      g.kinds[slot_] = g.kinds[last];
      std::memcpy(&g.recs[slot_ * 12], &g.recs[last * 12], 12 * sizeof(double));
      g.group[slot_] = g.group[last];
      m->slot_ = slot_;
    }
    g.blocks.pop_back();
    g.kinds.pop_back();
    g.recs.resize(last * 12);
    g.group.pop_back();
    g.generation++;
  }
  DeviceCostFunction(const DeviceCostFunction&) = delete;
  DeviceCostFunction& operator=(const DeviceCostFunction&) = delete;
  int kind() const { return kind_; }
  const double* record() const { return rec_; }

  bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const override {
    lislam_ctx* ctx = detail::factor_context();
    if (!ctx) {
      std::fprintf(stderr, "lislam_factors: no context (call lislam::SetFactorContext first)\n");
      return false;
    }
    static const double zero_t[3] = {0.0, 0.0, 0.0};
    const double* q = parameters[0];
    const double* pt = kind_ == 4 ? nullptr : parameters[1];
    detail::FactorRegistry& g = detail::factor_registry();
    std::lock_guard<std::mutex> lock(g.mu);
    // a batch that holds this block at these values (the ground factor has no t block: its
    // residual ignores t, so any batch at its q serves it)
    auto at = [&](const detail::FactorBatch& e) {
      return std::memcmp(e.cq, q, sizeof(e.cq)) == 0 && (kind_ == 4 || std::memcmp(e.ct, pt, sizeof(e.ct)) == 0);
    };
    detail::FactorBatch* b = nullptr;
    for (detail::FactorBatch& e : g.batch)
      if (e.generation == g.generation && slot_ < e.index.size() && e.index[slot_] >= 0 && at(e)) b = &e;
    if (!b) {
      // a new parameter point of this block's problem: every block of its group, and every block not
      // evaluated yet, at (q, t) in one launch, into the least recently used batch
      b = &g.batch[0];
      for (detail::FactorBatch& e : g.batch)
        if (e.used < b->used) b = &e;
      unsigned long long grp = g.group[slot_];
      if (grp == 0) grp = ++g.next_group;
      const double* t = kind_ == 4 ? zero_t : pt;
      const size_t n = g.blocks.size();
      b->index.assign(n, -1);
      std::vector<int32_t> kinds;
      std::vector<double> recs;
      for (size_t i = 0; i < n; i++) {
        if (g.group[i] != grp && g.group[i] != 0) continue;
        b->index[i] = (int32_t)kinds.size();
        kinds.push_back(g.kinds[i]);
        recs.insert(recs.end(), &g.recs[i * 12], &g.recs[i * 12] + 12);
      }
      const size_t rows = kinds.size();
      b->res.resize(rows * 3);
      b->jq.resize(rows * 12);
      b->jt.resize(rows * 9);
      b->generation = 0;
      if (lislam_eval_factors_raw(ctx, (int32_t)rows, kinds.data(), recs.data(), q, t, b->res.data(), b->jq.data(),
                                  b->jt.data()) != LISLAM_OK)
        return false;
      g.launches++;
      b->group = grp;
      std::memcpy(b->cq, q, sizeof(b->cq));
      std::memcpy(b->ct, t, sizeof(b->ct));
      b->generation = g.generation;
    }
    // the block belongs to the group of the first batch that serves it
    if (g.group[slot_] == 0) g.group[slot_] = b->group;
    b->used = ++g.clock;
    const size_t row = (size_t)b->index[slot_];
    const bool want_q = jacobians && jacobians[0], want_t = jacobians && kind_ != 4 && jacobians[1];
    const double* r = &b->res[row * 3];
    const double* jq = &b->jq[row * 12];
    const double* jt = &b->jt[row * 9];
    for (int i = 0; i < residuals_; i++) {
      residuals[i] = r[i];
      if (want_q)
        for (int c = 0; c < 4; c++) jacobians[0][i * 4 + c] = jq[i * 4 + c];
      if (want_t)
        for (int c = 0; c < 3; c++) jacobians[1][i * 3 + c] = jt[i * 3 + c];
    }
    return true;
  }

 private:
  int kind_, residuals_;
  double rec_[12];
  size_t slot_ = 0;
};

/* Evaluate many Create()d blocks at one (q, t) in a single launch: residuals[n][3] and raw
 * Jacobians jac_q[n][3][4], jac_t[n][3][3] (rows past a block's size are zero; outputs
 * optional).  Returns the lislam status. */
inline int EvaluateBlocks(const std::vector<const CostFunction*>& blocks, const double* q, const double* t,
                          double* residuals, double* jac_q, double* jac_t) {
  lislam_ctx* ctx = detail::factor_context();
  if (!ctx) return LISLAM_ERR_STATE;
  std::vector<int32_t> kinds(blocks.size());
  std::vector<double> recs(blocks.size() * 12);
  for (size_t i = 0; i < blocks.size(); i++) {
    const DeviceCostFunction* d = dynamic_cast<const DeviceCostFunction*>(blocks[i]);
    if (!d) return LISLAM_ERR_ARG;
    kinds[i] = d->kind();
    for (int k = 0; k < 12; k++) recs[i * 12 + k] = d->record()[k];
  }
  return lislam_eval_factors_raw(ctx, (int32_t)blocks.size(), kinds.data(), recs.data(), q, t, residuals, jac_q,
                                 jac_t);
}

namespace detail {
inline void put3(double* r, const Vector3d& v) { r[0] = v.x(); r[1] = v.y(); r[2] = v.z(); }
}  // namespace detail

}  // namespace lislam

/* ------------------------------------------------------------------ the reference functors */

struct front_end_residual {  // lidarFeaturePointsFunction.hpp:21-58
  front_end_residual(lislam::Vector3d src_point_, lislam::Vector3d dst_point_)
      : src_point(src_point_), dst_point(dst_point_) {}

  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    const T cp[3] = {T(src_point.x()), T(src_point.y()), T(src_point.z())};
    T p[3];
    lislam::detail::rotate(q[0], q[1], q[2], q[3], cp, p);
    residual[0] = (p[0] + t[0]) - T(dst_point.x());
    residual[1] = (p[1] + t[1]) - T(dst_point.y());
    residual[2] = (p[2] + t[2]) - T(dst_point.z());
    return true;
  }

  static lislam::CostFunction* Create(const lislam::Vector3d src_point_, const lislam::Vector3d dst_point_) {
    double rec[12] = {0};
    lislam::detail::put3(rec, src_point_);
    lislam::detail::put3(rec + 3, dst_point_);
    return new lislam::DeviceCostFunction(3, 3, rec);
  }

  lislam::Vector3d src_point, dst_point;
};

struct FeatureMatchingResidual {  // lidarFeaturePointsFunction.hpp:61-99
  FeatureMatchingResidual(lislam::Vector3d curr_point_, lislam::Vector3d prev_point_)
      : curr_point(curr_point_), prev_point(prev_point_) {}

  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    const T cp[3] = {T(curr_point.x()), T(curr_point.y()), T(curr_point.z())};
    T p[3];
    lislam::detail::rotate(q[0], q[1], q[2], q[3], cp, p);
    residual[0] = (p[0] + t[0]) - T(prev_point.x());
    residual[1] = (p[1] + t[1]) - T(prev_point.y());
    residual[2] = (p[2] + t[2]) - T(prev_point.z());
    return true;
  }

  static lislam::CostFunction* Create(const lislam::Vector3d curr_point_, const lislam::Vector3d prev_point_) {
    double rec[12] = {0};
    lislam::detail::put3(rec, curr_point_);
    lislam::detail::put3(rec + 3, prev_point_);
    return new lislam::DeviceCostFunction(3, 3, rec);
  }

  lislam::Vector3d curr_point, prev_point;
};

struct LidarGroundPlaneNormFactor {  // lidarFeaturePointsFunction.hpp:101-141
  LidarGroundPlaneNormFactor(lislam::Vector3d curr_point_, lislam::Vector3d plane_unit_norm_,
                             double negative_OA_dot_norm_)
      : curr_point(curr_point_), plane_unit_norm(plane_unit_norm_), negative_OA_dot_norm(negative_OA_dot_norm_) {}

  template <typename T>
  bool operator()(const T* q, T* residual) const {
    const T cp[3] = {T(curr_point.x()), T(curr_point.y()), T(curr_point.z())};
    T p[3];
    lislam::detail::rotate(q[0], q[1], q[2], q[3], cp, p);
    residual[0] = (T(plane_unit_norm.x()) * p[0] + T(plane_unit_norm.y()) * p[1] + T(plane_unit_norm.z()) * p[2]) +
                  T(negative_OA_dot_norm);
    return true;
  }

  static lislam::CostFunction* Create(const lislam::Vector3d curr_point_, const lislam::Vector3d plane_unit_norm_,
                                      const double negative_OA_dot_norm_) {
    double rec[12] = {0};
    lislam::detail::put3(rec, curr_point_);
    lislam::detail::put3(rec + 3, plane_unit_norm_);
    rec[6] = negative_OA_dot_norm_;
    return new lislam::DeviceCostFunction(4, 1, rec);
  }

  lislam::Vector3d curr_point;
  lislam::Vector3d plane_unit_norm;
  double negative_OA_dot_norm;
};

struct LidarPlaneFactor {  // lidarFeaturePointsFunction.hpp:143-196
  LidarPlaneFactor(lislam::Vector3d curr_point_, lislam::Vector3d last_point_j_, lislam::Vector3d last_point_l_,
                   lislam::Vector3d last_point_m_, double s_)
      : curr_point(curr_point_), last_point_j(last_point_j_), last_point_l(last_point_l_),
        last_point_m(last_point_m_), s(s_) {
    ljm_norm = (last_point_j - last_point_l).cross(last_point_j - last_point_m);
    ljm_norm.normalize();
  }

  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    const T cp[3] = {T(curr_point.x()), T(curr_point.y()), T(curr_point.z())};
    const T qq[4] = {q[0], q[1], q[2], q[3]};
    T ql[4], p[3];
    lislam::detail::slerp_from_identity(T(s), qq, ql);
    lislam::detail::rotate(ql[0], ql[1], ql[2], ql[3], cp, p);
    const T lp[3] = {p[0] + T(s) * t[0], p[1] + T(s) * t[1], p[2] + T(s) * t[2]};
    residual[0] = ((lp[0] - T(last_point_j.x())) * T(ljm_norm.x()) + (lp[1] - T(last_point_j.y())) * T(ljm_norm.y())) +
                  (lp[2] - T(last_point_j.z())) * T(ljm_norm.z());
    return true;
  }

  static lislam::CostFunction* Create(const lislam::Vector3d curr_point_, const lislam::Vector3d last_point_j_,
                                      const lislam::Vector3d last_point_l_, const lislam::Vector3d last_point_m_,
                                      const double s_) {
    double rec[12];
    lislam::detail::put3(rec, curr_point_);
    lislam::detail::put3(rec + 3, last_point_j_);
    if (s_ != 1.0) {  // DISTORTION 1: (curr, j, the constructor's unit normal, s), kind 6
      const LidarPlaneFactor f(curr_point_, last_point_j_, last_point_l_, last_point_m_, s_);
      lislam::detail::put3(rec + 6, f.ljm_norm);
      rec[9] = s_;
      rec[10] = rec[11] = 0.0;
      return new lislam::DeviceCostFunction(6, 1, rec);
    }
    lislam::detail::put3(rec + 6, last_point_l_);
    lislam::detail::put3(rec + 9, last_point_m_);
    return new lislam::DeviceCostFunction(1, 1, rec);
  }

  lislam::Vector3d curr_point, last_point_j, last_point_l, last_point_m;
  lislam::Vector3d ljm_norm;
  double s;
};

struct LidarPlaneNormFactor {  // lidarFeaturePointsFunction.hpp:199-240
  LidarPlaneNormFactor(lislam::Vector3d curr_point_, lislam::Vector3d plane_unit_norm_, double negative_OA_dot_norm_)
      : curr_point(curr_point_), plane_unit_norm(plane_unit_norm_), negative_OA_dot_norm(negative_OA_dot_norm_) {}

  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    const T cp[3] = {T(curr_point.x()), T(curr_point.y()), T(curr_point.z())};
    T p[3];
    lislam::detail::rotate(q[0], q[1], q[2], q[3], cp, p);
    const T pw[3] = {p[0] + t[0], p[1] + t[1], p[2] + t[2]};
    residual[0] = (T(plane_unit_norm.x()) * pw[0] + T(plane_unit_norm.y()) * pw[1] + T(plane_unit_norm.z()) * pw[2]) +
                  T(negative_OA_dot_norm);
    return true;
  }

  static lislam::CostFunction* Create(const lislam::Vector3d curr_point_, const lislam::Vector3d plane_unit_norm_,
                                      const double negative_OA_dot_norm_) {
    double rec[12] = {0};
    lislam::detail::put3(rec, curr_point_);
    lislam::detail::put3(rec + 3, plane_unit_norm_);
    rec[6] = negative_OA_dot_norm_;
    return new lislam::DeviceCostFunction(2, 1, rec);
  }

  lislam::Vector3d curr_point;
  lislam::Vector3d plane_unit_norm;
  double negative_OA_dot_norm;
};

struct LidarEdgeFactor {  // lidarFeaturePointsFunction.hpp:243-293
  LidarEdgeFactor(lislam::Vector3d curr_point_, lislam::Vector3d last_point_a_, lislam::Vector3d last_point_b_,
                  double s_)
      : curr_point(curr_point_), last_point_a(last_point_a_), last_point_b(last_point_b_), s(s_) {}

  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    using std::sqrt;
    const T cp[3] = {T(curr_point.x()), T(curr_point.y()), T(curr_point.z())};
    const T lpa[3] = {T(last_point_a.x()), T(last_point_a.y()), T(last_point_a.z())};
    const T lpb[3] = {T(last_point_b.x()), T(last_point_b.y()), T(last_point_b.z())};
    const T qq[4] = {q[0], q[1], q[2], q[3]};
    T ql[4], p[3];
    lislam::detail::slerp_from_identity(T(s), qq, ql);
    lislam::detail::rotate(ql[0], ql[1], ql[2], ql[3], cp, p);
    const T lp[3] = {p[0] + T(s) * t[0], p[1] + T(s) * t[1], p[2] + T(s) * t[2]};
    const T da[3] = {lp[0] - lpa[0], lp[1] - lpa[1], lp[2] - lpa[2]};
    const T db[3] = {lp[0] - lpb[0], lp[1] - lpb[1], lp[2] - lpb[2]};
    const T nu[3] = {da[1] * db[2] - da[2] * db[1], da[2] * db[0] - da[0] * db[2], da[0] * db[1] - da[1] * db[0]};
    const T de[3] = {lpa[0] - lpb[0], lpa[1] - lpb[1], lpa[2] - lpb[2]};
    const T nde = sqrt((de[0] * de[0] + de[1] * de[1]) + de[2] * de[2]);
    residual[0] = nu[0] / nde;
    residual[1] = nu[1] / nde;
    residual[2] = nu[2] / nde;
    return true;
  }

  static lislam::CostFunction* Create(const lislam::Vector3d curr_point_, const lislam::Vector3d last_point_a_,
                                      const lislam::Vector3d last_point_b_, const double s_) {
    double rec[12] = {0};
    lislam::detail::put3(rec, curr_point_);
    lislam::detail::put3(rec + 3, last_point_a_);
    lislam::detail::put3(rec + 6, last_point_b_);
    if (s_ != 1.0) {  // DISTORTION 1: (curr, a, b, s), kind 5
      rec[9] = s_;
      return new lislam::DeviceCostFunction(5, 3, rec);
    }
    return new lislam::DeviceCostFunction(0, 3, rec);
  }

  lislam::Vector3d curr_point, last_point_a, last_point_b;
  double s;
};

#endif /* LISLAM_FACTORS_H_ */
