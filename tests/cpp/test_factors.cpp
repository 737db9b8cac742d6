// A ROS-free C++ consumer of the drop-in boundary (include/lislam.h + include/lislam_factors.h):
// residual blocks are built through the reference functors' Create() (lidarFeaturePointsFunction.hpp
// signatures), evaluated on the GPU through their CostFunction::Evaluate and through one batched
// lislam::EvaluateBlocks launch, and compared with the oracle's Ceres-Jet autodiff restatement
// (oracle/oracle_solver.hpp, test infrastructure) and with the header functors' own operator()<double>.
// Run by tests/test_gpu_factors_cpp.py; prints "factors ok" and exits 0 on success.
#include <cmath>
#include <cstdio>
#include <memory>
#include <random>
#include <vector>

#include "lislam.h"
#include "lislam_factors.h"
#include "oracle_solver.hpp"

static int g_fail = 0;
static void check(bool ok, const char* what, int i, double a, double b) {
  if (!ok) {
    if (g_fail < 20) std::fprintf(stderr, "MISMATCH %s block %d: %.17g vs %.17g\n", what, i, a, b);
    g_fail++;
  }
}
static bool close(double a, double b, double rtol, double atol) { return std::fabs(a - b) <= atol + rtol * std::fabs(b); }

int main() {
  lislam_config cfg{64, 1024, 0.3f, 4, 0};
  lislam_ctx* ctx = nullptr;
  if (lislam_ctx_create(&cfg, 0, &ctx) != LISLAM_OK) {
    std::fprintf(stderr, "lislam_ctx_create failed\n");
    return 2;
  }
  lislam::SetFactorContext(ctx);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-5.0, 5.0), A(-0.3, 0.3);
  auto v3 = [&]() { return lislam::Vector3d(U(rng), U(rng), U(rng)); };
  const int n_per = 40;
  std::vector<std::unique_ptr<lislam::CostFunction>> owned;
  std::vector<const lislam::CostFunction*> blocks;
  struct Ref {
    int kind;
    double rec[12];
  };
  std::vector<Ref> refs;
  // parameters: a unit quaternion (x, y, z, w) near identity and a translation
  double q[4] = {A(rng), A(rng), A(rng), 0.0}, t[3] = {U(rng), U(rng), U(rng)};
  q[3] = std::sqrt(1.0 - q[0] * q[0] - q[1] * q[1] - q[2] * q[2]);
  for (int kind = 0; kind < 5; kind++) {
    for (int i = 0; i < n_per; i++) {
      Ref r{kind, {0}};
      lislam::Vector3d c = v3(), a = v3(), b = v3(), m = v3();
      lislam::Vector3d nrm = v3();
      nrm.normalize();
      const double d = U(rng);
      lislam::CostFunction* f = nullptr;
      double host_r[3] = {0, 0, 0};
      int R = 1;
      switch (kind) {
        case 0: {
          f = LidarEdgeFactor::Create(c, a, b, 1.0);
          LidarEdgeFactor(c, a, b, 1.0)(q, t, host_r);
          R = 3;
          for (int k = 0; k < 3; k++) { r.rec[k] = c.v[k]; r.rec[3 + k] = a.v[k]; r.rec[6 + k] = b.v[k]; }
          break;
        }
        case 1: {
          f = LidarPlaneFactor::Create(c, a, b, m, 1.0);
          LidarPlaneFactor(c, a, b, m, 1.0)(q, t, host_r);
          for (int k = 0; k < 3; k++) { r.rec[k] = c.v[k]; r.rec[3 + k] = a.v[k]; r.rec[6 + k] = b.v[k]; r.rec[9 + k] = m.v[k]; }
          break;
        }
        case 2: {
          f = LidarPlaneNormFactor::Create(c, nrm, d);
          LidarPlaneNormFactor(c, nrm, d)(q, t, host_r);
          for (int k = 0; k < 3; k++) { r.rec[k] = c.v[k]; r.rec[3 + k] = nrm.v[k]; }
          r.rec[6] = d;
          break;
        }
        case 3: {
          f = (i & 1) ? FeatureMatchingResidual::Create(c, a) : front_end_residual::Create(c, a);
          if (i & 1) FeatureMatchingResidual(c, a)(q, t, host_r);
          else front_end_residual(c, a)(q, t, host_r);
          R = 3;
          for (int k = 0; k < 3; k++) { r.rec[k] = c.v[k]; r.rec[3 + k] = a.v[k]; }
          break;
        }
        default: {
          f = LidarGroundPlaneNormFactor::Create(c, nrm, d);
          LidarGroundPlaneNormFactor(c, nrm, d)(q, host_r);
          for (int k = 0; k < 3; k++) { r.rec[k] = c.v[k]; r.rec[3 + k] = nrm.v[k]; }
          r.rec[6] = d;
        }
      }
      if (!f || f->num_residuals() != R) {
        std::fprintf(stderr, "Create failed for kind %d\n", kind);
        return 3;
      }
      const int idx = (int)refs.size();
      // the block's own Evaluate (one GPU launch)
      double res[3], jq[12], jt[9];
      const double* params[2] = {q, t};
      double* jacs[2] = {jq, jt};
      if (!f->Evaluate(params, res, jacs)) {
        std::fprintf(stderr, "Evaluate failed: %s\n", lislam_last_error(ctx));
        return 4;
      }
      // oracle: Ceres-Jet autodiff of the restated functor (7 columns: q x y z w, t)
      double orr[3] = {0, 0, 0}, oJ[21] = {0};
      const double tz[3] = {0, 0, 0};
      switch (kind) {
        case 0: {
          oracle::EdgeFactor F{{c.v[0], c.v[1], c.v[2]}, {a.v[0], a.v[1], a.v[2]}, {b.v[0], b.v[1], b.v[2]}, 1.0};
          oracle::autodiff_eval(F, q, t, orr, oJ);
          break;
        }
        case 1: {
          oracle::PlaneFactor F(c.v, a.v, b.v, m.v, 1.0);
          oracle::autodiff_eval(F, q, t, orr, oJ);
          break;
        }
        case 3: {
          oracle::P2PFactor F{{c.v[0], c.v[1], c.v[2]}, {a.v[0], a.v[1], a.v[2]}};
          oracle::autodiff_eval(F, q, t, orr, oJ);
          break;
        }
        default: {  // plane-norm; the ground factor is the same expression without t
          oracle::PlaneNormFactor F{{c.v[0], c.v[1], c.v[2]}, {nrm.v[0], nrm.v[1], nrm.v[2]}, d};
          oracle::autodiff_eval(F, q, kind == 4 ? tz : t, orr, oJ);
        }
      }
      for (int k = 0; k < R; k++) {
        check(close(res[k], orr[k], 1e-12, 1e-12), "residual vs oracle", idx, res[k], orr[k]);
        check(close(res[k], host_r[k], 1e-12, 1e-12), "residual vs header operator()", idx, res[k], host_r[k]);
        for (int cc = 0; cc < 4; cc++)
          check(close(jq[k * 4 + cc], oJ[k * 7 + cc], 1e-9, 1e-10), "d r / d q vs oracle autodiff", idx, jq[k * 4 + cc],
                oJ[k * 7 + cc]);
        if (kind != 4)
          for (int cc = 0; cc < 3; cc++)
            check(close(jt[k * 3 + cc], oJ[k * 7 + 4 + cc], 1e-9, 1e-10), "d r / d t vs oracle autodiff", idx,
                  jt[k * 3 + cc], oJ[k * 7 + 4 + cc]);
      }
      refs.push_back(r);
      blocks.push_back(f);
      owned.emplace_back(f);
    }
  }
  // every block in one launch == the per-block evaluations above (same device code)
  const size_t n = blocks.size();
  std::vector<double> R3(n * 3), JQ(n * 12), JT(n * 9);
  if (lislam::EvaluateBlocks(blocks, q, t, R3.data(), JQ.data(), JT.data()) != LISLAM_OK) {
    std::fprintf(stderr, "EvaluateBlocks failed: %s\n", lislam_last_error(ctx));
    return 5;
  }
  for (size_t i = 0; i < n; i++) {
    double res[3], jq[12], jt[9];
    const double* params[2] = {q, t};
    double* jacs[2] = {jq, jt};
    blocks[i]->Evaluate(params, res, jacs);
    for (int k = 0; k < blocks[i]->num_residuals(); k++) {
      check(R3[i * 3 + k] == res[k], "batched residual", (int)i, R3[i * 3 + k], res[k]);
      for (int cc = 0; cc < 4; cc++) check(JQ[i * 12 + k * 4 + cc] == jq[k * 4 + cc], "batched J_q", (int)i, 0, 0);
    }
  }
  // laserOdometry's problem size (64 lines: 768 edge + 1536 plane blocks, laserOdometry.cpp:
  // 556-700): Ceres evaluates every residual block through Evaluate() at each parameter point of
  // the solve; the first call at a new point evaluates all registered blocks in ONE launch and the
  // others are served from it (lislam::FactorLaunches), bit-equal to a per-list EvaluateBlocks.
  {
    std::vector<std::unique_ptr<lislam::CostFunction>> prob;
    std::vector<const lislam::CostFunction*> pb;
    for (int i = 0; i < 2304; i++) {
      lislam::CostFunction* f = i < 768 ? LidarEdgeFactor::Create(v3(), v3(), v3(), 1.0)
                                        : LidarPlaneFactor::Create(v3(), v3(), v3(), v3(), 1.0);
      prob.emplace_back(f);
      pb.push_back(f);
    }
    const int points = 5;
    for (int pt = 0; pt < points; pt++) {
      double qq[4] = {A(rng), A(rng), A(rng), 0.0}, tt[3] = {U(rng), U(rng), U(rng)};
      qq[3] = std::sqrt(1.0 - qq[0] * qq[0] - qq[1] * qq[1] - qq[2] * qq[2]);
      const long long before = lislam::FactorLaunches();
      std::vector<double> R3p(pb.size() * 3), JQp(pb.size() * 12), JTp(pb.size() * 9);
      if (lislam::EvaluateBlocks(pb, qq, tt, R3p.data(), JQp.data(), JTp.data()) != LISLAM_OK) return 7;
      const double* params[2] = {qq, tt};
      for (int pass = 0; pass < 2; pass++) {  // cost-only pass, then with Jacobians (as Ceres does)
        for (size_t i = 0; i < pb.size(); i++) {
          double res[3], jq[12], jt[9];
          double* jacs[2] = {jq, jt};
          if (!pb[i]->Evaluate(params, res, pass ? jacs : nullptr)) return 8;
          for (int k = 0; k < pb[i]->num_residuals(); k++) {
            check(res[k] == R3p[i * 3 + k], "2304-block residual", (int)i, res[k], R3p[i * 3 + k]);
            if (pass) {
              for (int cc = 0; cc < 4; cc++) check(jq[k * 4 + cc] == JQp[i * 12 + k * 4 + cc], "2304-block J_q", (int)i, 0, 0);
              for (int cc = 0; cc < 3; cc++) check(jt[k * 3 + cc] == JTp[i * 9 + k * 3 + cc], "2304-block J_t", (int)i, 0, 0);
            }
          }
        }
      }
      const long long used = lislam::FactorLaunches() - before;
      if (used != 1) {
        std::fprintf(stderr, "point %d: %lld launches for 2304 blocks x 2 passes (want 1)\n", pt, used);
        g_fail++;
      }
    }
    std::printf("batched: 2304 blocks, %d parameter points, 1 launch each\n", points);
    // Ceres' evaluator points the parameter blocks into its own x / candidate-x vectors, so the
    // pointers Evaluate sees change between evaluations of one problem: each point is evaluated
    // from two buffers in turn (cost pass from one, Jacobian pass from the other, holding the same
    // values), and a point seen before (an accepted candidate re-evaluated at x) is served from its
    // batch.  Still one launch per new point, none for a repeated one.
    double bufq[2][4], buft[2][3];
    const long long before = lislam::FactorLaunches();
    double prev_q[4] = {0, 0, 0, 1}, prev_t[3] = {0, 0, 0};
    for (int pt = 0; pt < points; pt++) {
      double qq[4] = {A(rng), A(rng), A(rng), 0.0}, tt[3] = {U(rng), U(rng), U(rng)};
      qq[3] = std::sqrt(1.0 - qq[0] * qq[0] - qq[1] * qq[1] - qq[2] * qq[2]);
      if (pt == points - 1) {  // the previous point again (from the other buffer)
        std::memcpy(qq, prev_q, sizeof(qq));
        std::memcpy(tt, prev_t, sizeof(tt));
      }
      for (int pass = 0; pass < 2; pass++) {
        const int w = (pt + pass) % 2;
        std::memcpy(bufq[w], qq, sizeof(qq));
        std::memcpy(buft[w], tt, sizeof(tt));
        const double* params[2] = {bufq[w], buft[w]};
        for (size_t i = 0; i < pb.size(); i++) {
          double res[3], jq[12], jt[9];
          double* jacs[2] = {jq, jt};
          if (!pb[i]->Evaluate(params, res, pass ? jacs : nullptr)) return 8;
        }
      }
      std::memcpy(prev_q, qq, sizeof(qq));
      std::memcpy(prev_t, tt, sizeof(tt));
    }
    const long long used = lislam::FactorLaunches() - before;
    if (used != points - 1) {
      std::fprintf(stderr, "alternating buffers: %lld launches for %d points (%d new; want 1 each)\n", used, points,
                   points - 1);
      g_fail++;
    }
    std::printf("alternating parameter buffers: %lld launches for %d points (%d new)\n", used, points, points - 1);
  }
  // Two problems alive at once, each over its own parameter blocks at its own pose (two Ceres
  // problems, evaluated in turn): each problem's pass is one launch of ITS blocks, the other's
  // batch survives it, and the values equal a per-problem EvaluateBlocks.
  {
    std::vector<std::unique_ptr<lislam::CostFunction>> own[2];
    std::vector<const lislam::CostFunction*> lists[2];
    for (int p = 0; p < 2; p++)
      for (int i = 0; i < 600; i++) {
        lislam::CostFunction* f = i % 3 == 0 ? LidarEdgeFactor::Create(v3(), v3(), v3(), 1.0)
                                             : LidarPlaneFactor::Create(v3(), v3(), v3(), v3(), 1.0);
        own[p].emplace_back(f);
        lists[p].push_back(f);
      }
    double xq[2][4], xt[2][3];
    const long long before = lislam::FactorLaunches();
    const int rounds = 3;
    for (int round = 0; round < rounds; round++) {
      for (int p = 0; p < 2; p++) {
        xq[p][0] = A(rng); xq[p][1] = A(rng); xq[p][2] = A(rng);
        xq[p][3] = std::sqrt(1.0 - xq[p][0] * xq[p][0] - xq[p][1] * xq[p][1] - xq[p][2] * xq[p][2]);
        for (int k = 0; k < 3; k++) xt[p][k] = U(rng);
      }
      std::vector<double> ref[2];
      for (int p = 0; p < 2; p++) {
        ref[p].resize(lists[p].size() * 3);
        std::vector<double> jq(lists[p].size() * 12), jt(lists[p].size() * 9);
        if (lislam::EvaluateBlocks(lists[p], xq[p], xt[p], ref[p].data(), jq.data(), jt.data()) != LISLAM_OK) return 9;
      }
      for (int pass = 0; pass < 2; pass++)
        for (int p = 0; p < 2; p++) {
          const double* params[2] = {xq[p], xt[p]};
          for (size_t i = 0; i < lists[p].size(); i++) {
            double res[3];
            if (!lists[p][i]->Evaluate(params, res, nullptr)) return 10;
            for (int k = 0; k < lists[p][i]->num_residuals(); k++)
              check(res[k] == ref[p][i * 3 + k], "two-problem residual", (int)i, res[k], ref[p][i * 3 + k]);
          }
        }
    }
    const long long used = lislam::FactorLaunches() - before;  // (EvaluateBlocks is not counted)
    // the first pass of the first round: problem 0's launch holds every block not evaluated yet
    // (problem 1's too), problem 1's first call then launches its own; after that, one per point
    if (used > 2 * rounds) {
      std::fprintf(stderr, "two problems: %lld launches for %d rounds (want <= %d)\n", used, rounds, 2 * rounds);
      g_fail++;
    }
    std::printf("two live problems: %lld launches over %d rounds of 2 x 600 blocks\n", used, rounds);
  }
  // DISTORTION 1 (s != 1: Identity.slerp(s, q), s t; lidarFeaturePointsFunction.hpp:155-162,255-262):
  // kind 5 / 6 blocks, differentiated on the device with dual numbers, against the oracle's Jet
  // autodiff of the same functors and the header's operator()<double>; a quaternion near the
  // identity too (|w| >= 1 - eps: Eigen's linear branch) and one with w < 0.
  {
    const double qs[3][4] = {{q[0], q[1], q[2], q[3]}, {0.0, 0.0, 1e-9, 1.0}, {-q[0], -q[1], -q[2], -q[3]}};
    const double ss[3] = {0.0, 0.37, 0.85};
    int idx = 0;
    for (int iq = 0; iq < 3; iq++) {
      for (int is = 0; is < 3; is++) {
        for (int i = 0; i < 8; i++, idx++) {
          const bool edge = i & 1;
          lislam::Vector3d c = v3(), a = v3(), b = v3(), m = v3();
          const double s = ss[is];
          std::unique_ptr<lislam::CostFunction> f(edge ? LidarEdgeFactor::Create(c, a, b, s)
                                                       : LidarPlaneFactor::Create(c, a, b, m, s));
          if (!f) {
            std::fprintf(stderr, "Create with s = %g failed\n", s);
            return 6;
          }
          double res[3], jq[12], jt[9], host_r[3] = {0, 0, 0}, orr[3] = {0, 0, 0}, oJ[21] = {0};
          const double* params[2] = {qs[iq], t};
          double* jacs[2] = {jq, jt};
          if (!f->Evaluate(params, res, jacs)) {
            std::fprintf(stderr, "Evaluate (s = %g) failed: %s\n", s, lislam_last_error(ctx));
            return 6;
          }
          const int R = edge ? 3 : 1;
          if (edge) {
            LidarEdgeFactor(c, a, b, s)(qs[iq], t, host_r);
            oracle::EdgeFactor F{{c.x(), c.y(), c.z()}, {a.x(), a.y(), a.z()}, {b.x(), b.y(), b.z()}, s};
            oracle::autodiff_eval(F, qs[iq], t, orr, oJ);
          } else {
            LidarPlaneFactor(c, a, b, m, s)(qs[iq], t, host_r);
            const double cv[3] = {c.x(), c.y(), c.z()}, jv[3] = {a.x(), a.y(), a.z()}, lv[3] = {b.x(), b.y(), b.z()},
                         mv[3] = {m.x(), m.y(), m.z()};
            oracle::PlaneFactor F(cv, jv, lv, mv, s);
            oracle::autodiff_eval(F, qs[iq], t, orr, oJ);
          }
          for (int k = 0; k < R; k++) {
            check(close(res[k], orr[k], 1e-12, 1e-12), "distortion residual vs oracle", idx, res[k], orr[k]);
            check(close(res[k], host_r[k], 1e-12, 1e-12), "distortion residual vs header operator()", idx, res[k], host_r[k]);
            for (int cc = 0; cc < 4; cc++)
              check(close(jq[k * 4 + cc], oJ[k * 7 + cc], 1e-9, 1e-10), "distortion d r / d q vs oracle autodiff", idx,
                    jq[k * 4 + cc], oJ[k * 7 + cc]);
            for (int cc = 0; cc < 3; cc++)
              check(close(jt[k * 3 + cc], oJ[k * 7 + 4 + cc], 1e-9, 1e-10), "distortion d r / d t vs oracle autodiff",
                    idx, jt[k * 3 + cc], oJ[k * 7 + 4 + cc]);
          }
        }
      }
    }
    std::printf("distortion blocks ok (%d)\n", idx);
  }
  lislam_ctx_destroy(ctx);
  if (g_fail) {
    std::fprintf(stderr, "%d mismatches\n", g_fail);
    return 1;
  }
  std::printf("factors ok: %zu blocks (5 kinds x %d)\n", n, n_per);
  return 0;
}
