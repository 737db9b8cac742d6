// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// Restatement of the per-scan feature front end:
//   a1  ImageHandler::cloud_handler           src/image_handler.h_ouster:103-140
//   a2  removeClosedPointCloud                src/scanRegistration.cpp:152-186 (call :241)
//   a3  startOri/endOri, scanID, relTime      src/scanRegistration.cpp:247-374
//   a4  per-line concatenation                src/scanRegistration.cpp:384-394
//   a5  curvature                             src/scanRegistration.cpp:397-412
//   a6  segment sort + sharp/flat selection   src/scanRegistration.cpp:427-568
//   a7  less-flat + per-line VoxelGrid 0.2    src/scanRegistration.cpp:570-589
// with the repair interpretation of SURVEY.md §8(c)-1: the segment loop closes after :577,
// so the VoxelGrid runs once per scan line (A-LOAM structure).
//
// ties (bit mask) selects how equal sort keys are ordered:
//   bit 0 clear / set: the segment curvature sort (:445) as libstdc++'s std::sort leaves ties
//                      (the reference build) / by ascending point index;
//   bit 1 clear / set: the VoxelGrid's (voxel, point) sort (PCL std::sort by voxel) likewise.
// 0 is the reference throughout; the HIP path uses 1 (index order in the segment sorts, whose ties
// decide nothing on the benchmark data, tests/test_oracle.py; std::sort's order in the VoxelGrid,
// whose ties are structural).  The orders differ only when two keys compare equal.
#include <algorithm>
#include <cstring>
#include <vector>

#include "oracle_common.hpp"

namespace oracle {

// ---------------------------------------------------------------- a1
// image_handler.h_ouster:113-139.  image_ambient is all zero (:109) and not materialized.
static void cloud_handler(const P4* in, int H, int W, uint8_t* img_range, uint8_t* img_int,
                          P4* track) {
  for (int u = 0; u < H; u++) {
    for (int v = 0; v < W; v++) {
      const P4& pt = in[u * W + v];
      float range = std::sqrt(pt.x * pt.x + pt.y * pt.y + pt.z * pt.z);
      float intensity = std::min(pt.i, 255.0f);
      if (img_range) img_range[u * W + v] = (uint8_t)std::min(range * 20, 255.0f);
      if (img_int) img_int[u * W + v] = (uint8_t)intensity;
      if (track) {
        P4* p = &track[u * W + v];
        if ((double)range >= 0.1) {
          p->x = pt.x; p->y = pt.y; p->z = pt.z; p->i = intensity;
        } else {
          p->x = p->y = p->z = 0; p->i = 0;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- a3 helpers
// scanRegistration.cpp:290-331.  Returns -1 for points outside the line range (count--).
static int scan_id_of(float angle, int n_scans) {
  int id;
  if (n_scans == 16) {
    id = int((angle + 15) / 2 + 0.5);
  } else if (n_scans == 32) {
    id = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
  } else if (n_scans == 64) {
    id = int((angle + 22.5) * 1.41 + 0.5) - 1;
  } else {  // 128
    id = int((angle + 22.5) * 2.83 + 0.5) - 1;
  }
  if (id > n_scans - 1 || id < 0) return -1;
  return id;
}

// ---------------------------------------------------------------- a7 VoxelGrid
// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.10 as shipped with ROS noetic; third party,
// not vendored, parity unpinned): bounds, voxel index ijk·divb_mul, sort by index, one centroid
// of all four fields per voxel, output ordered by voxel index.
struct VoxIdx {
  unsigned idx;
  unsigned cloud_point_index;
  bool operator<(const VoxIdx& o) const { return idx < o.idx; }
};

static void voxel_grid(const std::vector<P4>& in, float leaf, bool canonical, std::vector<P4>& out) {
  if (in.empty()) return;
  const float inv = 1.0f / leaf;
  float minp[3] = {in[0].x, in[0].y, in[0].z}, maxp[3] = {in[0].x, in[0].y, in[0].z};
  for (const P4& p : in) {
    minp[0] = std::min(minp[0], p.x); minp[1] = std::min(minp[1], p.y); minp[2] = std::min(minp[2], p.z);
    maxp[0] = std::max(maxp[0], p.x); maxp[1] = std::max(maxp[1], p.y); maxp[2] = std::max(maxp[2], p.z);
  }
  int64_t dx = (int64_t)((maxp[0] - minp[0]) * inv) + 1;
  int64_t dy = (int64_t)((maxp[1] - minp[1]) * inv) + 1;
  int64_t dz = (int64_t)((maxp[2] - minp[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)INT32_MAX) {  // PCL: leaf too small -> output = input
    out.insert(out.end(), in.begin(), in.end());
    return;
  }
  int min_b[3], max_b[3], div_b[3];
  for (int k = 0; k < 3; k++) {
    min_b[k] = (int)std::floor(minp[k] * inv);
    max_b[k] = (int)std::floor(maxp[k] * inv);
    div_b[k] = max_b[k] - min_b[k] + 1;
  }
  const int mul1 = div_b[0], mul2 = div_b[0] * div_b[1];
  std::vector<VoxIdx> iv(in.size());
  for (size_t n = 0; n < in.size(); n++) {
    int i0 = (int)(std::floor(in[n].x * inv) - (float)min_b[0]);
    int i1 = (int)(std::floor(in[n].y * inv) - (float)min_b[1]);
    int i2 = (int)(std::floor(in[n].z * inv) - (float)min_b[2]);
    iv[n].idx = (unsigned)(i0 + i1 * mul1 + i2 * mul2);
    iv[n].cloud_point_index = (unsigned)n;
  }
  if (canonical)
    std::stable_sort(iv.begin(), iv.end());
  else
    std::sort(iv.begin(), iv.end());
  size_t a = 0;
  while (a < iv.size()) {
    size_t b = a + 1;
    while (b < iv.size() && iv[b].idx == iv[a].idx) ++b;
    P4 c = in[iv[a].cloud_point_index];
    for (size_t l = a + 1; l < b; l++) {
      const P4& p = in[iv[l].cloud_point_index];
      c.x += p.x; c.y += p.y; c.z += p.z; c.i += p.i;
    }
    const float n = (float)(b - a);
    c.x /= n; c.y /= n; c.z /= n; c.i /= n;
    out.push_back(c);
    a = b;
  }
}

struct ScanRegOut {
  std::vector<P4> cloud;  // laserCloud (/velodyne_cloud_2)
  std::vector<int> start, end;
  std::vector<float> curv;
  std::vector<int8_t> label;
  std::vector<P4> sharp, less_sharp, flat, less_flat;
};

// scanRegistration.cpp:189-589 for one organized scan (points in ring-major order).
static void scan_registration(const P4* raw, int npts, int n_scans, float min_range, int ties,
                              ScanRegOut& o) {
  // a2: removeClosedPointCloud(laserCloudIn, laserCloudIn, MINIMUM_RANGE) — thres is a float.
  const float thres = min_range;
  std::vector<P4> in;
  in.reserve(npts);
  for (int i = 0; i < npts; i++) {
    const P4& p = raw[i];
    if (p.x * p.x + p.y * p.y + p.z * p.z < thres * thres) continue;
    in.push_back(p);
  }
  const int cloudSize = (int)in.size();
  o.start.assign(n_scans, 0);
  o.end.assign(n_scans, 0);
  if (cloudSize == 0) {  // the reference reads points[0] of an empty cloud (UB); we emit nothing
    for (int i = 0; i < n_scans; i++) { o.start[i] = 5; o.end[i] = -6; }
    return;
  }
  // a3
  float startOri = -atan2_f(in[0].y, in[0].x);
  float endOri = (float)((double)(-atan2_f(in[cloudSize - 1].y, in[cloudSize - 1].x)) + 2 * M_PI);
  if ((double)(endOri - startOri) > 3 * M_PI)
    endOri = (float)((double)endOri - 2 * M_PI);
  else if ((double)(endOri - startOri) < M_PI)
    endOri = (float)((double)endOri + 2 * M_PI);

  bool halfPassed = false;
  std::vector<std::vector<P4>> scans(n_scans);
  for (int i = 0; i < cloudSize; i++) {
    P4 point = in[i];
    float angle = (float)((double)(atan_f(point.z / std::sqrt(point.x * point.x + point.y * point.y)) * 180) / M_PI);
    int scanID = scan_id_of(angle, n_scans);
    if (scanID < 0) continue;
    float ori = -atan2_f(point.y, point.x);
    if (!halfPassed) {
      if ((double)ori < (double)startOri - M_PI / 2)
        ori = (float)((double)ori + 2 * M_PI);
      else if ((double)ori > (double)startOri + M_PI * 3 / 2)
        ori = (float)((double)ori - 2 * M_PI);
      if ((double)(ori - startOri) > M_PI) halfPassed = true;
    } else {
      ori = (float)((double)ori + 2 * M_PI);
      if ((double)ori < (double)endOri - M_PI * 3 / 2)
        ori = (float)((double)ori + 2 * M_PI);
      else if ((double)ori > (double)endOri + M_PI / 2)
        ori = (float)((double)ori - 2 * M_PI);
    }
    float relTime = (ori - startOri) / (endOri - startOri);
    point.i = (float)(scanID + 0.1 * relTime);
    scans[scanID].push_back(point);
  }
  // a4
  std::vector<P4>& cloud = o.cloud;
  cloud.clear();
  for (int i = 0; i < n_scans; i++) {
    o.start[i] = (int)cloud.size() + 5;
    cloud.insert(cloud.end(), scans[i].begin(), scans[i].end());
    o.end[i] = (int)cloud.size() - 6;
  }
  const int N = (int)cloud.size();
  // a5
  std::vector<float>& curv = o.curv;
  curv.assign(N, 0.f);
  std::vector<int> sortInd(N), picked(N, 0);
  std::vector<int8_t>& label = o.label;
  label.assign(N, 0);
  for (int i = 0; i < N; i++) sortInd[i] = i;
  for (int i = 5; i < N - 5; i++) {
    const P4* p = cloud.data();
    float dX = p[i - 5].x + p[i - 4].x + p[i - 3].x + p[i - 2].x + p[i - 1].x - 10 * p[i].x + p[i + 1].x + p[i + 2].x + p[i + 3].x + p[i + 4].x + p[i + 5].x;
    float dY = p[i - 5].y + p[i - 4].y + p[i - 3].y + p[i - 2].y + p[i - 1].y - 10 * p[i].y + p[i + 1].y + p[i + 2].y + p[i + 3].y + p[i + 4].y + p[i + 5].y;
    float dZ = p[i - 5].z + p[i - 4].z + p[i - 3].z + p[i - 2].z + p[i - 1].z - 10 * p[i].z + p[i + 1].z + p[i + 2].z + p[i + 3].z + p[i + 4].z + p[i + 5].z;
    curv[i] = dX * dX + dY * dY + dZ * dZ;
  }
  // neighbour suppression (:481-504 / :539-566)
  auto suppress = [&](int ind) {
    for (int l = 1; l <= 5; l++) {
      float dx = cloud[ind + l].x - cloud[ind + l - 1].x;
      float dy = cloud[ind + l].y - cloud[ind + l - 1].y;
      float dz = cloud[ind + l].z - cloud[ind + l - 1].z;
      if ((double)(dx * dx + dy * dy + dz * dz) > 0.05) break;
      picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
      float dx = cloud[ind + l].x - cloud[ind + l + 1].x;
      float dy = cloud[ind + l].y - cloud[ind + l + 1].y;
      float dz = cloud[ind + l].z - cloud[ind + l + 1].z;
      if ((double)(dx * dx + dy * dy + dz * dz) > 0.05) break;
      picked[ind + l] = 1;
    }
  };
  // a6/a7
  for (int i = 0; i < n_scans; i++) {
    const int s = o.start[i], e = o.end[i];
    if (e - s < 6) continue;
    std::vector<P4> lessFlatScan;
    for (int j = 0; j < 6; j++) {
      int sp = s + (e - s) * j / 6;
      int ep = s + (e - s) * (j + 1) / 6 - 1;
      if (ties & 1)
        std::stable_sort(sortInd.begin() + sp, sortInd.begin() + ep + 1,
                         [&](int a, int b) { return curv[a] < curv[b]; });
      else
        std::sort(sortInd.begin() + sp, sortInd.begin() + ep + 1,
                  [&](int a, int b) { return curv[a] < curv[b]; });
      int largestPickedNum = 0;
      for (int k = ep; k >= sp; k--) {
        int ind = sortInd[k];
        if (picked[ind] == 0 && (double)curv[ind] > 0.1) {
          largestPickedNum++;
          if (largestPickedNum <= 2) {
            label[ind] = 2;
            o.sharp.push_back(cloud[ind]);
            o.less_sharp.push_back(cloud[ind]);
          } else if (largestPickedNum <= 20) {
            label[ind] = 1;
            o.less_sharp.push_back(cloud[ind]);
          } else {
            break;
          }
          picked[ind] = 1;
          suppress(ind);
        }
      }
      int smallestPickedNum = 0;
      for (int k = sp; k <= ep; k++) {
        int ind = sortInd[k];
        if (picked[ind] == 0 && (double)curv[ind] < 0.1) {
          label[ind] = -1;
          o.flat.push_back(cloud[ind]);
          smallestPickedNum++;
          if (smallestPickedNum >= 4) break;
          picked[ind] = 1;
          suppress(ind);
        }
      }
      for (int k = sp; k <= ep; k++)
        if (label[k] <= 0) lessFlatScan.push_back(cloud[k]);
    }
    voxel_grid(lessFlatScan, 0.2f, (ties & 2) != 0, o.less_flat);
  }
}

}  // namespace oracle

using namespace oracle;

extern "C" {

// One scan through a1..a7.  Output buffers are caller-owned; capacities are H*W for the
// per-point arrays, 12*n_scans / 120*n_scans / 24*n_scans for sharp / less_sharp / flat and
// H*W for less_flat.  Any output pointer may be NULL.  Returns 0.
int oracle_scan_registration(const float* xyzi, int H, int W, int n_scans, float min_range,
                             int ties, uint8_t* img_range, uint8_t* img_int, float* cloud_track,
                             float* laser_cloud, int* n_cloud, int* scan_start, int* scan_end,
                             float* curvature, int8_t* label, float* sharp, int* n_sharp,
                             float* less_sharp, int* n_less_sharp, float* flat, int* n_flat,
                             float* less_flat, int* n_less_flat) {
  const P4* raw = reinterpret_cast<const P4*>(xyzi);
  cloud_handler(raw, H, W, img_range, img_int, reinterpret_cast<P4*>(cloud_track));
  ScanRegOut o;
  scan_registration(raw, H * W, n_scans, min_range, ties, o);
  auto put = [](const std::vector<P4>& v, float* dst, int* n) {
    if (n) *n = (int)v.size();
    if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(P4));
  };
  put(o.cloud, laser_cloud, n_cloud);
  if (scan_start) std::memcpy(scan_start, o.start.data(), n_scans * sizeof(int));
  if (scan_end) std::memcpy(scan_end, o.end.data(), n_scans * sizeof(int));
  if (curvature && !o.curv.empty()) std::memcpy(curvature, o.curv.data(), o.curv.size() * sizeof(float));
  if (label && !o.label.empty()) std::memcpy(label, o.label.data(), o.label.size());
  put(o.sharp, sharp, n_sharp);
  put(o.less_sharp, less_sharp, n_less_sharp);
  put(o.flat, flat, n_flat);
  put(o.less_flat, less_flat, n_less_flat);
  return 0;
}

// Standalone PCL-semantics VoxelGrid (for the unit tests of a7).
int oracle_voxel_grid(const float* xyzi, int n, float leaf, int canonical, float* out, int* n_out) {
  std::vector<P4> in(reinterpret_cast<const P4*>(xyzi), reinterpret_cast<const P4*>(xyzi) + n);
  std::vector<P4> o;
  voxel_grid(in, leaf, canonical != 0, o);
  *n_out = (int)o.size();
  if (out && !o.empty()) std::memcpy(out, o.data(), o.size() * sizeof(P4));
  return 0;
}

}  // extern "C"
