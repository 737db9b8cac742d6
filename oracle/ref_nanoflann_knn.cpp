// TEST INFRASTRUCTURE ONLY — a driver around the reference's own vendored nanoflann (v1.3.2,
// /root/reference/include/nanoflann.hpp:62, through /root/reference/include/KDTreeVectorOfVectorsAdaptor.h),
// compiled from those headers where they lie by `make -C oracle ref` into oracle/_ref/.  It is the
// only reference code that compiles in this image, so it pins the exact-kNN
// restatement (oracle IkdMap::knn / nn1, and the GPU's k_knn) with the reference's own kd-tree:
// tests/golden/make_nanoflann_golden.py runs it once and commits the neighbour sets it returns.
//
// Usage: nanoflann_knn <in.bin> <out.bin>
//   in:  int32 n_target, n_query, k; float32 target[n_target][3]; float32 query[n_query][3]
//   out: int32 found[n_query]; int32 idx[n_query][k]; float32 dist_sq[n_query][k]  (ascending)
// float coordinates and float distances, as PCL's KdTreeFLANN<PointXYZI> and the ikd-Tree use them
// (laserOdometry.cpp:452,574; laserMapping.cpp:673,753; ikd_Tree.cpp:2224-2235).
#include <KDTreeVectorOfVectorsAdaptor.h>

#include <cstdint>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
    return 2;
  }
  std::FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 3;
  int32_t hdr[3];
  if (std::fread(hdr, 4, 3, f) != 3) return 4;
  const int nt = hdr[0], nq = hdr[1], k = hdr[2];
  if (nt < 1 || nq < 0 || k < 1) return 5;
  std::vector<float> t((size_t)nt * 3), q((size_t)nq * 3);
  if (std::fread(t.data(), 4, t.size(), f) != t.size() || std::fread(q.data(), 4, q.size(), f) != q.size()) return 6;
  std::fclose(f);

  typedef std::vector<std::vector<float>> cloud_t;
  cloud_t pts((size_t)nt, std::vector<float>(3));
  for (int i = 0; i < nt; i++)
    for (int d = 0; d < 3; d++) pts[i][d] = t[(size_t)i * 3 + d];
  // leaf size 10: the adaptor's default, as Scancontext.cpp builds it
  KDTreeVectorOfVectorsAdaptor<cloud_t, float, 3, nanoflann::metric_L2, size_t> tree(3, pts, 10);

  std::vector<int32_t> found((size_t)nq, 0), idx((size_t)nq * k, -1);
  std::vector<float> dist((size_t)nq * k, 0.f);
  std::vector<size_t> ri((size_t)k);
  std::vector<float> rd((size_t)k);
  for (int i = 0; i < nq; i++) {
    nanoflann::KNNResultSet<float, size_t> rs((size_t)k);
    rs.init(ri.data(), rd.data());
    tree.index->findNeighbors(rs, &q[(size_t)i * 3], nanoflann::SearchParams());
    const int n = (int)rs.size();
    found[i] = n;
    for (int j = 0; j < n; j++) {
      idx[(size_t)i * k + j] = (int32_t)ri[j];
      dist[(size_t)i * k + j] = rd[j];
    }
  }
  std::FILE* o = std::fopen(argv[2], "wb");
  if (!o) return 7;
  std::fwrite(found.data(), 4, found.size(), o);
  std::fwrite(idx.data(), 4, idx.size(), o);
  std::fwrite(dist.data(), 4, dist.size(), o);
  std::fclose(o);
  return 0;
}
