// The order in which libstdc++'s std::sort leaves equal keys, computed the way the HIP kernels
// compute it (lislam_device.hpp introsort_order): every partition step of std::__introsort_loop is
// evaluated with prefix counts instead of the two-pointer walk, the heap-sort fallback runs
// serially, and the final insertion sort — stable for equal keys — becomes a stable sort by key.
// The device finishes with a window rank instead of the insertion sort (final_positions in
// lislam_features.hip): an element's final position is its position after the loop, minus the
// greater keys among the 15 before it, plus the smaller keys among the 15 after it.
// This file checks that formulation against std::sort itself on many arrays with heavy ties (the
// situation of PCL VoxelGrid's std::sort of (voxel, point) pairs by voxel,
// scanRegistration.cpp:574-578), and on scan-line segments sorted by curvature the way
// scanRegistration.cpp:445 sorts them (std::sort of point indices with comp(i, j) =
// curvature[i] < curvature[j], float curvatures with many equal values; the device keys are the
// floats' bits, which order non-negative floats alike).  Prints "introsort ok" and exits 0.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

struct E {
  uint32_t key;
  uint32_t id;
  bool operator<(const E& o) const { return key < o.key; }  // VoxelGrid: compares the voxel only
};

// --- the emulation (mirrors the device code step for step) ---------------------------------
static void move_median_to_first(std::vector<E>& a, int result, int x, int y, int z) {
  auto lt = [&](int i, int j) { return a[i].key < a[j].key; };
  int pick;
  if (lt(x, y)) {
    if (lt(y, z)) pick = y;
    else if (lt(x, z)) pick = z;
    else pick = x;
  } else if (lt(x, z)) {
    pick = x;
  } else if (lt(y, z)) {
    pick = z;
  } else {
    pick = y;
  }
  std::swap(a[result], a[pick]);
}

// std::__unguarded_partition(first + 1, last, first) by prefix counts: the m-th element >= pivot
// from the left (L[m]) swaps with the m-th element <= pivot from the right (R[m]) while
// L[m] < R[m]; the cut is where the left walk stops after the last swap.
static int partition_by_counts(std::vector<E>& a, int f, int l) {
  const int mid = f + (l - f) / 2;
  move_median_to_first(a, f, f + 1, mid, l - 1);
  const uint32_t p = a[f].key;
  const int lo = f + 1, hi = l - 1;
  int total_le = 0;
  for (int i = lo; i <= hi; i++) total_le += !(p < a[i].key);
  std::vector<int> R(total_le);
  int ge_before = 0, le_seen = 0, mstar = 0, next_ge = -1;
  for (int i = lo; i <= hi; i++) {
    const bool ge = !(a[i].key < p), le = !(p < a[i].key);
    if (le) {
      le_seen++;
      R[total_le - le_seen] = i;  // right rank: number of <= elements after i
    }
    if (ge) {
      const int after = total_le - le_seen;  // <= elements strictly after i
      if (after >= ge_before + 1) mstar++;
      else if (next_ge < 0 && ge_before == mstar) next_ge = i;
      ge_before++;
    }
  }
  // L[mstar] (next_ge) is the first >= element whose rank is not matched
  int cut = mstar > 0 ? R[mstar - 1] : l;
  if (next_ge >= 0 && next_ge < cut) cut = next_ge;
  std::vector<int> L;
  for (int i = lo; i <= hi && (int)L.size() < mstar; i++)
    if (!(a[i].key < p)) L.push_back(i);
  for (int m = 0; m < mstar; m++) std::swap(a[L[m]], a[R[m]]);
  return cut;
}

static void adjust_heap(E* first, long hole, long len, E value) {
  const long top = hole;
  long child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (first[child].key < first[child - 1].key) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  long parent = (hole - 1) / 2;
  while (hole > top && first[parent].key < value.key) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

static void heap_sort(E* first, long len) {
  if (len >= 2)
    for (long parent = (len - 2) / 2;; parent--) {
      adjust_heap(first, parent, len, first[parent]);
      if (parent == 0) break;
    }
  for (long last = len; last > 1;) {
    --last;
    E v = first[last];
    first[last] = first[0];
    adjust_heap(first, 0, last, v);
  }
}

// The introsort loop only (blocks of at most 16 elements left for the final insertion sort).
static std::vector<E> introsort_loop(std::vector<E> a) {
  const int n = (int)a.size();
  if (n == 0) return a;
  int lg = 0;
  while ((2 << lg) <= n) lg++;
  struct Range { int f, l, d; };
  std::vector<Range> stack{{0, n, 2 * lg}};
  while (!stack.empty()) {
    Range r = stack.back();
    stack.pop_back();
    while (r.l - r.f > 16) {
      if (r.d == 0) {
        heap_sort(a.data() + r.f, r.l - r.f);
        break;
      }
      r.d--;
      const int cut = partition_by_counts(a, r.f, r.l);
      stack.push_back({cut, r.l, r.d});
      r.l = cut;
    }
  }
  return a;
}

static std::vector<E> emulate(std::vector<E> a) {
  a = introsort_loop(a);
  std::stable_sort(a.begin(), a.end());  // the final insertion sort never reorders equal keys
  return a;
}

// The device's finish: every element's final position from a +-15 window rank.
static std::vector<E> window_rank(const std::vector<E>& a) {
  const int n = (int)a.size();
  std::vector<E> out(n);
  for (int j = 0; j < n; j++) {
    int mv = 0;
    for (int d = 1; d <= 15; d++) {
      if (j - d >= 0 && a[j - d].key > a[j].key) mv--;
      if (j + d < n && a[j + d].key < a[j].key) mv++;
    }
    out[j + mv] = a[j];
  }
  return out;
}

static bool same_order(const std::vector<E>& got, const std::vector<E>& ref) {
  for (size_t i = 0; i < ref.size(); i++)
    if (got[i].id != ref[i].id || got[i].key != ref[i].key) return false;
  return true;
}

static uint32_t fbits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

int main() {
  std::mt19937 rng(1);
  int cases = 0, bad = 0;
  for (int n = 0; n <= 1100; n += (n < 80 ? 1 : 7)) {
    for (int mode = 0; mode < 6; mode++) {
      std::vector<E> a(n);
      for (int i = 0; i < n; i++) {
        uint32_t k;
        switch (mode) {
          case 0: k = rng() % 4; break;                          // few distinct keys
          case 1: k = rng() % (n / 3 + 1); break;                // voxel-like runs
          case 2: k = (uint32_t)(i / 3) + rng() % 3; break;      // nearly sorted (a scan line)
          case 3: k = (uint32_t)((n - i) / 2); break;            // descending runs
          case 4: k = 7; break;                                   // all equal
          default: k = rng(); break;                              // distinct
        }
        a[i] = E{k, (uint32_t)i};
      }
      std::vector<E> ref = a;
      std::sort(ref.begin(), ref.end());
      const std::vector<E> got = emulate(a);
      const std::vector<E> win = window_rank(introsort_loop(a));
      cases++;
      if (!same_order(got, ref) || !same_order(win, ref)) {
        if (bad < 10) std::fprintf(stderr, "n=%d mode=%d differs\n", n, mode);
        bad++;
      }
    }
  }
  // scan-line segments (scanRegistration.cpp:440-445): indices sp..ep sorted by float curvature,
  // curvatures with ties (snapped / duplicated points give exactly equal sums)
  for (int n = 1; n <= 400; n += (n < 40 ? 1 : 3)) {
    for (int mode = 0; mode < 4; mode++) {
      std::vector<float> curv(n);
      for (int i = 0; i < n; i++) {
        switch (mode) {
          case 0: curv[i] = 0.01f * (float)(rng() % 5); break;              // a few values, 0 included
          case 1: curv[i] = (rng() % 3 == 0) ? 0.f : (float)(rng() % 1000) * 1e-3f; break;  // many zeros
          case 2: curv[i] = (float)((i / 4) % 7) * 0.125f; break;             // duplicated runs
          default: curv[i] = std::ldexp((float)(rng() % 64), -(int)(rng() % 8)); break;
        }
      }
      const int sp = 5;
      std::vector<int> ind(sp + n);
      for (int i = 0; i < sp + n; i++) ind[i] = i;
      std::vector<float> curv_full(sp + n, 0.f);
      for (int i = 0; i < n; i++) curv_full[sp + i] = curv[i];
      std::sort(ind.begin() + sp, ind.end(), [&](int i, int j) { return curv_full[i] < curv_full[j]; });
      std::vector<E> a(n);
      for (int i = 0; i < n; i++) a[i] = E{fbits(curv[i]), (uint32_t)i};
      const std::vector<E> win = window_rank(introsort_loop(a));
      cases++;
      for (int i = 0; i < n; i++)
        if ((int)win[i].id + sp != ind[sp + i]) {
          if (bad < 10) std::fprintf(stderr, "segment n=%d mode=%d differs at %d\n", n, mode, i);
          bad++;
          break;
        }
    }
  }
  // inputs that drive std::sort into its heap-sort fallback (median-of-3 killer for this pivot rule)
  for (int n : {64, 200, 513, 1024}) {
    std::vector<E> a(n);
    for (int i = 0; i < n; i++) a[i] = E{(uint32_t)(i % 2 == 0 ? i : n - i), (uint32_t)i};
    std::vector<E> ref = a;
    std::sort(ref.begin(), ref.end());
    const std::vector<E> got = emulate(a);
    const std::vector<E> win = window_rank(introsort_loop(a));
    cases++;
    if (!same_order(got, ref) || !same_order(win, ref)) { bad++; std::fprintf(stderr, "killer n=%d differs\n", n); }
  }
  if (bad) {
    std::fprintf(stderr, "%d of %d cases differ\n", bad, cases);
    return 1;
  }
  std::printf("introsort ok: %d cases\n", cases);
  return 0;
}
