"""CPU pins of the scan-to-map oracle (oracle/oracle_map.cpp): exact k-NN against scipy's
cKDTree, Add_Points' box downsampling against a literal pure-Python transcription of
ikd_Tree.cpp:569-640, the plane / line fits against numpy least squares / eigh, and the solve
against the ground truth of a synthetic map.  No GPU."""
import math

import numpy as np
import pytest
from scipy.spatial import cKDTree


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def test_knn_matches_ckdtree(oracle):
    rng = np.random.default_rng(3)
    P = _f32(rng.uniform(-4, 4, (30000, 3)))
    m = oracle.IkdMap(0.4)
    m.build(P)
    Q = _f32(rng.uniform(-5, 5, (3000, 3)))
    for k in (1, 5, 8):
        pts, d2, found = m.knn(Q, k)
        dd, ii = cKDTree(P.astype(np.float64)).query(Q.astype(np.float64), k)
        ii = ii.reshape(len(Q), k)
        assert (found == k).all()
        assert np.array_equal(pts[:, :, 3].view(np.int32), ii)
        assert np.allclose(np.sqrt(d2), dd.reshape(len(Q), k), rtol=1e-5, atol=1e-6)


def test_knn_max_dist_and_small_map(oracle):
    m = oracle.IkdMap(0.2)
    P = _f32([[0, 0, 0], [1, 0, 0], [0, 2, 0]])
    m.build(P)
    pts, d2, found = m.knn(_f32([[0.1, 0, 0]]), 5)
    assert found[0] == 3 and np.all(np.isinf(d2[0, 3:]))
    pts, d2, found = m.knn(_f32([[0.1, 0, 0]]), 5, max_dist=1.0)
    assert found[0] == 2 and pts[0, 0, 3].view(np.int32) == 0 and pts[0, 1, 3].view(np.int32) == 1


def _ikd_add_points_python(stored, new, L):
    """Literal transcription of KD_TREE::Add_Points with downsample_on (ikd_Tree.cpp:594-640) over
    a list of (x, y, z, id); Search_by_range in ascending id."""
    pts = list(stored)
    for (x, y, z, i) in new:
        f = np.float32
        c = [f(x), f(y), f(z)]
        bmin = [f(np.floor(f(v) / f(L)) * f(L)) for v in c]
        bmax = [f(b + f(L)) for b in bmin]
        mid = [f(float(b) + float(f(hi - b)) / 2.0) for b, hi in zip(bmin, bmax)]

        def dist(p):
            return f(f(f(f(p[0] - mid[0]) * f(p[0] - mid[0])) + f(f(p[1] - mid[1]) * f(p[1] - mid[1]))) +
                     f(f(p[2] - mid[2]) * f(p[2] - mid[2])))

        S = sorted([p for p in pts if all(bmin[k] <= p[k] < bmax[k] for k in range(3))], key=lambda p: p[3])
        new_p = (c[0], c[1], c[2], i)
        min_d, res = dist(new_p), new_p
        for p in S:
            if dist(p) < min_d:
                min_d, res = dist(p), p
        same = all(abs(new_p[k] - res[k]) < 1e-6 for k in range(3))
        if len(S) > 1 or same:
            pts = [p for p in pts if p not in S]
            pts.append(res)
    return sorted(pts, key=lambda p: p[3])


def test_add_points_downsample_matches_literal_loop(oracle):
    rng = np.random.default_rng(5)
    L = 0.4
    base = _f32(rng.uniform(0, 2, (60, 3)))
    m = oracle.IkdMap(L)
    m.build(base)
    stored = [(float(p[0]), float(p[1]), float(p[2]), i) for i, p in enumerate(base)]
    next_id = len(base)
    for batch in range(3):
        new = _f32(rng.uniform(0, 2, (80, 3)))
        m.add_points(new, True)
        newl = [(float(p[0]), float(p[1]), float(p[2]), next_id + i) for i, p in enumerate(new)]
        next_id += len(new)
        stored = _ikd_add_points_python(stored, newl, L)
        got = m.points()
        ref = np.array([[p[0], p[1], p[2]] for p in stored], np.float32)
        ids = np.array([p[3] for p in stored], np.int32)
        assert np.array_equal(got[:, 3].view(np.int32), ids), batch
        assert np.array_equal(got[:, :3], ref), batch


def test_add_points_without_downsample_appends(oracle):
    m = oracle.IkdMap(0.4)
    m.build(_f32([[0, 0, 0]]))
    m.add_points(_f32([[0.01, 0, 0], [0.02, 0, 0]]), False)
    assert m.size() == 3


def test_plane_fit_matches_lstsq(oracle):
    rng = np.random.default_rng(11)
    m = oracle.IkdMap(0.2)
    # a tilted plane n.p + d = 0 sampled densely
    n = np.array([0.2, -0.3, 0.93])
    n /= np.linalg.norm(n)
    u = np.cross(n, [1, 0, 0]); u /= np.linalg.norm(u)
    v = np.cross(n, u)
    g = rng.uniform(-2, 2, (4000, 2))
    P = g[:, :1] * u + g[:, 1:] * v - 1.3 * n + rng.normal(0, 0.002, (4000, 1)) * n
    m.build(_f32(P))
    Q = _f32(rng.uniform(-1, 1, (200, 2)) @ np.stack([u, v]) - 1.3 * n)
    x = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    rec, kind = m.associate(1, Q, x)
    assert (kind == 2).mean() > 0.95
    pts, d2, found = m.knn(Q, 5)
    for i in np.nonzero(kind == 2)[0][:50]:
        A = pts[i, :, :3].astype(np.float64)
        sol = np.linalg.lstsq(A, -np.ones(5), rcond=None)[0]
        d = 1 / np.linalg.norm(sol)
        assert np.allclose(rec[i, 3:6], sol * d, atol=1e-9) and abs(rec[i, 6] - d) < 1e-9 * max(1, d)
        assert np.allclose(rec[i, :3], Q[i].astype(np.float64))


def test_line_fit_matches_eigh(oracle):
    rng = np.random.default_rng(12)
    m = oracle.IkdMap(0.4)
    d = np.array([0.1, 0.2, 0.97]); d /= np.linalg.norm(d)
    t = rng.uniform(-3, 3, 600)
    P = t[:, None] * d + rng.normal(0, 0.001, (600, 3)) + np.array([1.0, -2.0, 0.5])
    m.build(_f32(P))
    Q = _f32(rng.uniform(-2, 2, 100)[:, None] * d + np.array([1.0, -2.0, 0.5]) + rng.normal(0, 0.01, (100, 3)))
    x = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    rec, kind = m.associate(0, Q, x)
    assert (kind == 0).mean() > 0.9
    pts, d2, found = m.knn(Q, 5)
    for i in range(40):
        A = pts[i, :, :3].astype(np.float64)
        c = A.mean(0)
        w, V = np.linalg.eigh((A - c).T @ (A - c))
        assert (kind[i] == 0) == (w[2] > 3 * w[1] and d2[i, 4] < 1.0)
        if kind[i] != 0:
            continue
        a, b = rec[i, 3:6], rec[i, 6:9]
        assert np.allclose((a + b) / 2, c, atol=1e-12)
        dirv = (a - b) / np.linalg.norm(a - b)
        assert abs(abs(dirv @ V[:, 2]) - 1) < 1e-9


def test_map_solve_recovers_perturbed_pose(oracle, synth):
    M = synth.make_corridor_map(400_000, spacing=0.05)
    m = oracle.IkdMap(0.4)
    m.build(M)
    rng = np.random.default_rng(2)
    # queries: surface samples near x in [2, 12] seen from a sensor at (5, 0, 0), in the sensor frame
    sel = M[(M[:, 0] > 2) & (M[:, 0] < 12)]
    Q = sel[rng.choice(len(sel), 3000, replace=False)].copy()
    Q[:, 0] -= 5.0
    truth = np.array([0, 0, 0, 1, 5.0, 0, 0])
    x0 = synth.perturb_pose(truth[:4], truth[4:], 0.05, 0.5, seed=3)
    rec, kind = m.associate(1, Q, x0)
    x, summ = oracle.map_solve(rec, kind, x0, 10)
    assert summ[1] in (0, 1)
    assert np.linalg.norm(x[4:] - truth[4:]) < np.linalg.norm(x0[4:] - truth[4:])


def test_mapopt_corner_map_oracle(oracle, synth):
    """The corner ikd-Tree of mapOptimization (oracle): Build on the first keyframe with the
    corner cloud at the keyframe pose, Add_Points(downsample 0.8) afterwards; the ground stage is
    unchanged by it (same poses as mapopt_step)."""
    m1, m2, cm = oracle.IkdMap(0.4), oracle.IkdMap(0.4), oracle.IkdMap(0.8)
    s1 = s2 = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    sizes, total = [], 0
    for k in range(3):
        scan = synth.make_scan(20 + k, 16, 512)
        flat = scan.reshape(-1, 4)
        ground = np.ascontiguousarray(flat[np.abs(flat[:, :3]).sum(1) > 0], np.float32)
        corner = oracle.scan_registration(scan).less_sharp
        q, t = synth.ground_truth_pose(20 + k).as_qt()
        odom = synth.perturb_pose(q, t, 0.02, 0.2, seed=40 + k)
        p1, s1, u1 = oracle.mapopt_step(m1, ground, odom, s1)
        p2, s2, u2 = oracle.mapopt_step_corner(m2, cm, ground, corner, odom, s2)
        assert np.array_equal(p1, p2) and np.array_equal(u1, u2) and m1.size() == m2.size()
        if k == 0:  # Build keeps every point (no downsampling), transformed by the pose
            assert cm.size() == len(corner)
            pts = cm.points()
            qv, tv = p2[:4], p2[4:]
            R = _rot(qv)
            np.testing.assert_allclose(pts[:, :3], corner[:, :3].astype(np.float64) @ R.T + tv, atol=1e-4)
        total += len(corner)
        sizes.append(cm.size())
    # Add_Points(downsample) keeps one point per 0.8 m box among the map's points and the new
    # ones (ikd_Tree.cpp Add_Points): the map can shrink below the raw first keyframe
    assert 0 < sizes[1] < sizes[0] + total and 0 < sizes[2] <= total, sizes


def _rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
