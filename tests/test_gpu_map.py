"""GPU parity of the scan-to-map path (a19-a21) through the C ABI against the CPU oracle.

k-NN results (point ids, squared distances), Add_Points' surviving point sets and the VoxelGrid
are integer / index / float-copy work and must be bit-exact; residual-block records are fp64
fits written with the same operation order on both sides (compared bit-exact, with a 1e-12
relative fallback reported); poses within the north-star tolerance 1e-4 m / 1e-4 rad.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4  # BASELINE.json north_star


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(n_scans=64, width=1024)
    yield c
    c.close()


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def _by_id(p):
    ids = p[:, 3].view(np.int32)
    o = np.argsort(ids, kind="stable")
    return p[o]


def _knn_equal(g, r, k):
    gp, gd, gf = g
    rp, rd, rf = r
    assert np.array_equal(gf, rf)
    for i in range(len(gf)):
        f = gf[i]
        assert np.array_equal(gp[i, :f], rp[i, :f]), i
        assert np.array_equal(gd[i, :f], rd[i, :f]), i


@pytest.mark.parametrize("cell", [0.0, 0.1, 1.0])
def test_knn_random_bit_exact(pkg, oracle, ctx, cell):
    rng = np.random.default_rng(21)
    P = _f32(rng.uniform(-6, 6, (50000, 3)))
    Q = _f32(rng.uniform(-8, 8, (4000, 3)))  # includes queries outside the map's box
    g = pkg.mapping.IkdMap(ctx, 0.4, cell)
    g.build(P)
    o = oracle.IkdMap(0.4)
    o.build(P)
    for k in (1, 5, 8):
        _knn_equal(g.nearest_search(Q, k), o.knn(Q, k), k)
    for md in (0.05, 0.3, 1.0):
        _knn_equal(g.nearest_search(Q, 5, md), o.knn(Q, 5, md), 5)
    g.close()


def test_knn_corridor_and_far_queries(pkg, oracle, ctx, synth):
    M = synth.make_corridor_map(300_000, spacing=0.05)
    g = pkg.mapping.IkdMap(ctx, 0.4, 0.1)
    g.build(M)
    o = oracle.IkdMap(0.4)
    o.build(M)
    rng = np.random.default_rng(4)
    Q = M[rng.choice(len(M), 3000, replace=False), :3] + rng.normal(0, 0.03, (3000, 3))
    far = _f32(np.array([[500.0, 30.0, 9.0], [-50.0, 0.0, 0.0], [2.0, 0.0, 40.0]]))  # full-scan fallback
    Q = _f32(np.concatenate([Q, far]))
    _knn_equal(g.nearest_search(Q, 5), o.knn(Q, 5), 5)
    g.close()


@pytest.mark.parametrize("cell", [0.0, 0.1, 1.0])
def test_knn_16_lane_groups_bit_exact(pkg, oracle, ctx, synth, monkeypatch, cell):
    """Four queries per wave (LISLAM_KNN_LANES=16: one 16-lane row per query, every group-wide step
    a row op, groups leaving the shell loop at different shells) against the oracle: random map and
    queries (some outside the map's box), k 1 / 5 / 8, max distances, and the corridor map with
    far queries that take the whole-map scan."""
    monkeypatch.setenv("LISLAM_KNN_LANES", "16")
    rng = np.random.default_rng(21)
    P = _f32(rng.uniform(-6, 6, (50000, 3)))
    Q = _f32(rng.uniform(-8, 8, (4000, 3)))
    g = pkg.mapping.IkdMap(ctx, 0.4, cell)
    g.build(P)
    o = oracle.IkdMap(0.4)
    o.build(P)
    for k in (1, 5, 8):
        _knn_equal(g.nearest_search(Q, k), o.knn(Q, k), k)
    for md in (0.05, 0.3, 1.0):
        _knn_equal(g.nearest_search(Q, 5, md), o.knn(Q, 5, md), 5)
    g.close()
    M = synth.make_corridor_map(300_000, spacing=0.05)
    g = pkg.mapping.IkdMap(ctx, 0.4, 0.1)
    g.build(M)
    o = oracle.IkdMap(0.4)
    o.build(M)
    Q = M[rng.choice(len(M), 3001, replace=False), :3] + rng.normal(0, 0.03, (3001, 3))
    far = _f32(np.array([[500.0, 30.0, 9.0], [-50.0, 0.0, 0.0], [2.0, 0.0, 40.0]]))
    Q = _f32(np.concatenate([Q, far]))  # 3004 queries: the last workgroup is partly empty
    _knn_equal(g.nearest_search(Q, 5), o.knn(Q, 5), 5)
    g.close()


@pytest.mark.parametrize("lanes", ["16", "64"])
@pytest.mark.parametrize("near", ["-1", "0", "0.02", "0.1", "0.3", "2"])
@pytest.mark.parametrize("cell", [0.1, 0.3])
def test_knn_near_first_pass(pkg, oracle, ctx, synth, monkeypatch, near, cell, lanes):
    """The 3x3x3 block's near-cells-first split (LISLAM_KNN_NEAR, metres; -1: one pass) returns the
    same k-best as the oracle's k-d tree for every radius, including radii that cover no cell but
    the query's own (0), part of the block (0.02 .. 0.3) and all of it (2), with and without a
    max distance, with 64 and 16 lanes per query."""
    monkeypatch.setenv("LISLAM_KNN_NEAR", near)
    monkeypatch.setenv("LISLAM_KNN_LANES", lanes)
    M = synth.make_corridor_map(200_000, spacing=0.05)
    g = pkg.mapping.IkdMap(ctx, 0.4, cell)
    g.build(M)
    o = oracle.IkdMap(0.4)
    o.build(M)
    rng = np.random.default_rng(11)
    Q = _f32(M[rng.choice(len(M), 2000, replace=False), :3] + rng.normal(0, 0.08, (2000, 3)))
    _knn_equal(g.nearest_search(Q, 5), o.knn(Q, 5), 5)
    _knn_equal(g.nearest_search(Q, 8), o.knn(Q, 8), 8)
    _knn_equal(g.nearest_search(Q, 5, 0.01), o.knn(Q, 5, 0.01), 5)
    g.close()


def test_knn_small_and_empty_maps(pkg, oracle, ctx):
    g = pkg.mapping.IkdMap(ctx, 0.2)
    Q = _f32([[0.1, 0, 0], [5, 5, 5]])
    pts, d2, found = g.nearest_search(Q, 5)
    assert (found == 0).all() and np.isinf(d2).all()
    P = _f32([[0, 0, 0], [1, 0, 0], [0, 2, 0]])
    g.build(P)
    o = oracle.IkdMap(0.2)
    o.build(P)
    _knn_equal(g.nearest_search(Q, 5), o.knn(Q, 5), 5)
    _knn_equal(g.nearest_search(Q, 5, 1.0), o.knn(Q, 5, 1.0), 5)
    g.close()


@pytest.mark.parametrize("L,cell", [(0.4, 0.0), (0.4, 0.1), (0.8, 0.3)])
def test_add_points_downsample_bit_exact(pkg, oracle, ctx, L, cell):
    rng = np.random.default_rng(8)
    base = _f32(rng.uniform(0, 6, (20000, 3)))
    g = pkg.mapping.IkdMap(ctx, L, cell)
    o = oracle.IkdMap(L)
    g.build(base)
    o.build(base)
    for batch in range(4):
        new = _f32(rng.uniform(-1, 7, (6000, 3)))
        g.add_points(new, True)
        o.add_points(new, True)
        gp, op = _by_id(g.points()), o.points()
        assert g.size() == o.size() == len(op)
        assert np.array_equal(gp, op), batch
    g.close()


def test_add_points_no_downsample_and_empty_start(pkg, oracle, ctx):
    rng = np.random.default_rng(9)
    g = pkg.mapping.IkdMap(ctx, 0.4)
    o = oracle.IkdMap(0.4)
    a = _f32(rng.uniform(0, 3, (3000, 3)))
    g.add_points(a, True)  # downsampled insert into an empty map
    o.add_points(a, True)
    assert np.array_equal(_by_id(g.points()), o.points())
    b = _f32(rng.uniform(0, 3, (1000, 3)))
    g.add_points(b, False)
    o.add_points(b, False)
    assert np.array_equal(_by_id(g.points()), o.points())
    Q = _f32(rng.uniform(0, 3, (500, 3)))
    _knn_equal(g.nearest_search(Q, 5), o.knn(Q, 5), 5)
    g.close()


@pytest.mark.parametrize("leaf", [0.2, 0.8])
def test_voxel_grid_bit_exact(pkg, oracle, ctx, synth, leaf):
    scan = synth.make_scan(3)
    pts = _f32(scan.reshape(-1, 4))
    pts = pts[np.abs(pts[:, :3]).sum(1) > 0]
    g = pkg.mapping.voxel_grid(ctx, pts, leaf)
    r = oracle.voxel_grid(pts, leaf, canonical=True)
    assert np.array_equal(g, r)


def _records_equal(ga, ra):
    grec, gk = ga
    rrec, rk = ra
    assert np.array_equal(gk, rk)
    v = gk >= 0
    if not np.array_equal(grec[v], rrec[v]):
        assert np.allclose(grec[v], rrec[v], rtol=1e-12, atol=1e-12)


def test_associate_plane_and_line(pkg, oracle, ctx, synth):
    M = synth.make_corridor_map(300_000, spacing=0.05)
    E = synth.make_edge_map(40)
    rng = np.random.default_rng(6)
    truth = np.array([0, 0, 0, 1, 5.0, 0.1, 0.0])
    x0 = synth.perturb_pose(truth[:4], truth[4:], 0.05, 0.5, seed=2)
    gs, os_ = pkg.mapping.IkdMap(ctx, 0.4, 0.1), oracle.IkdMap(0.4)
    gs.build(M)
    os_.build(M)
    Qs = M[rng.choice(len(M), 4000, replace=False)].copy()
    Qs[:, :3] -= truth[4:7].astype(np.float32)
    _records_equal(gs.associate(1, Qs, x0), os_.associate(1, Qs, x0))
    gc, oc = pkg.mapping.IkdMap(ctx, 0.8, 0.2), oracle.IkdMap(0.8)
    gc.build(E)
    oc.build(E)
    Qc = E[rng.choice(len(E), 600, replace=False)].copy()
    Qc[:, :3] += rng.normal(0, 0.02, (600, 3)).astype(np.float32) - truth[4:7].astype(np.float32)
    _records_equal(gc.associate(0, Qc, x0), oc.associate(0, Qc, x0))
    gs.close()
    gc.close()


def test_normal_equations_and_solve(pkg, oracle, ctx, synth):
    M = synth.make_corridor_map(300_000, spacing=0.05)
    E = synth.make_edge_map(40)
    rng = np.random.default_rng(7)
    truth = np.array([0, 0, 0, 1, 5.0, 0.1, 0.0])
    x0 = synth.perturb_pose(truth[:4], truth[4:], 0.05, 0.5, seed=4)
    os_, oc = oracle.IkdMap(0.4), oracle.IkdMap(0.8)
    os_.build(M)
    oc.build(E)
    Qs = M[rng.choice(len(M), 3000, replace=False)].copy()
    Qs[:, :3] -= truth[4:7].astype(np.float32)
    Qc = E[rng.choice(len(E), 500, replace=False)].copy()
    Qc[:, :3] -= truth[4:7].astype(np.float32)
    rs, ks = os_.associate(1, Qs, x0)
    rc, kc = oc.associate(0, Qc, x0)
    rec = np.concatenate([rc, rs])
    kind = np.concatenate([kc, ks])
    # normal equations vs the oracle's autodiff functors (same Huber corrector)
    ne = pkg.mapping.normal_equations(ctx, rec, kind, x0)
    acc = np.zeros(28)
    for r9, kd in zip(rec, kind):
        if kd < 0:
            continue
        if kd == 0:
            r, J = oracle.eval_factor(0, r9, x0[:4], x0[4:])
        else:
            r, J = oracle.eval_factor(2, np.concatenate([r9[:7], np.zeros(5)]), x0[:4], x0[4:])
        # local parameterization: d/d delta = J_q(4) * P(4x3)
        q = x0[:4]
        P = np.array([[q[3], q[2], -q[1]], [-q[2], q[3], q[0]], [q[1], -q[0], q[3]], [-q[0], -q[1], -q[2]]])
        Jl = np.concatenate([J[:, :4] @ P, J[:, 4:]], axis=1)
        s = float(r @ r)
        if s > 0.01:
            rr = np.sqrt(s)
            acc[0] += 0.5 * (2 * 0.1 * rr - 0.01)
            sc = np.sqrt(0.1 / rr)
        else:
            acc[0] += 0.5 * s
            sc = 1.0
        Jl, r = Jl * sc, r * sc
        A = Jl.T @ Jl
        acc[1:22] += A[np.triu_indices(6)]
        acc[22:28] += Jl.T @ r
    assert np.allclose(ne, acc, rtol=1e-9, atol=1e-12)
    # the full solve (10 iterations, mapOptimization) vs the oracle's Ceres restatement
    xg, sg = pkg.mapping.pose_solve(ctx, rec, kind, x0, 10)
    xo, so = oracle.map_solve(rec, kind, x0, 10)
    assert np.max(np.abs(xg - xo)) < POSE_TOL, (xg, xo)
    assert sg[0] == so[0] and sg[1] == so[1]
    assert sg[2] == (kind == 0).sum() and sg[3] == (kind == 2).sum()


def test_mapopt_sequence(pkg, oracle, ctx, synth):
    """mapOptimization ground-map stage over a short drive: Build on the first frame, then
    VoxelGrid(0.8) + plane association + Ceres(10) + transformUpdate + Add_Points(0.4)."""
    go = pkg.mapping.MapOptimization(ctx, 0.4, 0.2)
    om = oracle.IkdMap(0.4)
    ostate = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    for k in range(5):
        scan = synth.make_scan(k).reshape(-1, 4)
        ground = _f32(scan[np.abs(scan[:, :3]).sum(1) > 0])
        q, t = synth.ground_truth_pose(k).as_qt()
        odom = synth.perturb_pose(q, t, 0.02, 0.2, seed=10 + k)  # drifting odometry
        pg, sg = go.callback(ground, odom)
        po, ostate, so = oracle.mapopt_step(om, ground, odom, ostate)
        assert np.max(np.abs(pg - po)) < POSE_TOL, (k, pg, po)
        assert np.max(np.abs(go.state - ostate)) < POSE_TOL, k
        assert list(sg) == list(so), (k, sg, so)
        assert go.map.size() == om.size(), k
    go.map.close()


@pytest.mark.parametrize("empty_first", [False, True])
def test_mapopt_corner_map(pkg, oracle, ctx, synth, empty_first):
    """mapOptimization with its corner ikd-Tree (KD_TREE(0.3, 0.6, 0.8), mapOptimization.cpp:505):
    pc_corner (the scan's less-sharp cloud) Built on the first keyframe (:193-195), then
    Add_Points(downsample) at the keyframe pose (:477-479).  Poses, summaries and both maps' live
    points against the oracle, frame by frame.  empty_first: the first keyframe's pc_corner is
    empty, so the tree is Built empty and the next cloud goes in through Add_Points (downsampled),
    not through a Build."""
    go = pkg.mapping.MapOptimization(ctx, 0.4, 0.2, corner=True)
    om, ocm = oracle.IkdMap(0.4), oracle.IkdMap(0.8)
    ostate = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    for k in range(5):
        scan = synth.make_scan(20 + k)
        flat = scan.reshape(-1, 4)
        ground = _f32(flat[np.abs(flat[:, :3]).sum(1) > 0])
        corner = oracle.scan_registration(scan).less_sharp
        if empty_first and k == 0:
            corner = corner[:0]
        q, t = synth.ground_truth_pose(20 + k).as_qt()
        odom = synth.perturb_pose(q, t, 0.02, 0.2, seed=40 + k)
        pg, sg = go.callback(ground, odom, corner)
        po, ostate, so = oracle.mapopt_step_corner(om, ocm, ground, corner, odom, ostate)
        assert np.max(np.abs(pg - po)) < POSE_TOL, (k, pg, po)
        assert list(sg) == list(so), (k, sg, so)
        assert go.map.size() == om.size(), k
        assert go.corner_map.size() == ocm.size(), (k, go.corner_map.size(), ocm.size())
        gp, op = _by_id(go.corner_map.points()), ocm.points()
        assert np.array_equal(gp[:, 3].view(np.int32), op[:, 3].view(np.int32)), k
        np.testing.assert_allclose(gp[:, :3], op[:, :3], atol=1e-4)
    assert go.corner_map.size() > 0
    go.close()


def test_mapopt_corner_fed_from_batch(pkg, oracle, ctx, synth):
    """lislam_batch_mapopt_corner: the scan's less-sharp cloud on the device is pc_corner."""
    S = 3
    scans = synth.make_sequence(S, start=40)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.ground(S)
    go = pkg.mapping.MapOptimization(ctx, 0.4, 0.2, corner=True)
    om, ocm = oracle.IkdMap(0.4), oracle.IkdMap(0.8)
    ostate = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    for k in range(S):
        g_ref, _, _ = oracle.ground_extract(scans[k])
        f = oracle.scan_registration(scans[k])
        merged = np.concatenate([g_ref, f.less_flat]).astype(np.float32)
        q, t = synth.ground_truth_pose(40 + k).as_qt()
        odom = synth.perturb_pose(q, t, 0.02, 0.2, seed=60 + k)
        pg, sg = go.callback_batch(b, k, odom)
        po, ostate, so = oracle.mapopt_step_corner(om, ocm, merged, f.less_sharp, odom, ostate)
        assert np.max(np.abs(pg - po)) < POSE_TOL, (k, pg, po)
        assert list(sg) == list(so), (k, sg, so)
        assert go.corner_map.size() == ocm.size(), k
    go.close()
    b.close()


def test_laser_mapping(pkg, oracle, ctx, synth):
    M = synth.make_corridor_map(300_000, spacing=0.05)
    E = synth.make_edge_map(40)
    rng = np.random.default_rng(13)
    truth = np.array([0, 0, 0, 1, 5.0, 0.1, 0.0])
    x0 = synth.perturb_pose(truth[:4], truth[4:], 0.05, 0.5, seed=5)
    gs, gc = pkg.mapping.IkdMap(ctx, 0.4, 0.1), pkg.mapping.IkdMap(ctx, 0.8, 0.2)
    os_, oc = oracle.IkdMap(0.4), oracle.IkdMap(0.8)
    for a, b, P in ((gs, os_, M), (gc, oc, E)):
        a.build(P)
        b.build(P)
    Qs = M[rng.choice(len(M), 3000, replace=False)].copy()
    Qs[:, :3] -= truth[4:7].astype(np.float32)
    Qc = E[rng.choice(len(E), 400, replace=False)].copy()
    Qc[:, :3] -= truth[4:7].astype(np.float32)
    xg, stg = pkg.mapping.laser_mapping(gc, gs, Qc, Qs, x0)
    xo, sto = oracle.laser_mapping(oc, os_, Qc, Qs, x0)
    assert np.max(np.abs(xg - xo)) < POSE_TOL, (xg, xo)
    assert list(stg) == list(sto)
    assert np.linalg.norm(xg[4:] - truth[4:]) < np.linalg.norm(x0[4:] - truth[4:])
    gs.close()
    gc.close()


def test_map_solve_modes_agree(pkg, oracle, ctx, synth, monkeypatch):
    """The pose solve with one launch per evaluation (k_lm_evalstep, default), in one launch
    (LISLAM_MAP_SOLVE=persistent: k_lm_solve) and on that launch's give-up path (a zero wait bound:
    every workgroup that has to wait gives up at once and k_lm_rescue finishes the solve on one
    workgroup) return the same bits, and the oracle's pose.  20k records: 79 workgroups per
    evaluation."""
    M = synth.make_corridor_map(400_000, spacing=0.05)
    gs = pkg.mapping.IkdMap(ctx, 0.4, 0.3)
    gs.build(M)
    os_ = oracle.IkdMap(0.4)
    os_.build(M)
    rng = np.random.default_rng(17)
    truth = np.array([0, 0, 0, 1, 4.0, 0.2, 0.0])
    x0 = synth.perturb_pose(truth[:4], truth[4:], 0.05, 0.5, seed=9)
    Qs = M[rng.choice(len(M), 20000, replace=False)].copy()
    Qs[:, :3] -= truth[4:7].astype(np.float32)
    empty = np.zeros((0, 4), np.float32)
    out = {}
    for mode, env in (("launches", {}), ("persistent", {"LISLAM_MAP_SOLVE": "persistent"}),
                      ("rescue", {"LISLAM_MAP_SOLVE": "persistent", "LISLAM_MAP_SOLVE_WAIT_US": "0"})):
        for k in ("LISLAM_MAP_SOLVE", "LISLAM_MAP_SOLVE_WAIT_US"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out[mode] = pkg.mapping.laser_mapping(gs, gs, empty, Qs, x0)
    for mode in ("persistent", "rescue"):
        assert np.array_equal(out[mode][0], out["launches"][0]), (mode, out[mode][0], out["launches"][0])
        assert list(out[mode][1]) == list(out["launches"][1]), mode
    xo, sto = oracle.laser_mapping(os_, os_, empty, Qs, x0)
    assert np.max(np.abs(out["launches"][0] - xo)) < POSE_TOL
    assert list(out["launches"][1]) == list(sto)
    gs.close()


def test_mapopt_fed_from_batch(pkg, oracle, ctx, synth):
    """mapOptimizationCallback's input assembled on the device (lislam_batch_mapopt): the scan's
    GroundPointOut followed by its less-flat cloud (mapOptimization.cpp:136-150), against the
    oracle's ground extraction + scan registration concatenated on the host."""
    S = 4
    scans = synth.make_sequence(S, start=12)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.ground(S)
    go = pkg.mapping.MapOptimization(ctx, 0.4, 0.2)
    om = oracle.IkdMap(0.4)
    ostate = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    for k in range(S):
        g_ref, _, _ = oracle.ground_extract(scans[k])
        lf = oracle.scan_registration(scans[k]).less_flat
        merged = np.concatenate([g_ref, lf]).astype(np.float32)
        q, t = synth.ground_truth_pose(12 + k).as_qt()
        odom = synth.perturb_pose(q, t, 0.02, 0.2, seed=30 + k)
        pg, sg = go.callback_batch(b, k, odom)
        po, ostate, so = oracle.mapopt_step(om, merged, odom, ostate)
        assert np.max(np.abs(pg - po)) < POSE_TOL, (k, pg, po)
        assert list(sg) == list(so), (k, sg, so)
        assert go.map.size() == om.size(), k
    go.map.close()
    b.close()


def test_laser_mapping_config5_full_map(pkg, oracle, ctx, synth):
    """Config 5 at its full size (bench.py --workload map): 20k surf queries of one 64x1024 scan
    against a 5M-point corridor map, pose perturbed 5 cm / 0.5 deg, 2 outer passes of exact 5-NN
    + plane fits + LidarPlaneNormFactor + Ceres(4) (laserMapping.cpp:620-850).  The 5-NN of a
    2000-query sample is bit-exact; pose within 1e-4 and block counts equal."""
    M = synth.make_corridor_map(5_000_000, spacing=0.05)
    k = 50
    scan = synth.make_scan(k).reshape(-1, 4)
    scan = scan[np.abs(scan[:, :3]).sum(1) > 0]
    rng = np.random.default_rng(7)
    Q = _f32(scan[rng.choice(len(scan), 20000, replace=False)])
    vi = np.floor(Q[:, :3] / 0.4).astype(np.int64)  # VoxelGrid output order (laserMapping.cpp:613-615)
    Q = Q[np.lexsort((vi[:, 0], vi[:, 1], vi[:, 2]))]
    q, t = synth.ground_truth_pose(k).as_qt()
    x0 = synth.perturb_pose(q, t, 0.05, 0.5, seed=3)
    g = pkg.mapping.IkdMap(ctx, 0.4, 0.3)  # the bench's hash-grid cell
    g.build(M)
    o = oracle.IkdMap(0.4)
    o.build(M)
    assert g.size() == o.size() == len(M)
    # the sample's queries in the map frame at the initial guess
    from scipy.spatial.transform import Rotation

    S = Q[:2000, :3].astype(np.float64)
    Sw = _f32(Rotation.from_quat(x0[:4]).apply(S) + x0[4:7])
    _knn_equal(g.nearest_search(Sw, 5), o.knn(Sw, 5), 5)
    empty = np.zeros((0, 4), np.float32)
    xg, stg = pkg.mapping.laser_mapping(g, g, empty, Q, x0)
    xo, sto = oracle.laser_mapping(o, o, empty, Q, x0)
    assert np.max(np.abs(xg - xo)) < POSE_TOL, (xg, xo)
    assert list(stg) == list(sto), (stg, sto)
    assert sto[1] > 19000  # almost every query found a plane
    g.close()
