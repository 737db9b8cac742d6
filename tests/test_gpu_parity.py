"""GPU parity of the HIP path (through the C ABI) against the CPU oracle on the same seeded inputs.

Integer / index / byte outputs and the float feature clouds must be bit-exact (same IEEE
operations, -ffp-contract=off on both sides, canonical tie order); poses within the north-star
tolerance 1e-4 m / 1e-4 rad (measured agreement is ~1e-15).
"""
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4  # BASELINE.json north_star: <= 1e-4 m / <= 1e-4 rad


@pytest.fixture(scope="module")
def contexts(pkg):
    made = {}

    def get(H, W):
        if (H, W) not in made:
            made[(H, W)] = pkg.Context(n_scans=H, width=W)
        return made[(H, W)]

    yield get
    for c in made.values():
        c.close()


FEATURES = ("laser_cloud", "sharp", "less_sharp", "flat", "less_flat")


def assert_features_equal(pkg, b, k, ref, images=True):
    n = pkg.native
    g = b.features(k)
    for name in FEATURES:
        a, r = getattr(g, name), getattr(ref, name)
        assert a.shape == r.shape, (k, name, a.shape, r.shape)
        assert np.array_equal(a, r), (k, name)
    assert b.count(n.OUT_LESS_FLAT, k) == ref.less_flat.shape[0]  # count-only download
    assert np.array_equal(b.download(n.OUT_CURVATURE, k), ref.curvature)
    assert np.array_equal(b.download(n.OUT_LABEL, k), ref.label)
    lo = b.download(n.OUT_LINE_OFFSETS, k)
    assert np.array_equal(lo[:-1] + 5, ref.scan_start) and np.array_equal(lo[1:] - 6, ref.scan_end)
    if images:
        assert np.array_equal(b.download(n.OUT_IMAGE_RANGE, k), ref.img_range.ravel())
        assert np.array_equal(b.download(n.OUT_IMAGE_INTENSITY, k), ref.img_intensity.ravel())
        assert np.array_equal(b.download(n.OUT_CLOUD_TRACK, k), ref.cloud_track.reshape(-1, 4))


@pytest.mark.parametrize("H,W,S", [(64, 1024, 4), (128, 2048, 2), (16, 256, 3), (32, 512, 3)])
def test_features_bit_exact(pkg, oracle, synth, contexts, H, W, S):
    ctx = contexts(H, W)
    scans = synth.make_sequence(S, H, W, start=10)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    for k in range(S):
        assert_features_equal(pkg, b, k, oracle.scan_registration(scans[k]))
    b.close()


def test_golden_fixture_on_gpu(pkg, contexts):
    import os

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "scan16x256_chain3.npz"))
    ctx = contexts(16, 256)
    b = pkg.Batch(ctx, 3)
    b.upload(g["scans"])
    b.extract(3)
    b.odometry(3, 2)
    for k in range(3):
        f = b.features(k)
        for name in FEATURES:
            assert np.array_equal(getattr(f, name), g[f"s{k}_{name}"]), (k, name)
        para = b.download(pkg.native.OUT_PARA, k)
        assert np.max(np.abs(para - g["odom_para"][k])) < POSE_TOL
        assert np.array_equal(b.download(pkg.native.OUT_STATS, k)[:6], g["odom_stats"][k])
    b.close()


def test_edge_cases(pkg, oracle, contexts):
    ctx = contexts(16, 256)
    rng = np.random.default_rng(0)
    cases = []
    cases.append(np.zeros((16, 256, 4), np.float32))                              # empty (all dropouts)
    up = np.zeros((16, 256, 4), np.float32); up[..., 2] = 10.0                      # outside every scan line
    cases.append(up)
    near = rng.uniform(-0.2, 0.2, size=(16, 256, 4)).astype(np.float32)             # all closer than 0.3 m
    cases.append(near)
    from importlib import import_module
    synth = import_module("intensity_based_lidar_slam_for_me-_amd.synth")
    s = synth.make_scan(5, 16, 256).reshape(-1, 4)
    cases.append(s[rng.permutation(s.shape[0])].reshape(16, 256, 4))              # not ring ordered
    part = synth.make_scan(6, 16, 256).copy(); part[:, :100] = 0                     # first points dropped
    cases.append(part)
    b = pkg.Batch(ctx, len(cases))
    b.upload(np.stack(cases))
    b.extract(len(cases))
    for k, c in enumerate(cases):
        assert_features_equal(pkg, b, k, oracle.scan_registration(c))
    b.close()


def test_long_lines_global_path(pkg, oracle, synth, contexts):
    """A scan whose points all fall into few lines (> 2048 points per line) runs the global-
    scratch path of k_scan_lines; results stay bit-exact."""
    ctx = contexts(16, 1024)
    s = synth.make_scan(2, 16, 1024).copy()
    s[8:] = s[:8]  # duplicate the top half: 2 x 1024 points per scan line
    b = pkg.Batch(ctx, 1)
    b.upload(s[None])
    b.extract(1)
    assert_features_equal(pkg, b, 0, oracle.scan_registration(s))
    b.close()


def test_ouster_point_step_layout(pkg, oracle, synth, contexts):
    """PointCloud2 with point_step 48 (Ouster os_cloud_node) gives the same features."""
    ctx = contexts(16, 256)
    scan = synth.make_scan(1, 16, 256)
    raw = np.zeros((16 * 256, 12), np.float32)
    raw[:, 0:3] = scan.reshape(-1, 4)[:, :3]
    raw[:, 4] = scan.reshape(-1, 4)[:, 3]
    raw[:, 5] = 123.0  # other fields
    reg = pkg.ScanRegistration(ctx)
    from importlib import import_module
    fe = import_module("intensity_based_lidar_slam_for_me-_amd.frontend")
    got = reg.laser_cloud_handler(raw, fe.OUSTER_LAYOUT)
    ref = oracle.scan_registration(scan)
    for name in FEATURES:
        assert np.array_equal(getattr(got, name), getattr(ref, name)), name
    assert np.array_equal(got.image_intensity, ref.img_intensity)


def test_upload_async_overlapped_batches(pkg, oracle, synth, contexts):
    """lislam_batch_upload_async (copy stream, 16-scan chunks parsed as they land): three batches
    of Ouster PointCloud2 bytes queued back to back, each extracted right after its upload, with
    the next upload issued before the previous extraction has run (its chunks wait for the previous
    parse, its parse for the previous extraction); 35 scans = two full chunks and a ragged one.
    Features equal the oracle's for every batch."""
    import ctypes

    import torch

    from importlib import import_module
    fe = import_module("intensity_based_lidar_slam_for_me-_amd.frontend")
    ctx = contexts(16, 256)
    S = 35
    batches = [synth.make_sequence(S, 16, 256, start=7 * j) for j in range(3)]
    wires = []
    for sc in batches:
        w = torch.zeros((S, 16 * 256, 12), dtype=torch.float32, pin_memory=True)
        w.numpy()[:, :, 0:3] = sc.reshape(S, -1, 4)[:, :, :3]
        w.numpy()[:, :, 4] = sc.reshape(S, -1, 4)[:, :, 3]
        w.numpy()[:, :, 5] = 7.0  # other fields
        wires.append(w)
    b = pkg.Batch(ctx, S)
    got = []
    for j, w in enumerate(wires):
        b.upload_async(ctypes.c_void_p(w.data_ptr()), S, fe.OUSTER_LAYOUT)
        b.extract(S)
        if j < 2:
            b.upload_async(ctypes.c_void_p(w.data_ptr()), S, fe.OUSTER_LAYOUT)  # the same bytes again,
            b.extract(S)                                                        # queued behind the first
        got.append([b.features(k) for k in (0, 16, 34)])
    for j, sc in enumerate(batches):
        for g, k in zip(got[j], (0, 16, 34)):
            ref = oracle.scan_registration(sc[k])
            for name in FEATURES:
                assert np.array_equal(getattr(g, name), getattr(ref, name)), (j, k, name)
    b.close()


@pytest.mark.parametrize("chain_len", [1, 3, 7])
def test_odometry_chains(pkg, oracle, synth, contexts, chain_len):
    S = 8
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(S, start=20)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, chain_len)
    feats = [oracle.scan_registration(s) for s in scans]
    for c0 in range(0, S - 1, chain_len):
        chain = feats[c0:c0 + chain_len + 1]
        pose, rel, st = oracle.odometry_chain(chain)
        for j in range(1, len(chain)):
            k = c0 + j
            para = b.download(pkg.native.OUT_PARA, k)
            pw = b.download(pkg.native.OUT_POSE, k)
            assert np.max(np.abs(para - rel[j])) < POSE_TOL, (k, para, rel[j])
            assert np.max(np.abs(pw - pose[j])) < POSE_TOL
            gst = b.download(pkg.native.OUT_STATS, k)
            assert np.array_equal(gst[:4], st[j][:4]), (k, gst, st[j])  # correspondence counts
    b.close()


@pytest.mark.parametrize("chain_len", [3, 7])
def test_odometry_gated_reference_default(pkg, oracle, synth, contexts, chain_len):
    """The reference's default gating (laserOdometry.cpp:403-417): only "skip_intensity" scans are
    optimized, the others carry the previous estimate into the pose."""
    S = 8
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(S, start=50)
    use = np.array([0, 1, 0, 0, 1, 1, 0, 1], np.int32)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, chain_len, use_aloam=use)
    feats = [oracle.scan_registration(s) for s in scans]
    for c0 in range(0, S - 1, chain_len):
        chain = feats[c0:c0 + chain_len + 1]
        pose, rel, st = oracle.odometry_chain(chain, use_aloam=use[c0:c0 + chain_len + 1])
        for j in range(1, len(chain)):
            k = c0 + j
            assert np.max(np.abs(b.download(pkg.native.OUT_PARA, k) - rel[j])) < POSE_TOL, k
            assert np.max(np.abs(b.download(pkg.native.OUT_POSE, k) - pose[j])) < POSE_TOL, k
            assert np.array_equal(b.download(pkg.native.OUT_STATS, k)[:4], st[j][:4]), k
    # the gate the ORB front end produces for this stream (detectfeatures' skipped frames)
    b.intensity_odometry(S, 1000, pkg.intensity.set_mask())
    flags = b.skip_flags(S)
    b.odometry(S, S - 1, use_aloam=flags)
    pose, rel, _ = oracle.odometry_chain(feats, use_aloam=flags)
    for k in range(1, S):
        assert np.max(np.abs(b.download(pkg.native.OUT_POSE, k) - pose[k])) < POSE_TOL
    b.close()


def test_odometry_node_stream_api(pkg, oracle, synth, contexts):
    """lislam_odom_step frame by frame == a single oracle chain over the whole stream."""
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(5, start=40)
    feats = [oracle.scan_registration(s) for s in scans]
    pose, rel, st = oracle.odometry_chain(feats)
    node = pkg.LaserOdometry(ctx)
    for k, f in enumerate(feats):
        para, pw, gst = node.step(f)
        assert np.max(np.abs(para - rel[k])) < POSE_TOL
        assert np.max(np.abs(pw - pose[k])) < POSE_TOL
        assert np.array_equal(gst[:4], st[k][:4])
    node.close()


def test_odometry_node_gated_stream(pkg, oracle, synth, contexts):
    """lislam_odom_step_gated frame by frame (the sharp cloud's frame_id decides) == the oracle's
    gated chain."""
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(6, start=70)
    feats = [oracle.scan_registration(s) for s in scans]
    use = np.array([0, 1, 0, 1, 1, 0], np.int32)
    pose, rel, st = oracle.odometry_chain(feats, use_aloam=use)
    node = pkg.LaserOdometry(ctx)
    for k, f in enumerate(feats):
        para, pw, gst = node.step(f, skip_flag="skip_intensity" if use[k] else "os_sensor")
        assert np.max(np.abs(para - rel[k])) < POSE_TOL, k
        assert np.max(np.abs(pw - pose[k])) < POSE_TOL, k
        assert np.array_equal(gst[:4], st[k][:4]), k
    node.close()


def test_scan_registration_single_api(pkg, oracle, synth, contexts):
    ctx = contexts(64, 1024)
    scan = synth.make_scan(77)
    got = pkg.ScanRegistration(ctx).laser_cloud_handler(scan)
    ref = oracle.scan_registration(scan)
    for name in FEATURES:
        assert np.array_equal(getattr(got, name), getattr(ref, name)), name


def test_factor_evaluation_vs_oracle_autodiff(pkg, oracle, contexts):
    ctx = contexts(16, 256)
    rng = np.random.default_rng(3)
    n = 60
    kind = np.arange(n) % 3
    pts = rng.normal(size=(n, 12))
    for i in range(n):
        if kind[i] == 2:
            v = rng.normal(size=3)
            pts[i, 3:6] = v / np.linalg.norm(v)
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    t = rng.normal(size=3)
    r, J = pkg.eval_factors(ctx, kind, pts, q, t)
    P = np.array([[q[3], q[2], -q[1]], [-q[2], q[3], q[0]], [q[1], -q[0], q[3]], [-q[0], -q[1], -q[2]]])
    for i in range(n):
        rr, JJ = oracle.eval_factor(int(kind[i]), pts[i], q, t)
        R = rr.shape[0]
        np.testing.assert_allclose(r[i, :R], rr, rtol=1e-12, atol=1e-12)
        Jl = np.concatenate([JJ[:, :4] @ P, JJ[:, 4:]], axis=1)
        np.testing.assert_allclose(J[i, :R], Jl, rtol=1e-9, atol=1e-10)


def test_high_res_pair_odometry(pkg, oracle, synth, contexts):
    """128 x 2048 (config 3): features bit-exact and one odometry pair within tolerance."""
    ctx = contexts(128, 2048)
    scans = synth.make_sequence(2, 128, 2048, start=3)
    b = pkg.Batch(ctx, 2)
    b.upload(scans)
    b.extract(2)
    b.odometry(2, 1)
    feats = [oracle.scan_registration(s) for s in scans]
    _, rel, st = oracle.odometry_chain(feats)
    assert np.max(np.abs(b.download(pkg.native.OUT_PARA, 1) - rel[1])) < POSE_TOL
    assert np.array_equal(b.download(pkg.native.OUT_STATS, 1)[:4], st[1][:4])
    b.close()


def test_pointcloud2_wire_format_in_out(pkg, oracle, synth, contexts):
    """fromROSMsg / toROSMsg on the device: a batch uploaded in Ouster's 48-byte layout extracts
    the same features, and the feature clouds come back as PCL PointXYZI PointCloud2 bytes."""
    from importlib import import_module
    fe = import_module("intensity_based_lidar_slam_for_me-_amd.frontend")
    ctx = contexts(16, 256)
    scans = synth.make_sequence(2, 16, 256, start=4)
    raw = np.zeros((2, 16 * 256, 12), np.float32)
    raw[..., 0:3] = scans.reshape(2, -1, 4)[..., :3]
    raw[..., 4] = scans.reshape(2, -1, 4)[..., 3]
    raw[..., 7] = -5.0  # a field the path does not read
    b = pkg.Batch(ctx, 2)
    b.upload(raw, fe.OUSTER_LAYOUT)
    b.extract(2)
    n = pkg.native
    for k in range(2):
        assert_features_equal(pkg, b, k, oracle.scan_registration(scans[k]))
        for what in (n.OUT_LASER_CLOUD, n.OUT_SHARP, n.OUT_LESS_FLAT):
            ref = b.download(what, k)
            msg = np.frombuffer(b.download_cloud(what, k), np.uint8).reshape(-1, 32)
            assert msg.shape[0] == ref.shape[0]
            f = msg.view(np.float32)
            assert np.array_equal(f[:, [0, 1, 2, 4]], ref)
            assert not msg[:, 12:16].any() and not msg[:, 20:].any()
    b.close()


@pytest.mark.parametrize("quantum", [0.05, 0.1, 0.2])
def test_voxel_grid_std_sort_order_heavy_ties(pkg, oracle, synth, contexts, quantum):
    """The a7 VoxelGrid replays the order libstdc++'s std::sort leaves equal voxels in
    (PCL VoxelGrid, scanRegistration.cpp:583-586): coordinates snapped to `quantum` put many
    points of a line into each 0.2 m voxel, so the centroids' summation order (introsort
    partitions, heap-sort fallback, final insertion sort) decides their float bits.  64 x 1024
    (register path) plus a doubled-line scan (global-scratch path), bit-exact against the oracle
    in the reference's VoxelGrid order; the index order (canonical) differs."""
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(3, start=70).copy()
    xyz = scans[..., :3]
    nz = np.abs(xyz).sum(-1) > 0
    xyz[nz] = np.round(xyz[nz] / quantum) * quantum
    b = pkg.Batch(ctx, 3)
    b.upload(scans)
    b.extract(3)
    differs = False
    for k in range(3):
        ref = oracle.scan_registration(scans[k])
        assert_features_equal(pkg, b, k, ref)
        can = oracle.scan_registration(scans[k], canonical=True).less_flat
        differs |= can.shape != ref.less_flat.shape or not np.array_equal(can, ref.less_flat)
    assert differs  # the tie order matters on these inputs
    b.close()
    # far points: voxel indices of 2^21 and more (the kernel's dense-numbering path)
    far = synth.make_sequence(2, start=80).copy()
    far[..., :3] *= np.float32(25.0)
    b = pkg.Batch(ctx, 2)
    b.upload(far)
    b.extract(2)
    for k in range(2):
        assert_features_equal(pkg, b, k, oracle.scan_registration(far[k]))
    b.close()
    ctx2 = contexts(16, 1024)
    s = synth.make_scan(9, 16, 1024).copy()
    s[8:] = s[:8]
    nz = np.abs(s[..., :3]).sum(-1) > 0
    s[..., :3][nz] = np.round(s[..., :3][nz] / quantum) * quantum
    b = pkg.Batch(ctx2, 1)
    b.upload(s[None])
    b.extract(1)
    assert_features_equal(pkg, b, 0, oracle.scan_registration(s))
    b.close()


@pytest.mark.parametrize("kind", ["snapped", "duplicated"])
def test_segment_sort_std_sort_order_ties(pkg, oracle, synth, contexts, kind):
    """Equal curvatures in a segment (scanRegistration.cpp:445): the sharp / flat walks reach
    them in the order libstdc++'s std::sort leaves them, which the kernel replays (introsort
    order + window rank) once a pick meets a tie.  Snapped coordinates (0.1 m grid) and runs
    of identical points (curvature exactly 0) make many curvatures tie; the labels, sharp, less-sharp and flat
    clouds are bit-exact against the oracle's reference order (ties=0), and the oracle's
    index-order segments (ties=1) pick differently on these inputs.  The global-scratch path
    (a doubled 2048-point line) is covered too.  TIES_INDEX matches the index-order oracle."""
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(2, start=40).copy()
    xyz = scans[..., :3]
    nz = np.abs(xyz).sum(-1) > 0
    if kind == "snapped":
        xyz[nz] = np.round(xyz[nz] / 0.1) * 0.1
    else:  # runs of 16 identical points: curvature exactly 0 inside each run
        scans[:] = scans[:, :, (np.arange(scans.shape[2]) // 16) * 16]
    b = pkg.Batch(ctx, 2)
    b.upload(scans)
    b.extract(2)
    moved = 0
    for k in range(2):
        ref = oracle.scan_registration(scans[k], ties=0)
        assert_features_equal(pkg, b, k, ref)
        seg_index = oracle.scan_registration(scans[k], ties=1)
        moved += int(np.sum(ref.label != seg_index.label))
    assert moved > 0  # the segment tie order decides picks on these inputs
    try:
        ctx.set_tie_order(ctx.TIES_INDEX)
        b.extract(2)
        for k in range(2):
            assert_features_equal(pkg, b, k, oracle.scan_registration(scans[k], canonical=True))
    finally:
        ctx.set_tie_order(ctx.TIES_REFERENCE)
    b.close()
    ctx2 = contexts(16, 1024)
    s2 = _tied_long_lines(synth)  # lines of 2048 points: the global-scratch line path
    b = pkg.Batch(ctx2, 1)
    b.upload(s2[None])
    b.extract(1)
    assert_features_equal(pkg, b, 0, oracle.scan_registration(s2, ties=0))
    b.close()


def _tied_long_lines(synth):
    s = synth.make_scan(9, 16, 1024).copy()
    s[8:] = s[:8]
    nz = np.abs(s[..., :3]).sum(-1) > 0
    s[..., :3][nz] = np.round(s[..., :3][nz] / 0.1) * 0.1
    return s


def test_tie_order_index_mode(pkg, oracle, synth, contexts):
    """lislam_set_tie_order(LISLAM_TIES_INDEX): the VoxelGrid sums a voxel's points in input order,
    bit-exact against the oracle's index-order mode (canonical); the reference order is the
    default and comes back when set again."""
    ctx = contexts(64, 1024)
    scans = synth.make_sequence(2, start=90)
    try:
        ctx.set_tie_order(ctx.TIES_INDEX)
        b = pkg.Batch(ctx, 2)
        b.upload(scans)
        b.extract(2)
        for k in range(2):
            assert_features_equal(pkg, b, k, oracle.scan_registration(scans[k], canonical=True))
        ctx.set_tie_order(ctx.TIES_REFERENCE)
        b.extract(2)
        for k in range(2):
            assert_features_equal(pkg, b, k, oracle.scan_registration(scans[k]))
        b.close()
    finally:
        ctx.set_tie_order(ctx.TIES_REFERENCE)
