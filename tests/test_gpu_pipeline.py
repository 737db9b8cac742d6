"""The reference's whole per-scan cycle through the C ABI against the oracle (SURVEY.md §8 rows
a1-a22 and (f) 2-4 together): scanRegistration + ImageHandler (features, images, GroundPointOut),
feature_tracker::detectfeatures (T_s2s, skipped frames), laserOdometry with the reference's default
gating (only "skip_intensity" frames optimize), odomHandler's fusion of the A-LOAM and intensity
odometry, and mapOptimization's ground map fed with GroundPointOut + less-flat — every stage on the
device, the host only relaying poses as the ROS topics would."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4


def _mat(p):
    x, y, z, w = p[:4]
    T = np.eye(4)
    T[:3, :3] = [[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                 [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                 [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]
    T[:3, 3] = p[4:7]
    return T


def _pose(T):
    R = T[:3, :3]
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0)
        q = np.array([(R[2, 1] - R[1, 2]) * 0.5 / s, (R[0, 2] - R[2, 0]) * 0.5 / s, (R[1, 0] - R[0, 1]) * 0.5 / s, 0.5 * s])
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = math.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q = np.zeros(4)
        q[i] = 0.5 * s
        q[3] = (R[k, j] - R[j, k]) * 0.5 / s
        q[j] = (R[j, i] + R[i, j]) * 0.5 / s
        q[k] = (R[k, i] + R[i, k]) * 0.5 / s
    q /= np.linalg.norm(q)
    return np.concatenate([q, T[:3, 3]])


def _intensity_odom(T_s2s):
    """tfBroadcast (intensity_feature_tracker.cpp:817-866): T_s2m = T_s2m * T_s2s per frame."""
    T, out = np.eye(4), []
    for k, p in enumerate(T_s2s):
        if k > 0:
            T = T @ _mat(p)
        out.append(_pose(T))
    return np.array(out)


def test_full_cycle_matches_oracle(pkg, oracle, synth):
    H, W = 64, 1024
    scans = synth.make_sequence(6, start=90)
    scans[3, ..., 3] = 0  # a blank intensity image: the tracker skips frames 3 and 4 (no matches)
    S = scans.shape[0]
    mask = oracle.hand_held_mask()
    nat = pkg.native
    with pkg.Context(n_scans=H, width=W) as ctx:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.intensity_odometry(S, 1000, mask)
        b.ground(S)
        orb = np.stack([b.download(nat.OUT_ORB_STATS, k) for k in range(S)])
        use = (orb[:, 0] == 0).astype(np.int32)  # the "skip_intensity" frames
        b.odometry(S, S - 1, use_aloam=use)
        aloam = np.stack([b.download(nat.OUT_POSE, k) for k in range(S)])
        inten = _intensity_odom(np.stack([b.download(nat.OUT_ORB_T, k) for k in range(S)]))
        fuser = pkg.loop.OdomHandler(ctx)
        fused = fuser.fuse(aloam, inten, use)
        fuser.close()
        gmap = pkg.mapping.MapOptimization(ctx, 0.4, 0.2)
        mapped = [gmap.callback_batch(b, k, fused[k]) for k in range(S)]
        gmap.map.close()
        b.close()

    feats = [oracle.scan_registration(s) for s in scans]
    rst, rT = oracle.intensity_odometry(np.stack([f.img_intensity for f in feats]),
                                        np.stack([f.cloud_track for f in feats]), 1000, mask)
    ruse = (rst[:, 0] == 0).astype(np.int32)
    ruse[0] = 0
    assert list(use) == [0, 0, 0, 1, 1, 0] and np.array_equal(use, ruse)
    pose, _, _ = oracle.odometry_chain(feats, use_aloam=ruse)
    assert np.max(np.abs(aloam - pose)) < POSE_TOL
    rinten = _intensity_odom(rT)
    assert np.max(np.abs(inten - rinten)) < POSE_TOL
    rfused = oracle.OdomFuser().step(pose, rinten, ruse)
    assert np.max(np.abs(fused - rfused)) < POSE_TOL
    om = oracle.IkdMap(0.4)
    state = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    for k in range(S):
        ground, _, _ = oracle.ground_extract(scans[k])
        merged = np.concatenate([ground, feats[k].less_flat]).astype(np.float32)
        po, state, so = oracle.mapopt_step(om, merged, rfused[k], state)
        pg, sg = mapped[k]
        assert np.max(np.abs(pg - po)) < POSE_TOL, (k, pg, po)
        assert list(sg) == list(so), (k, sg, so)
