"""CPU pins of the loop-closure ICP and odometry fusion restatements (oracle_map.cpp
oracle_loop_icp, oracle_fuse.cpp) against independent numpy
transcriptions: PCL 1.10's IterativeClosestPoint loop with an SVD Umeyama (numpy, double) and a
scipy kd-tree, and odomHandler's callback with numpy's general 4x4 inverse.  PCL and Eigen are
absent: parity against them is unpinned beyond the published algorithms.  No GPU."""
import math

import numpy as np
import pytest
from scipy.spatial import cKDTree

from loop_cases import corridor_loop, drift, random_room


def _voxel(P, leaf):
    """pcl::VoxelGrid (stable by voxel index, float centroid in input order)."""
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = P[:, :3].min(0), P[:, :3].max(0)
    min_b = np.floor(mn * inv).astype(np.int64)
    div = np.floor(mx * inv).astype(np.int64) - min_b + 1
    ijk = (np.floor(P[:, :3] * inv) - min_b.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    out = []
    s = 0
    while s < len(order):
        e = s
        while e < len(order) and idx[order[e]] == idx[order[s]]:
            e += 1
        c = P[order[s]].copy()
        for j in order[s + 1:e]:
            c = (c + P[j]).astype(np.float32)
        out.append((c / np.float32(e - s)).astype(np.float32))
        s = e
    return np.array(out, np.float32)


def _tf_d(P, T):
    X = P[:, :3].astype(np.float64)
    Y = ((T[:3, 0] * X[:, :1] + T[:3, 1] * X[:, 1:2]) + T[:3, 2] * X[:, 2:3]) + T[:3, 3]
    return np.concatenate([Y.astype(np.float32), P[:, 3:4]], 1)


def icp_np(cur, T_cur, hist, T_hist, voxel=0.25, max_iter=100, eps=1e-6, fit_eps=1e-6, md=100.0):
    src = _voxel(_tf_d(cur, T_cur), voxel)
    tgt = _voxel(np.concatenate([_tf_d(h, T) for h, T in zip(hist, T_hist)]), voxel)
    tree = cKDTree(tgt[:, :3].astype(np.float64))
    S = src[:, :3].astype(np.float64)
    F = np.eye(4)
    prev, it, state = np.finfo(np.float64).max, 0, 0
    while True:
        d, j = tree.query(S)
        ok = d * d <= md * md
        a, b = S[ok], tgt[j[ok], :3].astype(np.float64)
        ms, mt = a.mean(0), b.mean(0)
        U, _, Vt = np.linalg.svd((b - mt).T @ (a - ms) / len(a))
        D = np.eye(3)
        if np.linalg.det(U) * np.linalg.det(Vt) < 0:
            D[2, 2] = -1
        R = U @ D @ Vt
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = R, mt - R @ ms
        S = S @ R.T + T[:3, 3]
        F = T @ F
        it += 1
        mse = float(np.mean(d[ok] ** 2))
        if it >= max_iter:
            state = 1
        elif 0.5 * (np.trace(R) - 1) >= 1 - eps and T[:3, 3] @ T[:3, 3] <= eps:
            state = 2
        elif abs(mse - prev) < 1e-12:
            state = 3
        elif abs(mse - prev) / prev < fit_eps:
            state = 4
        prev = mse
        if state:
            break
    X = src[:, :3].astype(np.float64) @ F[:3, :3].T + F[:3, 3]
    d, _ = tree.query(X)
    return F, float(np.mean(d * d)), state, it, len(src), len(tgt)


def test_icp_oracle_matches_numpy_corridor(oracle, synth):
    cur, Tc, hs, Th, T_true = corridor_loop(synth, n_scans=32, width=512)
    Ti, Tc2m, fit, info = oracle.loop_icp(cur, Tc, hs, Th)
    F, fnp, state, it, ns, nt = icp_np(cur, Tc, hs, Th)
    assert (info[4], info[5]) == (ns, nt)
    assert info[1] == 1 and info[2] == state
    assert abs(info[3] - it) <= 1
    assert np.max(np.abs(Ti - F)) < 1e-4
    assert abs(fit - fnp) < 1e-4 * max(1.0, fnp)
    assert np.allclose(Tc2m, Ti @ Tc, atol=1e-12)


def test_icp_oracle_recovers_known_transform(oracle):
    rng = np.random.default_rng(3)
    room = random_room(rng)
    D = drift(0.15, -0.1, 0.03, 3.0, 1.0)
    cur = _tf_d(room, np.linalg.inv(D))  # the room seen from the drifted pose
    cfg = oracle.IcpConfig(use_downsample=False)
    Ti, Tc2m, fit, info = oracle.loop_icp(cur, np.eye(4), [room], [np.eye(4)], cfg)
    assert info[0] == 1 and info[1] == 1
    assert np.max(np.abs(Ti - D)) < 1e-3
    assert fit < 1e-4


def test_icp_oracle_horn_equals_svd_single_step(oracle):
    """One iteration on exact correspondences: Horn's quaternion (Jacobi) == SVD Umeyama."""
    rng = np.random.default_rng(7)
    room = random_room(rng, 1500)
    D = drift(0.02, 0.01, -0.01, 0.5, 0.2)
    cur = _tf_d(room, np.linalg.inv(D))
    cfg = oracle.IcpConfig(use_downsample=False, max_iterations=1)
    Ti, _, _, info = oracle.loop_icp(cur, np.eye(4), [room], [np.eye(4)], cfg)
    assert info[2] == 1 and info[3] == 1
    tree = cKDTree(room[:, :3].astype(np.float64))
    S = cur[:, :3].astype(np.float64)
    _, j = tree.query(S)
    a, b = S, room[j, :3].astype(np.float64)
    ms, mt = a.mean(0), b.mean(0)
    U, _, Vt = np.linalg.svd((b - mt).T @ (a - ms))
    R = U @ Vt
    assert np.max(np.abs(Ti[:3, :3] - R)) < 1e-6
    assert np.max(np.abs(Ti[:3, 3] - (mt - R @ ms))) < 1e-5


def test_icp_oracle_edge_cases(oracle, synth):
    cur = synth.make_scan(5, 16, 256).reshape(-1, 4)
    _, _, fit, info = oracle.loop_icp(cur, np.eye(4), [], [])
    assert info[0] == -1 and fit == np.finfo(np.float64).max
    tiny = np.zeros((5, 4), np.float32)
    _, _, _, info = oracle.loop_icp(tiny, np.eye(4), [cur], [np.eye(4)])
    assert info[0] == -2
    # crop box: everything beyond 2 m dropped before the voxel grid
    cfg = oracle.IcpConfig(use_crop=True, crop_size=2.0)
    _, _, _, info = oracle.loop_icp(cur, np.eye(4), [cur], [np.eye(4)], cfg)
    P = cur[np.all(np.abs(cur[:, :3]) <= 2.0, axis=1)]
    assert info[4] == len(_voxel(P, 0.25))
    # NaN points are removed
    nan = cur.copy()
    nan[::7, 0] = np.nan
    _, _, _, info2 = oracle.loop_icp(nan, np.eye(4), [cur], [np.eye(4)])
    assert info2[4] == len(_voxel(nan[np.isfinite(nan[:, 0])], 0.25))


# ------------------------------------------------------------------ odometry fusion
def _mat(p):
    x, y, z, w = p[:4]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, p[4:]
    return T


def random_poses(rng, n):
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return np.concatenate([q, rng.normal(scale=5, size=(n, 3))], 1)


def fuse_np(aloam, inten, skip):
    out, cur, pa, pi = [], None, None, None
    for a, b, s in zip(aloam, inten, skip):
        A, I = _mat(a), _mat(b)
        if cur is None:
            cur = I
        else:
            cur = cur @ (np.linalg.inv(pa) @ A if s else np.linalg.inv(pi) @ I)
        pa, pi = A, I
        R = cur[:3, :3]
        out.append(np.concatenate([_quat(R), cur[:3, 3]]))
    return np.array(out)


def _quat(R):
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0)
        return np.array([(R[2, 1] - R[1, 2]) * 0.5 / s, (R[0, 2] - R[2, 0]) * 0.5 / s, (R[1, 0] - R[0, 1]) * 0.5 / s, 0.5 * s])
    i = int(np.argmax(np.diag(R)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = math.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
    q = np.zeros(4)
    q[i] = 0.5 * s
    q[3] = (R[k, j] - R[j, k]) * 0.5 / s
    q[j] = (R[j, i] + R[i, j]) * 0.5 / s
    q[k] = (R[k, i] + R[i, k]) * 0.5 / s
    return q


def test_fusion_oracle_matches_numpy(oracle):
    rng = np.random.default_rng(11)
    a, b = random_poses(rng, 40), random_poses(rng, 40)
    skip = (rng.random(40) < 0.3).astype(np.int32)
    f = oracle.OdomFuser()
    got = np.concatenate([f.step(a[:15], b[:15], skip[:15]), f.step(a[15:], b[15:], skip[15:])])
    assert np.max(np.abs(got - fuse_np(a, b, skip))) < 1e-9


def test_fusion_oracle_semantics(oracle):
    """No skips: the fused pose follows the intensity odometry; all skips after the first pair:
    the A-LOAM increments are chained onto the first intensity pose."""
    rng = np.random.default_rng(12)
    a, b = random_poses(rng, 10), random_poses(rng, 10)
    got = oracle.OdomFuser().step(a, b, np.zeros(10, np.int32))
    for k in range(10):
        assert np.allclose(_mat(got[k]), _mat(b[k]), atol=1e-9)
    got = oracle.OdomFuser().step(a, b, np.ones(10, np.int32))
    for k in range(10):
        assert np.allclose(_mat(got[k]), _mat(b[0]) @ np.linalg.inv(_mat(a[0])) @ _mat(a[k]), atol=1e-9)
