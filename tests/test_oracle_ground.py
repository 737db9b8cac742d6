"""CPU pins of the ground-plane oracle (oracle/oracle_ground.cpp, ImageHandler::groundPlaneExtraction
image_handler.h_ouster:41-100) against an independent numpy transcription of the same PCL 1.10
single-thread SACSegmentation steps: mt19937(12345) >> 1 samples, drawIndexSample's partial
Fisher-Yates, the collinearity test, SSE-order float reductions, adaptive RANSAC k, sequential
float covariance, pcl::eigen33 and the double-precision ground test.  (PCL is absent: parity
unpinned against it.)  No GPU."""
import math

import numpy as np
import pytest

f32 = np.float32


def _sum4(e0, e1, e2, e3):
    return f32(f32(e0 + e2) + f32(e1 + e3))


def _sum3(e0, e1, e2):
    return f32(e0 + f32(e1 + e2))


def _plane(p0, p1, p2):
    a = [f32(p1[k] - p0[k]) for k in range(3)]
    b = [f32(p2[k] - p0[k]) for k in range(3)]
    c = [f32(a[1] * b[2] - a[2] * b[1]), f32(a[2] * b[0] - a[0] * b[2]), f32(a[0] * b[1] - a[1] * b[0]), f32(0)]
    z = _sum4(c[0] * c[0], c[1] * c[1], c[2] * c[2], c[3] * c[3])
    if z > 0:
        s = f32(np.sqrt(z))
        c = [f32(v / s) for v in c]
    c[3] = f32(-_sum4(c[0] * p0[0], c[1] * p0[1], c[2] * p0[2], c[3] * f32(1)))
    return c


def _dist(c, P):
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    return np.abs(((c[0] * x) + (c[2] * z)) + ((c[1] * y) + (c[3] * f32(1))))


def _roots2(b, c):
    d = f32(float(f32(b * b)) - 4.0 * float(c))
    if d < 0.0:
        d = f32(0)
    sd = f32(np.sqrt(d))
    return [f32(0), f32(f32(0.5) * f32(b - sd)), f32(f32(0.5) * f32(b + sd))]


def _roots(m):
    m00, m01, m02, m11, m12, m22 = m[0], m[1], m[2], m[4], m[5], m[8]
    c0 = f32(f32(f32(f32(f32(m00 * m11) * m22) + f32(f32(f32(f32(2) * m01) * m02) * m12)) - f32(f32(m00 * m12) * m12))
             - f32(f32(m11 * m02) * m02))
    c0 = f32(c0 - f32(f32(m22 * m01) * m01))
    c1 = f32(f32(f32(f32(f32(m00 * m11) - f32(m01 * m01)) + f32(m00 * m22)) - f32(m02 * m02)) + f32(m11 * m22))
    c1 = f32(c1 - f32(m12 * m12))
    c2 = f32(f32(m00 + m11) + m22)
    if abs(c0) < np.finfo(np.float32).eps:
        return _roots2(c2, c1)
    inv3, sq3 = f32(1.0 / 3.0), f32(np.sqrt(f32(3)))
    c2o3 = f32(c2 * inv3)
    a3 = f32(f32(c1 - f32(c2 * c2o3)) * inv3)
    a3 = min(a3, f32(0))
    hb = f32(f32(0.5) * f32(c0 + f32(c2o3 * f32(f32(f32(f32(2) * c2o3) * c2o3) - c1))))
    q = f32(f32(hb * hb) + f32(f32(a3 * a3) * a3))
    q = min(q, f32(0))
    rho = f32(np.sqrt(-a3))
    th = f32(f32(math.atan2(float(f32(np.sqrt(-q))), float(hb))) * inv3)
    ct, st = f32(math.cos(float(th))), f32(math.sin(float(th)))
    r = [f32(c2o3 + f32(f32(f32(2) * rho) * ct)), f32(c2o3 - f32(rho * f32(ct + f32(sq3 * st)))),
         f32(c2o3 - f32(rho * f32(ct - f32(sq3 * st))))]
    if r[0] >= r[1]:
        r[0], r[1] = r[1], r[0]
    if r[1] >= r[2]:
        r[1], r[2] = r[2], r[1]
        if r[0] >= r[1]:
            r[0], r[1] = r[1], r[0]
    if r[0] <= 0:
        r = _roots2(c2, c1)
    return r


def _eigen33_min(mat):
    scale = max(abs(v) for v in mat)
    if scale <= np.finfo(np.float32).tiny:
        scale = f32(1)
    m = [f32(v / scale) for v in mat]
    r = _roots(m)
    for k in (0, 4, 8):
        m[k] = f32(m[k] - r[0])

    def cross(i, j):
        a, b = m[3 * i:3 * i + 3], m[3 * j:3 * j + 3]
        return [f32(a[1] * b[2] - a[2] * b[1]), f32(a[2] * b[0] - a[0] * b[2]), f32(a[0] * b[1] - a[1] * b[0])]

    vs = [cross(0, 1), cross(0, 2), cross(1, 2)]
    ls = [_sum3(v[0] * v[0], v[1] * v[1], v[2] * v[2]) for v in vs]
    if ls[0] >= ls[1] and ls[0] >= ls[2]:
        i = 0
    elif ls[1] >= ls[0] and ls[1] >= ls[2]:
        i = 1
    else:
        i = 2
    s = f32(np.sqrt(ls[i]))
    return [f32(v / s) for v in vs[i]]


def ground_np(P):
    """numpy transcription of the oracle's steps (see the module docstring)."""
    P = P.reshape(-1, 4).astype(np.float32)
    z = P[:, 2]
    C = P[(z.astype(np.float64) >= -2.0) & (z.astype(np.float64) <= -0.45), :3]
    n = C.shape[0]
    info = [-1, 0, 0, 0]
    if n < 3:
        return np.zeros((0, 4), np.float32), None, info
    bg = np.random.MT19937(0)
    bg._legacy_seeding(12345)
    raw = iter(bg.random_raw(200000))
    sh = np.arange(n)
    it, best, k, model = 0, -(2**31 - 1), 1.0, None
    logp = math.log(1.0 - 0.99)
    while it < k:
        got = False
        for _ in range(1000):
            for i in range(3):
                j = i + (int(next(raw)) >> 1) % (n - i)
                sh[i], sh[j] = sh[j], sh[i]
            p0, p1, p2 = C[sh[0]], C[sh[1]], C[sh[2]]
            with np.errstate(divide="ignore", invalid="ignore"):
                d = [f32(f32(p1[k_] - p0[k_]) / f32(p2[k_] - p0[k_])) for k_ in range(3)]
            got = bool((d[0] != d[1]) or (d[2] != d[1]))
            if got:
                break
        if not got:
            break
        c = _plane(p0, p1, p2)
        cnt = int((_dist(c, C) < 0.01).sum())
        if cnt > best:
            best, model = cnt, c
            w = best / n
            pno = min(max(1.0 - math.pow(w, 3.0), np.finfo(np.float64).eps), 1.0 - np.finfo(np.float64).eps)
            k = logp / math.log(pno)
        it += 1
        if it > 50:
            break
    info[1] = it
    if model is None:
        info[0] = -2
        return np.zeros((0, 4), np.float32), None, info
    info[2] = best
    inl = C[_dist(model, C) < 0.01]
    info[3] = inl.shape[0]
    coef = list(model)
    if inl.shape[0] > 3:
        x, y, zz = inl[:, 0], inl[:, 1], inl[:, 2]
        terms = [x * x, x * y, x * zz, y * y, y * zz, zz * zz, x, y, zz]
        acc = [f32(np.cumsum(t, dtype=np.float32)[-1] / f32(inl.shape[0])) for t in terms]
        cov = [f32(acc[0] - acc[6] * acc[6]), f32(acc[1] - acc[6] * acc[7]), f32(acc[2] - acc[6] * acc[8]), 0,
               f32(acc[3] - acc[7] * acc[7]), f32(acc[4] - acc[7] * acc[8]), 0, 0, f32(acc[5] - acc[8] * acc[8])]
        cov[3], cov[6], cov[7] = cov[1], cov[2], cov[5]
        ev = _eigen33_min(cov)
        coef = [ev[0], ev[1], ev[2], f32(0)]
        coef[3] = f32(-_sum4(coef[0] * acc[6], coef[1] * acc[7], coef[2] * acc[8], coef[3] * f32(1)))
    nz = _sum3(coef[0] * f32(0), coef[1] * f32(0), coef[2] * f32(1))
    if not float(nz) > math.cos(15 * math.pi / 180):
        info[0] = 0
        return np.zeros((0, 4), np.float32), np.array(coef, np.float32), info
    info[0] = 1
    A, B, Cc, D = (float(v) for v in coef)
    X = P[:, :3].astype(np.float64)
    h = np.abs(((A * X[:, 0] + B * X[:, 1]) + Cc * X[:, 2]) + D) / math.sqrt((A * A + B * B) + Cc * Cc)
    keep = (h <= 0.03) & (P[:, 2] < 0)
    g = np.concatenate([P[keep, :3], np.ones((int(keep.sum()), 1), np.float32)], 1)
    return g, np.array(coef, np.float32), info


@pytest.mark.parametrize("k", [0, 3, 11])
def test_ground_oracle_matches_numpy(oracle, synth, k):
    scan = synth.make_scan(k, 32, 512)
    g, plane, info = oracle.ground_extract(scan)
    gn, pn, infon = ground_np(scan)
    assert list(info) == infon
    assert info[0] == 1 and g.shape[0] > 1000  # the corridor floor
    assert np.array_equal(plane, pn)
    assert np.array_equal(g, gn)


def test_ground_oracle_edge_cases(oracle, synth):
    # no candidates in the z band
    g, plane, info = oracle.ground_extract(np.zeros((16, 64, 4), np.float32))
    assert info[0] == -1 and g.shape[0] == 0
    # a tilted plane: rejected by the orientation test (n . z <= cos 15 deg)
    rng = np.random.default_rng(1)
    xy = rng.uniform(-5, 5, size=(4000, 2)).astype(np.float32)
    z = (-1.0 + 0.5 * xy[:, 0]).astype(np.float32)  # 26.6 deg slope
    P = np.stack([xy[:, 0], xy[:, 1], z, np.zeros_like(z)], 1)
    g, plane, info = oracle.ground_extract(P)
    gn, pn, infon = ground_np(P)
    assert list(info) == infon and info[0] in (0, 1)
    assert np.array_equal(plane, pn) and np.array_equal(g, gn)
    if info[0] == 0:
        assert g.shape[0] == 0
