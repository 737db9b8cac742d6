"""Second, independent restatement (numpy / pure Python) of the reference front end, used to pin
the C++ oracle.  Test infrastructure only.

Vectorized numpy for a1..a5 (scanRegistration.cpp:152-412, image_handler.h_ouster:103-140) with
explicit float32 / float64 typing of every reference expression; pure-Python loops for the
greedy selection a6 and the VoxelGrid a7 (small scans only).
"""
from __future__ import annotations

import math

import numpy as np

f32, f64 = np.float32, np.float64
PI = math.pi


def atan2_f(y, x):
    return np.arctan2(y.astype(f64), x.astype(f64)).astype(f32)


def atan_f(v):
    return np.arctan(v.astype(f64)).astype(f32)


def cloud_handler(scan):
    p = scan.reshape(-1, 4)
    x, y, z, i = p[:, 0], p[:, 1], p[:, 2], p[:, 3]
    rng = np.sqrt(x * x + y * y + z * z)  # float32 throughout
    inten = np.minimum(i, f32(255.0))
    img_range = np.minimum(rng * f32(20), f32(255.0)).astype(np.uint8)
    img_int = inten.astype(np.uint8)
    keep = rng.astype(f64) >= 0.1
    track = np.where(keep[:, None], np.stack([x, y, z, inten], 1), f32(0)).astype(f32)
    return img_range, img_int, track


def scan_id(angle, n_scans):
    a = angle.astype(f64)
    if n_scans == 16:
        sid = (((angle + f32(15)) / f32(2)).astype(f64) + 0.5).astype(np.int64)  # float (angle+15)/2
    elif n_scans == 32:
        sid = ((a + 92.0 / 3.0) * 3.0 / 4.0).astype(np.int64)
    elif n_scans == 64:
        sid = ((a + 22.5) * 1.41 + 0.5).astype(np.int64) - 1
    else:
        sid = ((a + 22.5) * 2.83 + 0.5).astype(np.int64) - 1
    return np.where((sid > n_scans - 1) | (sid < 0), -1, sid)


def laser_cloud(scan, n_scans, min_range=0.3):
    """a2..a4: filtered, scan-grouped cloud with intensity = scanID + 0.1 relTime; line offsets."""
    p = scan.reshape(-1, 4).astype(f32)
    thr = f32(min_range)
    d2 = p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1] + p[:, 2] * p[:, 2]
    p = p[~(d2 < thr * thr)]
    if p.shape[0] == 0:
        return np.zeros((0, 4), f32), np.zeros(n_scans + 1, np.int64)
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    startOri = -atan2_f(y[:1], x[:1])[0]
    endOri = f32(f64(-atan2_f(y[-1:], x[-1:])[0]) + 2 * PI)
    if f64(endOri - startOri) > 3 * PI:
        endOri = f32(f64(endOri) - 2 * PI)
    elif f64(endOri - startOri) < PI:
        endOri = f32(f64(endOri) + 2 * PI)
    angle = ((atan_f(z / np.sqrt(x * x + y * y)) * f32(180)).astype(f64) / PI).astype(f32)
    sid = scan_id(angle, n_scans)
    ok = sid >= 0
    p, sid = p[ok], sid[ok]
    x, y = p[:, 0], p[:, 1]
    ori = -atan2_f(y, x)
    # before halfPassed
    o1 = ori.astype(f64)
    np_ori = np.where(o1 < f64(startOri) - PI / 2, (o1 + 2 * PI).astype(f32),
                      np.where(o1 > f64(startOri) + PI * 3 / 2, (o1 - 2 * PI).astype(f32), ori))
    cond = (np_ori - startOri).astype(f64) > PI
    flip = int(np.argmax(cond)) if cond.any() else p.shape[0]
    o2 = (o1 + 2 * PI).astype(f32).astype(f64)
    pa_ori = np.where(o2 < f64(endOri) - PI * 3 / 2, (o2 + 2 * PI).astype(f32),
                      np.where(o2 > f64(endOri) + PI / 2, (o2 - 2 * PI).astype(f32), o2.astype(f32)))
    idx = np.arange(p.shape[0])
    fo = np.where(idx <= flip, np_ori, pa_ori).astype(f32)
    rel = ((fo - startOri) / (endOri - startOri)).astype(f32)
    inten = (sid.astype(f64) + 0.1 * rel.astype(f64)).astype(f32)
    p = p.copy()
    p[:, 3] = inten
    order = np.argsort(sid, kind="stable")
    counts = np.bincount(sid, minlength=n_scans)
    off = np.concatenate([[0], np.cumsum(counts)])
    return p[order], off


def curvature(cloud):
    n = cloud.shape[0]
    c = np.zeros(n, f32)
    if n < 11:
        return c
    out = []
    for d in range(3):
        v = cloud[:, d]
        s = v[0:n - 10].copy()
        for k in range(1, 5):
            s = s + v[k:n - 10 + k]
        s = s - f32(10) * v[5:n - 5]
        for k in range(6, 11):
            s = s + v[k:n - 10 + k]
        out.append(s)
    dX, dY, dZ = out
    c[5:n - 5] = dX * dX + dY * dY + dZ * dZ
    return c


def voxel_grid(pts, leaf=0.2):
    """PCL VoxelGrid with ties in voxel index resolved by input order (pure Python sums)."""
    if len(pts) == 0:
        return np.zeros((0, 4), f32)
    pts = np.asarray(pts, f32)
    inv = f32(1.0) / f32(leaf)
    mn, mx = pts[:, :3].min(0), pts[:, :3].max(0)
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(pts[:, :3] * inv) - minb.astype(f32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    out = []
    a = 0
    while a < len(order):
        b = a + 1
        while b < len(order) and idx[order[b]] == idx[order[a]]:
            b += 1
        c = pts[order[a]].copy()
        for l in range(a + 1, b):
            c = (c + pts[order[l]]).astype(f32)
        out.append((c / f32(b - a)).astype(f32))
        a = b
    return np.array(out, f32)


def select_features(cloud, off, curv, n_scans):
    """a6/a7 as pure-Python loops (canonical (curvature, index) order)."""
    N = cloud.shape[0]
    picked = np.zeros(N, np.int8)
    label = np.zeros(N, np.int8)
    sharp, less_sharp, flat, less_flat = [], [], [], []

    def d2(a, b):
        d = cloud[a, :3] - cloud[b, :3]
        return f64(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])

    def suppress(ind):
        for l in range(1, 6):
            if d2(ind + l, ind + l - 1) > 0.05:
                break
            picked[ind + l] = 1
        for l in range(-1, -6, -1):
            if d2(ind + l, ind + l + 1) > 0.05:
                break
            picked[ind + l] = 1

    for i in range(n_scans):
        s, e = int(off[i]) + 5, int(off[i + 1]) - 6
        if e - s < 6:
            continue
        lf_scan = []
        for j in range(6):
            sp = s + (e - s) * j // 6
            ep = s + (e - s) * (j + 1) // 6 - 1
            inds = sorted(range(sp, ep + 1), key=lambda k: (curv[k], k))
            largest = 0
            for ind in reversed(inds):
                if picked[ind] == 0 and f64(curv[ind]) > 0.1:
                    largest += 1
                    if largest <= 2:
                        label[ind] = 2
                        sharp.append(cloud[ind])
                        less_sharp.append(cloud[ind])
                    elif largest <= 20:
                        label[ind] = 1
                        less_sharp.append(cloud[ind])
                    else:
                        break
                    picked[ind] = 1
                    suppress(ind)
            smallest = 0
            for ind in inds:
                if picked[ind] == 0 and f64(curv[ind]) < 0.1:
                    label[ind] = -1
                    flat.append(cloud[ind])
                    smallest += 1
                    if smallest >= 4:
                        break
                    picked[ind] = 1
                    suppress(ind)
            for k in range(sp, ep + 1):
                if label[k] <= 0:
                    lf_scan.append(cloud[k])
        vg = voxel_grid(lf_scan)
        if len(vg):
            less_flat.extend(list(vg))

    def arr(v):
        return np.array(v, f32).reshape(-1, 4)

    return arr(sharp), arr(less_sharp), arr(flat), arr(less_flat), label
