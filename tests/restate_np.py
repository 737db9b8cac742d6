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


def libstdcxx_sort(keys):
    """The permutation libstdc++'s std::sort applies to `keys` (pure Python, serial): the
    two-pointer introsort loop (median of first + 1 / mid / last - 1 moved to first,
    __unguarded_partition), heap sort below depth 2 floor(log2 n), then the final insertion sort
    (16-element head, unguarded tail).  An independent restatement of what the oracle gets from
    calling std::sort and the HIP kernels compute with prefix counts."""
    a = list(range(len(keys)))
    k = keys

    def lt(x, y):
        return k[x] < k[y]

    def adjust_heap(first, hole, n, v):
        top = hole
        child = hole
        while child < (n - 1) // 2:
            child = 2 * (child + 1)
            if lt(a[first + child], a[first + child - 1]):
                child -= 1
            a[first + hole] = a[first + child]
            hole = child
        if n % 2 == 0 and child == (n - 2) // 2:
            child = 2 * (child + 1)
            a[first + hole] = a[first + child - 1]
            hole = child - 1
        parent = (hole - 1) // 2
        while hole > top and lt(a[first + parent], v):
            a[first + hole] = a[first + parent]
            hole = parent
            parent = (hole - 1) // 2
        a[first + hole] = v

    def heap_sort(first, last):
        n = last - first
        if n >= 2:
            parent = (n - 2) // 2
            while True:
                adjust_heap(first, parent, n, a[first + parent])
                if parent == 0:
                    break
                parent -= 1
        while last - first > 1:
            last -= 1
            v = a[last]
            a[last] = a[first]
            adjust_heap(first, 0, last - first, v)

    def partition_pivot(first, last):
        mid = first + (last - first) // 2
        x, y, z = first + 1, mid, last - 1
        if lt(a[x], a[y]):
            m = y if lt(a[y], a[z]) else (z if lt(a[x], a[z]) else x)
        elif lt(a[x], a[z]):
            m = x
        elif lt(a[y], a[z]):
            m = z
        else:
            m = y
        a[first], a[m] = a[m], a[first]
        lo, hi, piv = first + 1, last, a[first]
        while True:
            while lt(a[lo], piv):
                lo += 1
            hi -= 1
            while lt(piv, a[hi]):
                hi -= 1
            if not lo < hi:
                return lo
            a[lo], a[hi] = a[hi], a[lo]
            lo += 1

    def loop(first, last, depth):
        while last - first > 16:
            if depth == 0:
                heap_sort(first, last)
                return
            depth -= 1
            cut = partition_pivot(first, last)
            loop(cut, last, depth)
            last = cut

    def linear_insert(i):
        v = a[i]
        j = i - 1
        while lt(v, a[j]):
            a[j + 1] = a[j]
            j -= 1
        a[j + 1] = v

    def insertion_sort(first, last):
        for i in range(first + 1, last):
            if lt(a[i], a[first]):
                v = a[i]
                a[first + 1:i + 1] = a[first:i]
                a[first] = v
            else:
                linear_insert(i)

    n = len(a)
    if n:
        loop(0, n, 2 * (n.bit_length() - 1))
        if n > 16:
            insertion_sort(0, 16)
            for i in range(16, n):
                linear_insert(i)
        else:
            insertion_sort(0, n)
    return a


def voxel_grid(pts, leaf=0.2, std_sort=True):
    """PCL VoxelGrid (pure Python sums): the (voxel, point) pairs sorted by voxel as std::sort
    leaves them (std_sort, the reference and the HIP path) or with ties in input order."""
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
    order = libstdcxx_sort([int(v) for v in idx]) if std_sort else np.argsort(idx, kind="stable")
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
    """a6/a7 as pure-Python loops: segment walks in (curvature, index) order, the VoxelGrid in
    std::sort's order (the oracle's TIES_GPU)."""
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
