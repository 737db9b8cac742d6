"""Host-side mirror of the reference's scan-to-map interfaces over the lislam C ABI.

``IkdMap`` plays the vendored ``KD_TREE`` (``src/ikd-Tree/ikd_Tree.h:256-279``: ``Build``,
``Add_Points``, ``Nearest_Search``, ``size``, ``flatten``) on a device-resident map;
``MapOptimization.callback`` plays the ground-map stage of
``mapOptimization::mapOptimizationCallback`` (``src/mapOptimization.cpp:99-479``);
``laser_mapping`` plays the optimization of ``laserMapping::process``
(``src/laserMapping.cpp:620-850``).  All compute runs in ``liblislam.so`` on the GPU; inputs may
be numpy arrays (host) or any object exposing a device pointer via ``data_ptr()`` (torch CUDA
tensors), which the library reads in place.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native as nat


def _as_points(points):
    """(pointer, n, stride, keepalive) of a float32 (n, 3|4) host array or device tensor."""
    if hasattr(points, "data_ptr"):  # torch tensor (host or device), float32, contiguous
        t = points.contiguous()
        if str(t.dtype) != "torch.float32" or t.dim() != 2 or t.shape[1] < 3:
            raise ValueError("points must be a float32 (n, 3|4) tensor")
        return ctypes.c_void_p(t.data_ptr()), t.shape[0], t.shape[1], t
    a = np.ascontiguousarray(points, np.float32)
    if a.ndim != 2 or (a.shape[1] < 3 and a.shape[0] > 0):
        raise ValueError("points must be (n, 3|4)")
    return ctypes.c_void_p(a.ctypes.data), a.shape[0], a.shape[1], a


class IkdMap:
    """Device-resident ikd-Tree point set (lislam_map)."""

    def __init__(self, ctx, downsample_size: float = 0.2, cell_size: float = 0.0):
        self.ctx = ctx
        h = ctypes.c_void_p()
        cfg = nat.MapConfig(downsample_size, cell_size)
        nat.check(ctx.lib.lislam_map_create(ctx.h, ctypes.byref(cfg), ctypes.byref(h)), ctx.h, "lislam_map_create")
        self.h = h

    def close(self):
        if self.h:
            self.ctx.lib.lislam_map_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build(self, points):
        """KD_TREE::Build."""
        p, n, s, _k = _as_points(points)
        nat.check(self.ctx.lib.lislam_map_build(self.h, p, n, s), self.ctx.h, "lislam_map_build")

    def add_points(self, points, downsample_on: bool = True) -> int:
        """KD_TREE::Add_Points; returns the number of inputs that entered the map."""
        p, n, s, _k = _as_points(points)
        added = ctypes.c_int64()
        nat.check(self.ctx.lib.lislam_map_add_points(self.h, p, n, s, int(downsample_on), ctypes.byref(added)),
                  self.ctx.h, "lislam_map_add_points")
        return added.value

    def size(self) -> int:
        n = ctypes.c_int64()
        nat.check(self.ctx.lib.lislam_map_size(self.h, ctypes.byref(n)), self.ctx.h, "lislam_map_size")
        return n.value

    def points(self) -> np.ndarray:
        """KD_TREE::flatten: live points (n, 4) = x, y, z, id bits (storage order)."""
        n = self.size()
        out = np.zeros((max(n, 1), 4), np.float32)
        got = ctypes.c_int64()
        nat.check(self.ctx.lib.lislam_map_points(self.h, nat.ptr(out), out.shape[0], ctypes.byref(got)), self.ctx.h,
                  "lislam_map_points")
        return out[: got.value]

    def nearest_search(self, queries, k: int = 5, max_dist: float = 0.0):
        """Batched KD_TREE::Nearest_Search: (points (n, k, 4), d2 (n, k), found (n,))."""
        p, n, s, _k = _as_points(queries)
        pts = np.zeros((n, k, 4), np.float32)
        d2 = np.zeros((n, k), np.float32)
        found = np.zeros(n, np.int32)
        nat.check(self.ctx.lib.lislam_map_nearest_search(self.h, p, n, s, k, max_dist, nat.ptr(pts), nat.ptr(d2),
                                                         nat.ptr(found)), self.ctx.h, "lislam_map_nearest_search")
        return pts, d2, found

    def associate(self, match: int, points, x):
        """Line (0) / plane (1) association at pose x: (records (n, 9), kinds (n,))."""
        p, n, s, _k = _as_points(points)
        rec = np.zeros((n, 9))
        kind = np.zeros(n, np.int32)
        xx = np.ascontiguousarray(x, np.float64)
        nat.check(self.ctx.lib.lislam_map_associate(self.h, match, p, n, s, nat.ptr(xx), nat.ptr(rec), nat.ptr(kind)),
                  self.ctx.h, "lislam_map_associate")
        return rec, kind


def normal_equations(ctx, records, kinds, x) -> np.ndarray:
    """cost, J^T J (21), J^T r (6) of residual-block records at x (28 doubles)."""
    rec = np.ascontiguousarray(records, np.float64).reshape(-1, 9)
    kd = np.ascontiguousarray(kinds, np.int32)
    out = np.zeros(28)
    xx = np.ascontiguousarray(x, np.float64)
    nat.check(ctx.lib.lislam_normal_equations(ctx.h, nat.ptr(rec), nat.ptr(kd), rec.shape[0], nat.ptr(xx), nat.ptr(out)),
              ctx.h, "lislam_normal_equations")
    return out


def pose_solve(ctx, records, kinds, x0, max_iterations: int):
    """ceres::Solve of the records: (x (7,), summary (iterations, termination, edges, planes))."""
    rec = np.ascontiguousarray(records, np.float64).reshape(-1, 9)
    kd = np.ascontiguousarray(kinds, np.int32)
    x = np.array(x0, np.float64)
    summ = np.zeros(4, np.int32)
    nat.check(ctx.lib.lislam_pose_solve(ctx.h, nat.ptr(rec), nat.ptr(kd), rec.shape[0], nat.ptr(x), max_iterations,
                                        nat.ptr(summ)), ctx.h, "lislam_pose_solve")
    return x, summ


def voxel_grid(ctx, points, leaf: float) -> np.ndarray:
    """pcl::VoxelGrid of (n, 4) float32 points (x, y, z, intensity)."""
    a = np.ascontiguousarray(points, np.float32).reshape(-1, 4)
    out = np.zeros((max(a.shape[0], 1), 4), np.float32)
    n = ctypes.c_int32()
    nat.check(ctx.lib.lislam_voxel_grid(ctx.h, nat.ptr(a), a.shape[0], leaf, nat.ptr(out), ctypes.byref(n)), ctx.h,
              "lislam_voxel_grid")
    return out[: n.value]


class MapOptimization:
    """Ground-map stage of the mapOptimization node (ikd-Tree map of downsample 0.4,
    mapOptimization.cpp:504) and, with corner=True, its corner ikd-Tree (downsample 0.8,
    :505), which takes pc_corner at the same keyframe pose (:193-195, :477-479)."""

    def __init__(self, ctx, downsample_size: float = 0.4, cell_size: float = 0.0, corner: bool = False,
                 corner_downsample: float = 0.8):
        self.map = IkdMap(ctx, downsample_size, cell_size)
        self.corner_map = IkdMap(ctx, corner_downsample, cell_size) if corner else None
        self.state = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)  # q_wmap_wodom, t_wmap_wodom

    def callback(self, ground, odom, pc_corner=None):
        """One frame: ground = GroundPointOut (sensor frame, (n, 4)), odom = q_wodom_curr, t_wodom_curr,
        pc_corner = the corner cloud (sensor frame, (m, 4); with corner=True).
        Returns (q_w_curr, t_w_curr (7,), summary (planes, iterations, termination; -1 = built))."""
        g = np.ascontiguousarray(ground, np.float32).reshape(-1, 4)
        od = np.ascontiguousarray(odom, np.float64)
        pose = np.zeros(7)
        summ = np.zeros(3, np.int32)
        ctx = self.map.ctx
        if self.corner_map is None:
            nat.check(ctx.lib.lislam_mapopt_step(self.map.h, nat.ptr(g), g.shape[0], nat.ptr(od), nat.ptr(self.state),
                                                 nat.ptr(pose), nat.ptr(summ)), ctx.h, "lislam_mapopt_step")
            return pose, summ
        c = np.ascontiguousarray(pc_corner if pc_corner is not None else np.zeros((0, 4)), np.float32).reshape(-1, 4)
        nat.check(ctx.lib.lislam_mapopt_step_corner(self.map.h, self.corner_map.h, nat.ptr(g), g.shape[0], nat.ptr(c),
                                                    c.shape[0], nat.ptr(od), nat.ptr(self.state), nat.ptr(pose),
                                                    nat.ptr(summ)), ctx.h, "lislam_mapopt_step_corner")
        return pose, summ

    def laser_odometry_handler(self, odom) -> np.ndarray:
        """laserOdometryHandler (mapOptimization.cpp:19-49): the high-frequency pose
        q_w_curr = q_wmap_wodom * q_wodom_curr, t_w_curr = q_wmap_wodom * t_wodom_curr + t_wmap_wodom
        from the latest map correction (13 flops of ROS glue, computed on the host)."""
        qm, tm = self.state[:4], self.state[4:]
        qo, to = np.asarray(odom[:4], np.float64), np.asarray(odom[4:7], np.float64)

        def qmul(a, b):
            ax, ay, az, aw = a
            bx, by, bz, bw = b
            return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                             aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])

        qw = qmul(qm, qo)
        tq = qmul(qmul(qm, np.array([to[0], to[1], to[2], 0.0])), qm * np.array([-1, -1, -1, 1.0]))[:3]
        return np.concatenate([qw, tq + tm])

    def callback_batch(self, batch, scan: int, odom):
        """The same frame fed from a batch on the device: GroundPointOut of `scan` (batch.ground
        first) + its less-flat cloud, as mapOptimizationCallback assembles them (:136-150); with
        corner=True the scan's less-sharp cloud is pc_corner (mapOptimizationNode.cpp:63)."""
        od = np.ascontiguousarray(odom, np.float64)
        pose = np.zeros(7)
        summ = np.zeros(3, np.int32)
        ctx = self.map.ctx
        cm = self.corner_map.h if self.corner_map is not None else None
        nat.check(ctx.lib.lislam_batch_mapopt_corner(batch.h, self.map.h, cm, scan, nat.ptr(od), nat.ptr(self.state),
                                                     nat.ptr(pose), nat.ptr(summ)), ctx.h, "lislam_batch_mapopt_corner")
        return pose, summ

    def close(self):
        self.map.close()
        if self.corner_map is not None:
            self.corner_map.close()


def laser_mapping(corner_map: IkdMap, surf_map: IkdMap, corner, surf, x0):
    """laserMapping optimization: (x (7,), stats (corner / surf blocks of the two passes)).
    corner / surf: (n, 4) float32 host arrays or device tensors (read in place)."""
    cp, nc, cs, _kc = _as_points(corner if len(corner) else np.zeros((0, 4), np.float32))
    sp, ns, ss, _ks = _as_points(surf if len(surf) else np.zeros((0, 4), np.float32))
    if (nc and cs != 4) or (ns and ss != 4):
        raise ValueError("laser_mapping expects (n, 4) point arrays")
    x = np.array(x0, np.float64)
    st = np.zeros(4, np.int32)
    ctx = corner_map.ctx
    nat.check(ctx.lib.lislam_laser_mapping(corner_map.h, surf_map.h, cp, nc, sp, ns, nat.ptr(x), nat.ptr(st)), ctx.h,
              "lislam_laser_mapping")
    return x, st

def set_timing(ctx, on: bool):
    nat.check(ctx.lib.lislam_map_set_timing(ctx.h, int(on)), ctx.h, "lislam_map_set_timing")


def kernel_times(ctx):
    """{kernel: (total ms, launches)} of the mapping kernels since the previous read."""
    ms = np.zeros(len(nat.MAP_KERNELS), np.float32)
    n = np.zeros(len(nat.MAP_KERNELS), np.int32)
    nat.check(ctx.lib.lislam_map_kernel_times(ctx.h, ms.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                              n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), ctx.h,
              "lislam_map_kernel_times")
    return {k: (float(a), int(b)) for k, a, b in zip(nat.MAP_KERNELS, ms, n)}


class LaserMapping:
    """laserMapping::process over its 21 x 21 x 11 cube map (laserMapping.cpp:319-1002), device
    resident (lislam_lmap)."""

    NC = 21 * 21 * 11

    def __init__(self, ctx, line_res: float = 0.4, plane_res: float = 0.8):
        self.ctx = ctx
        h = ctypes.c_void_p()
        nat.check(ctx.lib.lislam_lmap_create(ctx.h, line_res, plane_res, ctypes.byref(h)), ctx.h, "lislam_lmap_create")
        self.h = h
        self.state = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)  # q_wmap_wodom, t_wmap_wodom

    def close(self):
        if self.h:
            self.ctx.lib.lislam_lmap_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, corner_last, surf_last, odom):
        """One frame: (q_w_curr t_w_curr (7,), stats (8,) = corner / surf map sizes, stack sizes,
        optimization stats or -1)."""
        pc, nc, _, kc = _as_points(corner_last)
        ps, ns, _, ks = _as_points(surf_last)
        od = np.ascontiguousarray(odom, np.float64)
        pose = np.zeros(7, np.float64)
        stats = np.zeros(8, np.int32)
        nat.check(self.ctx.lib.lislam_lmap_step(self.h, pc, nc, ps, ns, nat.ptr(od), nat.ptr(self.state), nat.ptr(pose),
                                                nat.ptr(stats)), self.ctx.h, "lislam_lmap_step")
        return pose, stats

    def counts(self):
        cc = np.zeros(self.NC, np.int32)
        sc = np.zeros(self.NC, np.int32)
        nat.check(self.ctx.lib.lislam_lmap_counts(self.h, nat.ptr(cc), nat.ptr(sc)), self.ctx.h, "lislam_lmap_counts")
        return cc, sc

    def points(self, which: int) -> np.ndarray:
        n = ctypes.c_int64()
        nat.check(self.ctx.lib.lislam_lmap_points(self.h, which, None, 0, ctypes.byref(n)), self.ctx.h, "lislam_lmap_points")
        out = np.zeros((max(n.value, 1), 4), np.float32)
        nat.check(self.ctx.lib.lislam_lmap_points(self.h, which, nat.ptr(out), n.value, ctypes.byref(n)), self.ctx.h,
                  "lislam_lmap_points")
        return out[: n.value]
