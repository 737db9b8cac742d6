"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of ``liboracle.so`` (the C++ restatement in this directory).  Imported only by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``; the product
package never imports it.  See ``oracle_common.hpp`` for the parity status.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(path)
        L.oracle_scan_registration.argtypes = [
            _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
            _u8p, _u8p, _f32p, _f32p, _i32p, _i32p, _i32p, _f32p, _i8p,
            _f32p, _i32p, _f32p, _i32p, _f32p, _i32p, _f32p, _i32p]
        L.oracle_scan_registration.restype = ctypes.c_int
        L.oracle_voxel_grid.argtypes = [_f32p, ctypes.c_int, ctypes.c_float, ctypes.c_int, _f32p, _i32p]
        L.oracle_odometry_chain.argtypes = [
            ctypes.c_int, _f32p, _i32p, _f32p, _i32p, _f32p, _i32p, _f32p, _i32p, _f64p, _f64p, _i32p]
        L.oracle_odometry_chain_gated.argtypes = [
            ctypes.c_int, _f32p, _i32p, _f32p, _i32p, _f32p, _i32p, _f32p, _i32p, _i32p, _f64p, _f64p, _i32p]
        L.oracle_nn1.argtypes = [_f32p, ctypes.c_int, _f32p, ctypes.c_int, _i32p, _f32p]
        L.oracle_eval_factor.argtypes = [ctypes.c_int, _f64p, _f64p, _f64p, _f64p, _f64p]
        vp = ctypes.c_void_p
        L.oracle_map_create.argtypes = [ctypes.c_float]
        L.oracle_map_create.restype = vp
        L.oracle_map_destroy.argtypes = [vp]
        L.oracle_map_build.argtypes = [vp, _f32p, ctypes.c_int, ctypes.c_int]
        L.oracle_map_add_points.argtypes = [vp, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_map_size.argtypes = [vp]
        L.oracle_map_points.argtypes = [vp, _f32p]
        L.oracle_map_knn.argtypes = [vp, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, _f32p,
                                     _f32p, _i32p]
        L.oracle_map_associate.argtypes = [vp, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int, _f64p, _f64p, _i32p]
        L.oracle_map_solve.argtypes = [_f64p, _i32p, ctypes.c_int, _f64p, ctypes.c_int, _i32p]
        L.oracle_mapopt_step.argtypes = [vp, _f32p, ctypes.c_int, _f64p, _f64p, _f64p, _i32p]
        L.oracle_mapopt_step_corner.argtypes = [vp, vp, _f32p, ctypes.c_int, _f32p, ctypes.c_int, _f64p, _f64p, _f64p,
                                                _i32p]
        L.oracle_laser_mapping.argtypes = [vp, vp, _f32p, ctypes.c_int, _f32p, ctypes.c_int, _f64p, _i32p]
        L.oracle_orb_detect.argtypes = [_u8p, vp, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _u8p, _f32p,
                                        ctypes.c_int]
        L.oracle_orb_level.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _i32p, _i32p]
        L.oracle_orb_match.argtypes = [_u8p, ctypes.c_int, _u8p, ctypes.c_int, _i32p]
        L.oracle_orb_fast.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, _i32p, _i32p]
        L.oracle_intensity_odometry.argtypes = [ctypes.c_int, _u8p, _f32p, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                _i32p, _f64p]
        L.oracle_ground_extract.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _i32p]
        L.oracle_lmap_create.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_lmap_create.restype = vp
        L.oracle_lmap_destroy.argtypes = [vp]
        L.oracle_lmap_counts.argtypes = [vp, _i32p, _i32p]
        L.oracle_lmap_points.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_lmap_points.restype = ctypes.c_int
        L.oracle_lmap_step.argtypes = [vp, _f32p, ctypes.c_int, _f32p, ctypes.c_int, _f64p, _f64p, _f64p, _i32p]
        L.oracle_ground_extract.restype = ctypes.c_int
        L.oracle_loop_icp.argtypes = [_f32p, _i32p, _f64p, _f32p, ctypes.c_int, _f64p, _f32p, _i32p, ctypes.c_int,
                                      _f64p, _f64p, _f64p, _f64p, _i32p]
        L.oracle_odom_fuse.argtypes = [_f64p, _f64p, _f64p, _i32p, ctypes.c_int, _f64p]
        _LIB = L
    return _LIB


class LaserMap:
    """laserMapping's 21 x 21 x 11 cube map + one-frame process (oracle_lmap_*)."""

    NC = 21 * 21 * 11

    def __init__(self, line_res: float = 0.4, plane_res: float = 0.8):
        self.h = lib().oracle_lmap_create(line_res, plane_res)
        self.state = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)  # q_wmap_wodom, t_wmap_wodom

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_lmap_destroy(self.h)
            self.h = None

    def step(self, corner_last: np.ndarray, surf_last: np.ndarray, odom: np.ndarray):
        """One laserMapping frame; returns (pose q_w_curr t_w_curr (7,), stats (8,))."""
        c = np.ascontiguousarray(corner_last, np.float32).reshape(-1, 4)
        s = np.ascontiguousarray(surf_last, np.float32).reshape(-1, 4)
        pose = np.zeros(7, np.float64)
        stats = np.zeros(8, np.int32)
        lib().oracle_lmap_step(self.h, c, c.shape[0], s, s.shape[0], np.ascontiguousarray(odom, np.float64),
                               self.state, pose, stats)
        return pose, stats

    def counts(self):
        cc = np.zeros(self.NC, np.int32)
        sc = np.zeros(self.NC, np.int32)
        lib().oracle_lmap_counts(self.h, cc, sc)
        return cc, sc

    def points(self, which: int) -> np.ndarray:
        n = lib().oracle_lmap_points(self.h, which, None)
        out = np.zeros((max(n, 1), 4), np.float32)
        lib().oracle_lmap_points(self.h, which, out.ctypes.data)
        return out[:n]


@dataclass
class IcpConfig:
    """loop_closure_parameters of config/spot.yaml:26-33 and the ICP settings of
    intensity_feature_tracker.cpp:219-232 (defaults = spot.yaml)."""

    use_crop: bool = False
    crop_size: float = 200.0
    use_downsample: bool = True
    voxel_size: float = 0.25
    max_correspondence_distance: float = 100.0
    max_iterations: int = 100
    transformation_epsilon: float = 1e-6
    euclidean_fitness_epsilon: float = 1e-6
    fitness_threshold: float = 0.5

    def arrays(self):
        f = np.array([self.crop_size, self.voxel_size, self.max_correspondence_distance, 0], np.float32)
        i = np.array([int(self.use_crop), int(self.use_downsample), self.max_iterations, 0], np.int32)
        d = np.array([self.transformation_epsilon, self.euclidean_fitness_epsilon, self.fitness_threshold], np.float64)
        return f, i, d


def _cloud4(c) -> np.ndarray:
    c = np.ascontiguousarray(c, np.float32)
    return c.reshape(-1, 4)


def loop_icp(cur, T_cur, hist, T_hist, cfg: IcpConfig | None = None):
    """The USE_ICP loop-closure block (intensity_feature_tracker.cpp:217-366) on one keyframe pair:
    cur = the keyframe's cloud_track (n, 4), T_cur its 4x4 pose; hist = list of history keyframe
    clouds with their 4x4 poses.  Returns (T_icp (4, 4), T_cur2map (4, 4), fitness, info (8,))."""
    cfg = cfg or IcpConfig()
    f, i, d = cfg.arrays()
    c = _cloud4(cur)
    hs = [_cloud4(h) for h in hist]
    counts = np.array([h.shape[0] for h in hs], np.int32)
    H = np.concatenate(hs) if hs else np.zeros((1, 4), np.float32)
    if H.shape[0] == 0:
        H = np.zeros((1, 4), np.float32)
    Th = np.ascontiguousarray(np.array(T_hist, np.float64).reshape(-1, 16)) if len(hs) else np.zeros((1, 16))
    T_icp = np.zeros(16)
    T_c2m = np.zeros(16)
    fit = np.zeros(1)
    info = np.zeros(8, np.int32)
    lib().oracle_loop_icp(f, i, d, c, c.shape[0], np.ascontiguousarray(T_cur, np.float64).reshape(16), H, counts,
                          len(hs), Th, T_icp, T_c2m, fit, info)
    return T_icp.reshape(4, 4), T_c2m.reshape(4, 4), float(fit[0]), info


class OdomFuser:
    """odomHandler's callback (odom_handler_node.cpp:44-132) over a stream of synchronized pairs."""

    def __init__(self):
        self.state = np.zeros(49, np.float64)

    def step(self, aloam, intensity, skip):
        a = np.ascontiguousarray(aloam, np.float64).reshape(-1, 7)
        b = np.ascontiguousarray(intensity, np.float64).reshape(-1, 7)
        s = np.ascontiguousarray(np.asarray(skip).reshape(-1), np.int32)
        out = np.zeros_like(a)
        lib().oracle_odom_fuse(self.state, a, b, s, a.shape[0], out)
        return out


def ground_extract(points: np.ndarray):
    """ImageHandler::groundPlaneExtraction (image_handler.h_ouster:41-100) of one cloud
    ((n, 3|4) float32, or an organized (H, W, 4) scan).  Returns (ground (m, 4) x y z 1,
    plane (4,) float32 A B C D, info (4,) int32 = status, iterations, best inliers, refit inliers)."""
    P = np.ascontiguousarray(points, np.float32)
    P = P.reshape(-1, P.shape[-1])
    out = np.zeros((P.shape[0], 4), np.float32)
    plane = np.zeros(4, np.float32)
    info = np.zeros(4, np.int32)
    m = lib().oracle_ground_extract(P, P.shape[0], P.shape[1], out, plane, info)
    return out[:m].copy(), plane, info


@dataclass
class ScanFeatures:
    """Outputs of scanRegistration for one scan (all float32 (n, 4) = x, y, z, intensity)."""
    img_range: np.ndarray
    img_intensity: np.ndarray
    cloud_track: np.ndarray
    laser_cloud: np.ndarray
    scan_start: np.ndarray
    scan_end: np.ndarray
    curvature: np.ndarray
    label: np.ndarray
    sharp: np.ndarray
    less_sharp: np.ndarray
    flat: np.ndarray
    less_flat: np.ndarray


# oracle_scanreg.cpp: bit 0 segment sort, bit 1 VoxelGrid by index.  TIES_REFERENCE (libstdc++'s
# std::sort order in both) is the reference and the HIP path's default (LISLAM_TIES_REFERENCE);
# TIES_CANONICAL (index order in both) is the HIP path's LISLAM_TIES_INDEX.
TIES_REFERENCE, TIES_CANONICAL = 0, 3


def scan_registration(scan: np.ndarray, min_range: float = 0.3, canonical: bool | None = None,
                      ties: int | None = None) -> ScanFeatures:
    """scanRegistration a1-a7 of one organized scan.  Tie order of equal sort keys: `ties`
    (TIES_*), or canonical=True (index order throughout) / False (the reference's std::sort
    throughout); the default is the reference's TIES_REFERENCE."""
    if ties is None:
        ties = TIES_CANONICAL if canonical else TIES_REFERENCE
    scan = np.ascontiguousarray(scan, dtype=np.float32)
    H, W = scan.shape[:2]
    N = H * W
    L = lib()
    img_r = np.zeros(N, np.uint8)
    img_i = np.zeros(N, np.uint8)
    track = np.zeros((N, 4), np.float32)
    cloud = np.zeros((N, 4), np.float32)
    ncl = np.zeros(1, np.int32)
    ss = np.zeros(H, np.int32)
    se = np.zeros(H, np.int32)
    curv = np.zeros(N, np.float32)
    lab = np.zeros(N, np.int8)
    sh = np.zeros((12 * H, 4), np.float32)
    ls = np.zeros((120 * H, 4), np.float32)
    fl = np.zeros((24 * H, 4), np.float32)
    lf = np.zeros((N, 4), np.float32)
    n = [np.zeros(1, np.int32) for _ in range(4)]
    L.oracle_scan_registration(scan.reshape(-1), H, W, H, min_range, int(ties), img_r, img_i,
                               track.reshape(-1), cloud.reshape(-1), ncl, ss, se, curv, lab,
                               sh.reshape(-1), n[0], ls.reshape(-1), n[1], fl.reshape(-1), n[2],
                               lf.reshape(-1), n[3])
    c = int(ncl[0])
    return ScanFeatures(img_r.reshape(H, W), img_i.reshape(H, W), track.reshape(H, W, 4), cloud[:c], ss, se,
                        curv[:c], lab[:c], sh[:n[0][0]], ls[:n[1][0]], fl[:n[2][0]], lf[:n[3][0]])


def voxel_grid(points: np.ndarray, leaf: float, canonical: bool = True) -> np.ndarray:
    pts = np.ascontiguousarray(points, dtype=np.float32)
    out = np.zeros_like(pts)
    n = np.zeros(1, np.int32)
    lib().oracle_voxel_grid(pts.reshape(-1), pts.shape[0], leaf, int(canonical), out.reshape(-1), n)
    return out[: n[0]]


def _pack(arrs):
    off = np.zeros(len(arrs) + 1, np.int32)
    off[1:] = np.cumsum([a.shape[0] for a in arrs])
    cat = np.concatenate([a.reshape(-1, 4) for a in arrs]) if off[-1] else np.zeros((1, 4), np.float32)
    return np.ascontiguousarray(cat, np.float32).reshape(-1), off


def odometry_chain(feats: list[ScanFeatures], use_aloam=None):
    """Fresh laserOdometry node over ``feats``; returns (world poses (n,7), para (n,7), stats (n,6)).
    use_aloam (n,) (None: every frame): frame k is optimized only where use_aloam[k] != 0
    (laserOdometry.cpp:403-417), the pose accumulates the previous estimate otherwise."""
    n = len(feats)
    s, so = _pack([f.sharp for f in feats])
    ls, lso = _pack([f.less_sharp for f in feats])
    fl, flo = _pack([f.flat for f in feats])
    lf, lfo = _pack([f.less_flat for f in feats])
    pose = np.zeros((n, 7), np.float64)
    rel = np.zeros((n, 7), np.float64)
    st = np.zeros((n, 6), np.int32)
    if use_aloam is None:
        lib().oracle_odometry_chain(n, s, so, ls, lso, fl, flo, lf, lfo, pose.reshape(-1), rel.reshape(-1),
                                    st.reshape(-1))
    else:
        u = np.ascontiguousarray(np.asarray(use_aloam).reshape(-1), np.int32)
        lib().oracle_odometry_chain_gated(n, s, so, ls, lso, fl, flo, lf, lfo, u, pose.reshape(-1), rel.reshape(-1),
                                          st.reshape(-1))
    return pose, rel, st


def nn1(target: np.ndarray, queries: np.ndarray):
    t = np.ascontiguousarray(target, np.float32)
    q = np.ascontiguousarray(queries, np.float32)
    idx = np.zeros(q.shape[0], np.int32)
    d2 = np.zeros(q.shape[0], np.float32)
    lib().oracle_nn1(t.reshape(-1), t.shape[0], q.reshape(-1), q.shape[0], idx, d2)
    return idx, d2


def eval_factor(kind: int, pts: np.ndarray, q: np.ndarray, t: np.ndarray):
    R = 3 if kind == 0 else 1
    r = np.zeros(R)
    J = np.zeros((R, 7))
    lib().oracle_eval_factor(kind, np.ascontiguousarray(pts, np.float64).reshape(-1),
                             np.ascontiguousarray(q, np.float64), np.ascontiguousarray(t, np.float64), r,
                             J.reshape(-1))
    return r, J


def _xyz4(points) -> np.ndarray:
    p = np.ascontiguousarray(points, np.float32).reshape(-1, points.shape[-1])
    if p.shape[1] == 4:
        return p
    out = np.zeros((p.shape[0], 4), np.float32)
    out[:, :3] = p[:, :3]
    return out


class IkdMap:
    """Restated ikd-Tree point set (oracle_map.cpp): Build / Add_Points / Nearest_Search."""

    def __init__(self, downsample_size: float = 0.2):
        self.h = lib().oracle_map_create(downsample_size)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_map_destroy(self.h)
            self.h = None

    def build(self, points):
        p = _xyz4(points)
        lib().oracle_map_build(self.h, p.reshape(-1), p.shape[0], 4)

    def add_points(self, points, downsample: bool = True) -> int:
        p = _xyz4(points)
        return lib().oracle_map_add_points(self.h, p.reshape(-1), p.shape[0], 4, int(downsample))

    def size(self) -> int:
        return lib().oracle_map_size(self.h)

    def points(self) -> np.ndarray:
        """Live points (n, 4) = x, y, z, id (int32 bits in column 3) in ascending id."""
        out = np.zeros((max(self.size(), 1), 4), np.float32)
        n = lib().oracle_map_points(self.h, out.reshape(-1))
        return out[:n]

    def knn(self, queries, k: int = 5, max_dist: float = float("inf")):
        q = _xyz4(queries)
        n = q.shape[0]
        pts = np.zeros((n, k, 4), np.float32)
        d2 = np.zeros((n, k), np.float32)
        found = np.zeros(n, np.int32)
        lib().oracle_map_knn(self.h, q.reshape(-1), n, 4, k, max_dist, pts.reshape(-1), d2.reshape(-1), found)
        return pts, d2, found

    def associate(self, kind: int, points, x):
        """kind 0 corner line / 1 surf plane: (records (n, 9), block kinds (n,): 0 edge, 2 plane-norm, -1)."""
        p = _xyz4(points)
        n = p.shape[0]
        rec = np.zeros((n, 9))
        valid = np.zeros(n, np.int32)
        lib().oracle_map_associate(self.h, kind, p.reshape(-1), n, 4, np.ascontiguousarray(x, np.float64), rec.reshape(-1),
                                   valid)
        return rec, valid


def map_solve(records: np.ndarray, kinds: np.ndarray, x0, max_iterations: int):
    x = np.array(x0, np.float64)
    summ = np.zeros(2, np.int32)
    rec = np.ascontiguousarray(records, np.float64)
    lib().oracle_map_solve(rec.reshape(-1), np.ascontiguousarray(kinds, np.int32), rec.shape[0], x, max_iterations, summ)
    return x, summ


def mapopt_step(m: IkdMap, ground, odom, state):
    """One mapOptimization ground step; returns (pose (7,), new state (7,), summary (3,))."""
    g = _xyz4(ground)
    st = np.array(state, np.float64)
    pose = np.zeros(7)
    summ = np.zeros(3, np.int32)
    lib().oracle_mapopt_step(m.h, g.reshape(-1), g.shape[0], np.ascontiguousarray(odom, np.float64), st, pose, summ)
    return pose, st, summ


def mapopt_step_corner(m: IkdMap, cm: IkdMap, ground, corner, odom, state):
    """mapOptimization step with its corner ikd-Tree (mapOptimization.cpp:193-195, :477-479):
    as mapopt_step, and pc_corner is added to cm at the keyframe pose."""
    g, c = _xyz4(ground), _xyz4(corner)
    st = np.array(state, np.float64)
    pose = np.zeros(7)
    summ = np.zeros(3, np.int32)
    lib().oracle_mapopt_step_corner(m.h, cm.h, g.reshape(-1), g.shape[0], c.reshape(-1), c.shape[0],
                                    np.ascontiguousarray(odom, np.float64), st, pose, summ)
    return pose, st, summ


def laser_mapping(corner_map: IkdMap, surf_map: IkdMap, corner, surf, x0):
    c, s = _xyz4(corner), _xyz4(surf)
    x = np.array(x0, np.float64)
    stats = np.zeros(4, np.int32)
    lib().oracle_laser_mapping(corner_map.h, surf_map.h, c.reshape(-1), c.shape[0], s.reshape(-1), s.shape[0], x, stats)
    return x, stats


def hand_held_mask(H: int = 64, W: int = 1024, crop: int = 3) -> np.ndarray:
    """feature_tracker::setMask (intensity_feature_tracker.cpp:1126-1136): 0 where j < crop or j > W - crop."""
    m = np.full((H, W), 255, np.uint8)
    j = np.arange(W)
    m[:, (j < crop) | (j > W - crop)] = 0
    return m


def _mask_ptr(mask):
    if mask is None:
        return None, None
    m = np.ascontiguousarray(mask, np.uint8)
    return ctypes.c_void_p(m.ctypes.data), m


def orb_detect(img: np.ndarray, track: np.ndarray, nfeatures: int = 1000, mask=None):
    """ORB detect + zero filter + compute: (keypoints (n, 6) = x, y, size, angle, response, octave,
    descriptors (n, 32) u8, points (n, 3))."""
    im = np.ascontiguousarray(img, np.uint8)
    H, W = im.shape
    tr = np.ascontiguousarray(track, np.float32).reshape(-1)
    cap = 8 * nfeatures + 64
    kp = np.zeros((cap, 6), np.float32)
    de = np.zeros((cap, 32), np.uint8)
    p3 = np.zeros((cap, 3), np.float32)
    mp, _keep = _mask_ptr(mask)
    n = lib().oracle_orb_detect(im.reshape(-1), mp, tr, W, H, nfeatures, kp.reshape(-1), de.reshape(-1), p3.reshape(-1), cap)
    return kp[:n], de[:n], p3[:n]


def orb_level(img: np.ndarray, level: int, blurred: bool = False) -> np.ndarray:
    im = np.ascontiguousarray(img, np.uint8)
    H, W = im.shape
    out = np.zeros(H * W, np.uint8)
    w = np.zeros(1, np.int32)
    h = np.zeros(1, np.int32)
    lib().oracle_orb_level(im.reshape(-1), W, H, level, int(blurred), out, w, h)
    return out[: w[0] * h[0]].reshape(h[0], w[0])


def orb_match(qdesc: np.ndarray, tdesc: np.ndarray) -> np.ndarray:
    q = np.ascontiguousarray(qdesc, np.uint8)
    t = np.ascontiguousarray(tdesc, np.uint8)
    out = np.zeros((max(q.shape[0], 1), 3), np.int32)
    m = lib().oracle_orb_match(q.reshape(-1), q.shape[0], t.reshape(-1), t.shape[0], out.reshape(-1))
    return out[:m]


def intensity_odometry(imgs: np.ndarray, tracks: np.ndarray, nfeatures: int = 1000, mask=None):
    """feature_tracker::detectfeatures over frames: (stats (n, 8), T_s2s (n, 7))."""
    im = np.ascontiguousarray(imgs, np.uint8)
    n, H, W = im.shape
    tr = np.ascontiguousarray(tracks, np.float32).reshape(-1)
    st = np.zeros((n, 8), np.int32)
    T = np.zeros((n, 7))
    mp, _keep = _mask_ptr(mask)
    lib().oracle_intensity_odometry(n, im.reshape(-1), tr, mp, W, H, nfeatures, st.reshape(-1), T.reshape(-1))
    return st, T


def orb_fast(img: np.ndarray, level: int = 0) -> np.ndarray:
    im = np.ascontiguousarray(img, np.uint8)
    H, W = im.shape
    out = np.zeros(H * W, np.int32)
    w = np.zeros(1, np.int32)
    h = np.zeros(1, np.int32)
    lib().oracle_orb_fast(im.reshape(-1), W, H, level, out, w, h)
    return out[: w[0] * h[0]].reshape(h[0], w[0])
