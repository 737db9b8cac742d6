"""Host-side mirror of the reference's per-scan interfaces over the lislam C ABI.

``ScanRegistration.laser_cloud_handler`` plays ``laserCloudHandler``
(``src/scanRegistration.cpp:189``) and returns the clouds that node publishes
(``:592-642``); ``LaserOdometry.step`` plays one pass of the laserOdometry main loop
(``src/laserOdometry.cpp:313-808``) in forced-geometric mode; ``Batch`` runs both stages for a
batch of scans resident in HBM.  All compute runs in ``liblislam.so`` on the GPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import native as nat

CAP_SHARP_PER_LINE, CAP_LESS_SHARP_PER_LINE, CAP_FLAT_PER_LINE = 12, 120, 24

PACKED_XYZI = nat.PointLayout(16, 0, 4, 8, 12)
OUSTER_LAYOUT = nat.PointLayout(48, 0, 4, 8, 16)  # os_cloud_node/points: x y z pad intensity ...
PCL_XYZI_LAYOUT = nat.PointLayout(32, 0, 4, 8, 16)  # pcl::PointXYZI as toROSMsg writes it


class Context:
    """One HIP device + stream (lislam_ctx)."""

    def __init__(self, n_scans: int = 64, width: int = 1024, min_range: float = 0.3, max_iterations: int = 4,
                 want_images: bool = True, device: int = 0):
        self.lib = nat.load()
        self.n_scans, self.width, self.device = n_scans, width, device
        cfg = nat.Config(n_scans, width, min_range, max_iterations, int(want_images))
        h = ctypes.c_void_p()
        rc = self.lib.lislam_ctx_create(ctypes.byref(cfg), device, ctypes.byref(h))
        if rc != nat.OK:
            raise nat.LislamError(f"lislam_ctx_create failed ({rc}) for n_scans={n_scans} width={width} device={device}")
        self.h = h

    def close(self):
        if self.h:
            self.lib.lislam_ctx_destroy(self.h)
            self.h = None

    def synchronize(self):
        nat.check(self.lib.lislam_synchronize(self.h), self.h, "lislam_synchronize")

    TIES_REFERENCE, TIES_INDEX = 0, 1
    ENGINE_OFF, ENGINE_AUTO, ENGINE_ON = 0, 1, 2  # lislam_set_odometry_schedule

    def set_odometry_schedule(self, mode: int):
        """lislam_set_odometry_schedule: ENGINE_OFF (per-round launches), ENGINE_ON (one persistent
        launch, k_odom_chain) or ENGINE_AUTO.  Results are the same."""
        nat.check(self.lib.lislam_set_odometry_schedule(self.h, int(mode)), self.h, "lislam_set_odometry_schedule")

    SHAPE_LATENCY = (1, 1)     # lislam_set_engine_shape: one query per wavefront, one engine at a time
    SHAPE_THROUGHPUT = (3, 5)  # three queries per wavefront, five engines in flight (pipelined contexts)

    def set_engine_shape(self, queries_per_wave: int = 0, depth: int = 0):
        """lislam_set_engine_shape: the chain engine's queries per wavefront (1..4) and engines in
        flight per device (1..6) for this context's launches; 0 keeps a value.  Results are the same."""
        nat.check(self.lib.lislam_set_engine_shape(self.h, int(queries_per_wave), int(depth)), self.h,
                  "lislam_set_engine_shape")

    def masked_queues(self) -> int:
        """CU-masked streams (hardware queues) the library holds on this context's device
        (lislam_device_queue_count)."""
        n = ctypes.c_int32(0)
        nat.check(self.lib.lislam_device_queue_count(int(self.device), ctypes.byref(n)), self.h,
                  "lislam_device_queue_count")
        return int(n.value)

    def set_tie_order(self, order: int):
        """Order of equal voxels in the a7 VoxelGrid (lislam_set_tie_order): TIES_REFERENCE
        (default, PCL 1.10's std::sort order, bit-exact) or TIES_INDEX (input order, faster)."""
        nat.check(self.lib.lislam_set_tie_order(self.h, int(order)), self.h, "lislam_set_tie_order")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Features:
    laser_cloud: np.ndarray
    sharp: np.ndarray
    less_sharp: np.ndarray
    flat: np.ndarray
    less_flat: np.ndarray
    image_range: np.ndarray | None = None
    image_intensity: np.ndarray | None = None
    cloud_track: np.ndarray | None = None


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class ScanRegistration:
    """scanRegistration node: PointCloud2 -> images + the five feature clouds."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def laser_cloud_handler(self, points: np.ndarray, layout: nat.PointLayout | None = None) -> Features:
        c = self.ctx
        H, W = c.n_scans, c.width
        N = H * W
        pts = np.ascontiguousarray(points)
        lay = layout or PACKED_XYZI
        cloud = np.zeros((N, 4), np.float32)
        sh = np.zeros((CAP_SHARP_PER_LINE * H, 4), np.float32)
        ls = np.zeros((CAP_LESS_SHARP_PER_LINE * H, 4), np.float32)
        fl = np.zeros((CAP_FLAT_PER_LINE * H, 4), np.float32)
        lf = np.zeros((N, 4), np.float32)
        ir = np.zeros(N, np.uint8)
        ii = np.zeros(N, np.uint8)
        tr = np.zeros((N, 4), np.float32)
        out = nat.ScanOut(_fp(cloud), N, 0, _fp(sh), sh.shape[0], 0, _fp(ls), ls.shape[0], 0, _fp(fl), fl.shape[0], 0,
                          _fp(lf), N, 0, ir.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                          ii.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _fp(tr))
        rc = c.lib.lislam_scan_registration(c.h, nat.ptr(pts), ctypes.byref(lay), ctypes.byref(out))
        nat.check(rc, c.h, "lislam_scan_registration")
        return Features(cloud[: out.n_laser_cloud], sh[: out.n_sharp], ls[: out.n_less_sharp], fl[: out.n_flat],
                        lf[: out.n_less_flat], ir.reshape(H, W), ii.reshape(H, W), tr.reshape(H, W, 4))


class ImageHandler:
    """ImageHandler's ground stage (src/image_handler.h_ouster:41-100) on the GPU."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def ground_plane_extraction(self, points: np.ndarray, layout: nat.PointLayout | None = None):
        """groundPlaneExtraction of one organized cloud (the context's n_scans x width points):
        (GroundPointOut (m, 4) x y z 1, plane (4,) A B C D, info (4,) = status, RANSAC iterations,
        best inliers, refit inliers; status 1 = ground, 0 = plane rejected by the n.z > cos 15 deg
        test, -1 / -2 / -3 = no model)."""
        c = self.ctx
        N = c.n_scans * c.width
        pts = np.ascontiguousarray(points)
        out = np.zeros((N, 4), np.float32)
        plane = np.zeros(4, np.float32)
        info = np.zeros(4, np.int32)
        n = ctypes.c_int32()
        rc = c.lib.lislam_ground_extract(c.h, nat.ptr(pts), ctypes.byref(layout or PACKED_XYZI), nat.ptr(out), N,
                                         ctypes.byref(n), nat.ptr(plane), nat.ptr(info))
        nat.check(rc, c.h, "lislam_ground_extract")
        return out[: n.value].copy(), plane, info


class LaserOdometry:
    """laserOdometry node.  step(f) is the forced geometric mode (every frame is optimized);
    step(f, skip_flag=...) follows the reference's default gating (laserOdometry.cpp:403-417): the
    frame is optimized only when the sharp cloud's frame_id is "skip_intensity"."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = ctypes.c_void_p()
        nat.check(ctx.lib.lislam_odom_create(ctx.h, ctypes.byref(h)), ctx.h, "lislam_odom_create")
        self.h = h

    SKIP_INTENSITY = "skip_intensity"

    def step(self, f: Features, skip_flag: str | None = None):
        arrs = [np.ascontiguousarray(a, np.float32) for a in (f.sharp, f.less_sharp, f.flat, f.less_flat)]
        fr = nat.Frame(_fp(arrs[0]), arrs[0].shape[0], _fp(arrs[1]), arrs[1].shape[0], _fp(arrs[2]), arrs[2].shape[0],
                       _fp(arrs[3]), arrs[3].shape[0])
        para = np.zeros(7)
        pose = np.zeros(7)
        st = np.zeros(8, np.int32)
        if skip_flag is None:
            rc = self.ctx.lib.lislam_odom_step(self.h, ctypes.byref(fr), nat.ptr(para), nat.ptr(pose), nat.ptr(st))
        else:
            rc = self.ctx.lib.lislam_odom_step_gated(self.h, ctypes.byref(fr), int(skip_flag == self.SKIP_INTENSITY),
                                                     nat.ptr(para), nat.ptr(pose), nat.ptr(st))
        nat.check(rc, self.ctx.h, "lislam_odom_step")
        return para, pose, st

    def close(self):
        if self.h:
            self.ctx.lib.lislam_odom_destroy(self.h)
            self.h = None


class Batch:
    """A device-resident batch of scans (a1..a7 + a12..a18 on HBM-resident data)."""

    def __init__(self, ctx: Context, max_scans: int):
        self.ctx = ctx
        self.max_scans = max_scans
        h = ctypes.c_void_p()
        nat.check(ctx.lib.lislam_batch_create(ctx.h, max_scans, ctypes.byref(h)), ctx.h, "lislam_batch_create")
        self.h = h

    def upload(self, scans: np.ndarray, layout: nat.PointLayout | None = None):
        a = np.ascontiguousarray(scans)
        n = a.shape[0]
        rc = self.ctx.lib.lislam_batch_upload(self.h, nat.ptr(a), n, ctypes.byref(layout or PACKED_XYZI))
        nat.check(rc, self.ctx.h, "lislam_batch_upload")

    def upload_async(self, ptr, n: int, layout: nat.PointLayout | None = None):
        """lislam_batch_upload_async of n scans at host address ptr (a ctypes pointer to pinned
        memory that stays valid until the context stream has passed the upload)."""
        rc = self.ctx.lib.lislam_batch_upload_async(self.h, ptr, n, ctypes.byref(layout or PACKED_XYZI))
        nat.check(rc, self.ctx.h, "lislam_batch_upload_async")

    def extract(self, n: int):
        nat.check(self.ctx.lib.lislam_batch_extract(self.h, n), self.ctx.h, "lislam_batch_extract")

    def odometry(self, n: int, chain_len: int, use_aloam=None):
        """a12-a18 over scans [0, n) in chains of chain_len pairs.  use_aloam (n,) switches to the
        reference's default gating (laserOdometry.cpp:403-417): scan k is optimized only where
        use_aloam[k] != 0 (see skip_flags)."""
        if use_aloam is None:
            nat.check(self.ctx.lib.lislam_batch_odometry(self.h, n, chain_len), self.ctx.h, "lislam_batch_odometry")
            return
        u = np.ascontiguousarray(np.asarray(use_aloam).reshape(-1), np.int32)
        if u.shape[0] < n:
            raise ValueError("use_aloam needs one flag per scan")
        nat.check(self.ctx.lib.lislam_batch_odometry_gated(self.h, n, chain_len, nat.ptr(u)), self.ctx.h,
                  "lislam_batch_odometry_gated")

    def odometry_status(self) -> int:
        """Engine launches that gave up since the previous call (a bounded device wait expired); each
        was re-run on the per-round schedule before its outputs could be read.  The call clears it."""
        st = ctypes.c_int32(0)
        nat.check(self.ctx.lib.lislam_batch_odometry_status(self.h, ctypes.byref(st)), self.ctx.h,
                  "lislam_batch_odometry_status")
        return int(st.value)

    ENGINES = ("per-round launches (k_odom_assoc16 + k_odom_lm2)", "single-launch engine (k_odom_chain)",
               "split engine (k_odom_roles + k_odom_items)")

    def odometry_engine(self) -> int:
        """The schedule of the last odometry call (lislam_batch_odometry_engine): 0 per-round
        launches, 1 the single-launch engine, 2 the split engine (ENGINES names them)."""
        k = ctypes.c_int32(0)
        nat.check(self.ctx.lib.lislam_batch_odometry_engine(self.h, ctypes.byref(k)), self.ctx.h,
                  "lislam_batch_odometry_engine")
        return int(k.value)

    def odometry_abort_code(self) -> int:
        """The error word of the last aborted engine launch (lislam_batch_odometry_abort_code)."""
        k = ctypes.c_int32(0)
        nat.check(self.ctx.lib.lislam_batch_odometry_abort_code(self.h, ctypes.byref(k)), self.ctx.h,
                  "lislam_batch_odometry_abort_code")
        return int(k.value)

    def skip_flags(self, n: int) -> np.ndarray:
        """use_aloam per scan from the ORB front end's results (intensity_odometry first): 1 where
        detectfeatures skipped the frame (the "skip_intensity" frame_id, scanRegistration.cpp:603-609)."""
        return np.array([int(self.download(nat.OUT_ORB_STATS, k)[0] == 0) for k in range(n)], np.int32)

    def intensity_odometry(self, n: int, nfeatures: int = 1000, mask=None):
        """feature_tracker::detectfeatures over scans [0, n) of the batch (ORB path a8-a11)."""
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        rc = self.ctx.lib.lislam_batch_intensity_odometry(self.h, n, nfeatures,
                                                          None if m is None else ctypes.c_void_p(m.ctypes.data))
        nat.check(rc, self.ctx.h, "lislam_batch_intensity_odometry")
        self._mask_keep = m

    def orb_cascade_info(self):
        """(converged on the device: 1 / redone with host rounds: 0 / host rounds only: -1, device
        decision passes) of the last intensity_odometry (lislam_batch_orb_cascade_info)."""
        info = np.zeros(2, np.int32)
        rc = self.ctx.lib.lislam_batch_orb_cascade_info(self.h, info.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        nat.check(rc, self.ctx.h, "lislam_batch_orb_cascade_info")
        return int(info[0]), int(info[1])

    def ground(self, n: int):
        """groundPlaneExtraction of scans [0, n) of the batch (results: ground_result)."""
        nat.check(self.ctx.lib.lislam_batch_ground(self.h, n), self.ctx.h, "lislam_batch_ground")

    def ground_result(self, scan: int):
        """(GroundPointOut (m, 4), plane (4,), info (4,)) of one scan after ground()."""
        return (self.download(nat.OUT_GROUND, scan), self.download(nat.OUT_GROUND_PLANE, scan),
                self.download(nat.OUT_GROUND_INFO, scan))

    def set_timing(self, on: bool):
        nat.check(self.ctx.lib.lislam_batch_set_timing(self.h, int(on)), self.ctx.h, "lislam_batch_set_timing")

    def kernel_times(self):
        """Per kernel (native.KERNELS): average ms per call and launches per call since the last
        read, plus the number of (extract, odometry) calls averaged."""
        ms = np.zeros(len(nat.KERNELS), np.float32)
        launches = np.zeros(len(nat.KERNELS), np.int32)
        calls = np.zeros(2, np.int32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        rc = self.ctx.lib.lislam_batch_kernel_times(self.h, _fp(ms), launches.ctypes.data_as(i32p),
                                                    calls.ctypes.data_as(i32p))
        nat.check(rc, self.ctx.h, "lislam_batch_kernel_times")
        return ms, launches, calls

    _DT = {nat.OUT_IMAGE_RANGE: (np.uint8, 1), nat.OUT_IMAGE_INTENSITY: (np.uint8, 1), nat.OUT_CLOUD_TRACK: (np.float32, 4),
           nat.OUT_LASER_CLOUD: (np.float32, 4), nat.OUT_CURVATURE: (np.float32, 1), nat.OUT_LABEL: (np.int8, 1),
           nat.OUT_LINE_OFFSETS: (np.int32, 1), nat.OUT_SHARP: (np.float32, 4), nat.OUT_LESS_SHARP: (np.float32, 4),
           nat.OUT_FLAT: (np.float32, 4), nat.OUT_LESS_FLAT: (np.float32, 4), nat.OUT_PARA: (np.float64, 1),
           nat.OUT_POSE: (np.float64, 1), nat.OUT_STATS: (np.int32, 1), nat.OUT_ORB_T: (np.float64, 1),
           nat.OUT_ORB_STATS: (np.int32, 1), nat.OUT_ORB_KEYPOINTS: (np.float32, 6), nat.OUT_ORB_POINTS: (np.float32, 4),
           nat.OUT_ORB_DESCRIPTORS: (np.uint8, 32), nat.OUT_GROUND: (np.float32, 4),
           nat.OUT_GROUND_PLANE: (np.float32, 1), nat.OUT_GROUND_INFO: (np.int32, 1)}

    def download(self, what: int, scan: int) -> np.ndarray:
        dt, w = self._DT[what]
        N = self.ctx.n_scans * self.ctx.width
        cap = max(N, 16)
        buf = np.zeros((cap, w) if w > 1 else cap, dt)
        n = ctypes.c_int32()
        rc = self.ctx.lib.lislam_batch_download(self.h, what, scan, nat.ptr(buf), cap, ctypes.byref(n))
        nat.check(rc, self.ctx.h, "lislam_batch_download")
        return buf[: n.value].copy()

    def count(self, what: int, scan: int) -> int:
        """Element count of one output (lislam_batch_download with no destination)."""
        n = ctypes.c_int32()
        nat.check(self.ctx.lib.lislam_batch_download(self.h, what, scan, None, 0, ctypes.byref(n)), self.ctx.h,
                  "lislam_batch_download")
        return n.value

    def download_cloud(self, what: int, scan: int, layout: nat.PointLayout | None = None) -> bytes:
        """toROSMsg of a point-cloud output: the PointCloud2 data bytes in `layout` (PCL PointXYZI
        by default), packed on the device."""
        lay = layout or PCL_XYZI_LAYOUT
        cap = max(self.ctx.n_scans * self.ctx.width, 16)
        buf = np.zeros(cap * lay.point_step, np.uint8)
        n = ctypes.c_int32()
        rc = self.ctx.lib.lislam_batch_download_cloud(self.h, what, scan, nat.ptr(buf), ctypes.byref(lay), cap,
                                                      ctypes.byref(n))
        nat.check(rc, self.ctx.h, "lislam_batch_download_cloud")
        return buf[: n.value * lay.point_step].tobytes()

    def features(self, scan: int) -> Features:
        return Features(self.download(nat.OUT_LASER_CLOUD, scan), self.download(nat.OUT_SHARP, scan),
                        self.download(nat.OUT_LESS_SHARP, scan), self.download(nat.OUT_FLAT, scan),
                        self.download(nat.OUT_LESS_FLAT, scan))

    def close(self):
        if self.h:
            self.ctx.lib.lislam_batch_destroy(self.h)
            self.h = None


def eval_factors(ctx: Context, kind: np.ndarray, pts: np.ndarray, q: np.ndarray, t: np.ndarray):
    """GPU evaluation of LidarEdgeFactor / LidarPlaneFactor / LidarPlaneNormFactor blocks."""
    kind = np.ascontiguousarray(kind, np.int32)
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 12)
    n = kind.shape[0]
    r = np.zeros((n, 3))
    J = np.zeros((n, 3, 6))
    rc = ctx.lib.lislam_eval_factors(ctx.h, n, nat.ptr(kind), nat.ptr(pts), nat.ptr(np.ascontiguousarray(q, np.float64)),
                                     nat.ptr(np.ascontiguousarray(t, np.float64)), nat.ptr(r), nat.ptr(J))
    nat.check(rc, ctx.h, "lislam_eval_factors")
    return r, J
