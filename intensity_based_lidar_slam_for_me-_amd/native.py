"""ctypes binding of ``liblislam.so`` (the C ABI declared in ``include/lislam.h``).

The HIP library is the only compute path: if it is missing this module raises, it never falls
back to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblislam.so")

OK = 0
ERR_ARG, ERR_DEVICE, ERR_CAPACITY, ERR_STATE = -1, -2, -3, -4

OUT_IMAGE_RANGE, OUT_IMAGE_INTENSITY, OUT_CLOUD_TRACK, OUT_LASER_CLOUD = 0, 1, 2, 3
OUT_CURVATURE, OUT_LABEL, OUT_LINE_OFFSETS = 4, 5, 6
OUT_SHARP, OUT_LESS_SHARP, OUT_FLAT, OUT_LESS_FLAT = 7, 8, 9, 10
OUT_PARA, OUT_POSE, OUT_STATS = 11, 12, 13
OUT_ORB_T, OUT_ORB_STATS, OUT_ORB_KEYPOINTS, OUT_ORB_POINTS, OUT_ORB_DESCRIPTORS = 14, 15, 16, 17, 18
OUT_GROUND, OUT_GROUND_PLANE, OUT_GROUND_INFO = 19, 20, 21

KERNELS = ("k_scan_front", "k_scan_lines", "k_scan_compact", "k_target_index", "k_odom_assoc", "k_odom_lm",
           "k_odom_chain")

EXPORTED_SYMBOLS = (
    "lislam_ctx_create", "lislam_ctx_destroy", "lislam_last_error", "lislam_synchronize",
    "lislam_set_stream", "lislam_get_stream", "lislam_scan_registration", "lislam_odom_create",
    "lislam_odom_destroy", "lislam_odom_step", "lislam_batch_create", "lislam_batch_destroy",
    "lislam_batch_upload", "lislam_batch_upload_async", "lislam_batch_download_cloud", "lislam_batch_input_device_ptr", "lislam_batch_extract",
    "lislam_batch_odometry", "lislam_batch_set_timing", "lislam_batch_kernel_times",
    "lislam_batch_download", "lislam_eval_factors", "lislam_eval_factors_raw", "lislam_set_tie_order", "lislam_set_odometry_schedule", "lislam_set_engine_shape", "lislam_batch_odometry_status",
    "lislam_batch_odometry_engine", "lislam_batch_odometry_abort_code", "lislam_device_queue_count",
    "lislam_map_create", "lislam_map_destroy", "lislam_map_build", "lislam_map_add_points", "lislam_map_size",
    "lislam_map_points", "lislam_map_nearest_search", "lislam_map_associate", "lislam_normal_equations",
    "lislam_pose_solve", "lislam_voxel_grid", "lislam_mapopt_step", "lislam_mapopt_step_corner", "lislam_laser_mapping",
    "lislam_map_set_timing", "lislam_map_kernel_times",
    "lislam_orb_detect", "lislam_orb_match", "lislam_intensity_tracker_create", "lislam_intensity_tracker_destroy",
    "lislam_intensity_tracker_step", "lislam_batch_intensity_odometry", "lislam_batch_orb_cascade_info", "lislam_batch_ground", "lislam_ground_extract",
    "lislam_lmap_create", "lislam_lmap_destroy", "lislam_lmap_step", "lislam_lmap_counts", "lislam_lmap_points",
    "lislam_batch_odometry_gated", "lislam_odom_step_gated", "lislam_batch_mapopt", "lislam_batch_mapopt_corner", "lislam_loop_icp", "lislam_odom_fuser_create", "lislam_odom_fuser_destroy", "lislam_odom_fuse",
)

MAP_KERNELS = ("k_knn", "k_fit", "k_lm_eval", "k_lm_step", "map_rebuild", "map_downsample", "k_orb_pyramid",
               "k_orb_fast", "k_orb_select", "k_orb_finish", "k_orb_blur", "k_orb_desc", "k_orb_match", "k_orb_lm",
               "k_ground_screen", "k_ground_ransac", "k_ground_extract", "k_lc_step", "k_lc_apply", "k_fuse",
               "k_orb_roiblur", "k_lm_solve")

MATCH_LINE, MATCH_PLANE = 0, 1


class Config(ctypes.Structure):
    _fields_ = [("n_scans", ctypes.c_int32), ("width", ctypes.c_int32), ("min_range", ctypes.c_float),
                ("max_iterations", ctypes.c_int32), ("want_images", ctypes.c_int32)]


class PointLayout(ctypes.Structure):
    _fields_ = [("point_step", ctypes.c_uint32), ("off_x", ctypes.c_uint32), ("off_y", ctypes.c_uint32),
                ("off_z", ctypes.c_uint32), ("off_intensity", ctypes.c_uint32)]


_fp = ctypes.POINTER(ctypes.c_float)
_i32 = ctypes.c_int32
_i32p = ctypes.POINTER(ctypes.c_int32)


class ScanOut(ctypes.Structure):
    _fields_ = [("laser_cloud", _fp), ("cap_laser_cloud", _i32), ("n_laser_cloud", _i32),
                ("sharp", _fp), ("cap_sharp", _i32), ("n_sharp", _i32),
                ("less_sharp", _fp), ("cap_less_sharp", _i32), ("n_less_sharp", _i32),
                ("flat", _fp), ("cap_flat", _i32), ("n_flat", _i32),
                ("less_flat", _fp), ("cap_less_flat", _i32), ("n_less_flat", _i32),
                ("image_range", ctypes.POINTER(ctypes.c_uint8)), ("image_intensity", ctypes.POINTER(ctypes.c_uint8)),
                ("cloud_track", _fp)]


class MapConfig(ctypes.Structure):
    _fields_ = [("downsample_size", ctypes.c_float), ("cell_size", ctypes.c_float)]


class IcpConfig(ctypes.Structure):
    """lislam_icp_config: loop_closure_parameters (config/spot.yaml:26-33) + the ICP settings of
    intensity_feature_tracker.cpp:219-232; defaults = spot.yaml."""

    _fields_ = [("use_crop", _i32), ("crop_size", ctypes.c_float), ("use_downsample", _i32),
                ("voxel_size", ctypes.c_float), ("max_correspondence_distance", ctypes.c_float),
                ("max_iterations", _i32), ("transformation_epsilon", ctypes.c_double),
                ("euclidean_fitness_epsilon", ctypes.c_double), ("fitness_threshold", ctypes.c_double)]

    def __init__(self, use_crop=False, crop_size=200.0, use_downsample=True, voxel_size=0.25,
                 max_correspondence_distance=100.0, max_iterations=100, transformation_epsilon=1e-6,
                 euclidean_fitness_epsilon=1e-6, fitness_threshold=0.5):
        super().__init__(int(use_crop), crop_size, int(use_downsample), voxel_size, max_correspondence_distance,
                         max_iterations, transformation_epsilon, euclidean_fitness_epsilon, fitness_threshold)


class Frame(ctypes.Structure):
    _fields_ = [("sharp", _fp), ("n_sharp", _i32), ("less_sharp", _fp), ("n_less_sharp", _i32),
                ("flat", _fp), ("n_flat", _i32), ("less_flat", _fp), ("n_less_flat", _i32)]


_LIB = None


def _preload_torch_runtime():
    """Load torch's HIP runtime first (when torch is importable) so that liblislam binds to the
    same libamdhip64 instance as torch in processes that use both."""
    if os.environ.get("LISLAM_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional plumbing
        pass


def load(path: str = LIB_PATH):
    """Load the HIP library; raises if it is missing (no CPU fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise RuntimeError(f"liblislam.so not built ({path}); run __graft_entry__.build()")
    _preload_torch_runtime()
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.lislam_ctx_create.argtypes = [ctypes.POINTER(Config), _i32, ctypes.POINTER(vp)]
    L.lislam_ctx_destroy.argtypes = [vp]
    L.lislam_last_error.argtypes = [vp]
    L.lislam_last_error.restype = ctypes.c_char_p
    L.lislam_synchronize.argtypes = [vp]
    L.lislam_set_stream.argtypes = [vp, vp]
    L.lislam_get_stream.argtypes = [vp, ctypes.POINTER(vp)]
    L.lislam_scan_registration.argtypes = [vp, vp, ctypes.POINTER(PointLayout), ctypes.POINTER(ScanOut)]
    L.lislam_odom_create.argtypes = [vp, ctypes.POINTER(vp)]
    L.lislam_odom_destroy.argtypes = [vp]
    L.lislam_odom_step.argtypes = [vp, ctypes.POINTER(Frame), vp, vp, vp]
    L.lislam_batch_create.argtypes = [vp, _i32, ctypes.POINTER(vp)]
    L.lislam_batch_destroy.argtypes = [vp]
    L.lislam_batch_upload.argtypes = [vp, vp, _i32, ctypes.POINTER(PointLayout)]
    L.lislam_batch_upload_async.argtypes = [vp, vp, _i32, ctypes.POINTER(PointLayout)]
    L.lislam_batch_input_device_ptr.argtypes = [vp, ctypes.POINTER(vp)]
    L.lislam_batch_extract.argtypes = [vp, _i32]
    L.lislam_batch_odometry.argtypes = [vp, _i32, _i32]
    L.lislam_batch_set_timing.argtypes = [vp, _i32]
    L.lislam_batch_kernel_times.argtypes = [vp, _fp, _i32p, _i32p]
    L.lislam_batch_download.argtypes = [vp, _i32, _i32, vp, _i32, _i32p]
    L.lislam_batch_download_cloud.argtypes = [vp, _i32, _i32, vp, ctypes.POINTER(PointLayout), _i32, _i32p]
    L.lislam_eval_factors.argtypes = [vp, _i32, vp, vp, vp, vp, vp, vp]
    L.lislam_eval_factors_raw.argtypes = [vp, _i32, vp, vp, vp, vp, vp, vp, vp]
    L.lislam_set_tie_order.argtypes = [vp, _i32]
    L.lislam_set_odometry_schedule.argtypes = [vp, _i32]
    L.lislam_set_engine_shape.argtypes = [vp, _i32, _i32]
    L.lislam_batch_odometry_status.argtypes = [vp, ctypes.POINTER(_i32)]
    L.lislam_batch_odometry_engine.argtypes = [vp, ctypes.POINTER(_i32)]
    L.lislam_batch_odometry_abort_code.argtypes = [vp, ctypes.POINTER(_i32)]
    L.lislam_device_queue_count.argtypes = [_i32, ctypes.POINTER(_i32)]
    i64, i64p = ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)
    L.lislam_map_create.argtypes = [vp, ctypes.POINTER(MapConfig), ctypes.POINTER(vp)]
    L.lislam_map_destroy.argtypes = [vp]
    L.lislam_map_build.argtypes = [vp, vp, i64, _i32]
    L.lislam_map_add_points.argtypes = [vp, vp, i64, _i32, _i32, i64p]
    L.lislam_map_size.argtypes = [vp, i64p]
    L.lislam_map_points.argtypes = [vp, vp, i64, i64p]
    L.lislam_map_nearest_search.argtypes = [vp, vp, _i32, _i32, _i32, ctypes.c_float, vp, vp, vp]
    L.lislam_map_associate.argtypes = [vp, _i32, vp, _i32, _i32, vp, vp, vp]
    L.lislam_normal_equations.argtypes = [vp, vp, vp, _i32, vp, vp]
    L.lislam_pose_solve.argtypes = [vp, vp, vp, _i32, vp, _i32, vp]
    L.lislam_voxel_grid.argtypes = [vp, vp, _i32, ctypes.c_float, vp, _i32p]
    L.lislam_mapopt_step.argtypes = [vp, vp, _i32, vp, vp, vp, vp]
    L.lislam_mapopt_step_corner.argtypes = [vp, vp, vp, _i32, vp, _i32, vp, vp, vp, vp]
    L.lislam_laser_mapping.argtypes = [vp, vp, vp, _i32, vp, _i32, vp, vp]
    L.lislam_orb_detect.argtypes = [vp, vp, vp, vp, _i32, _i32, _i32, vp, vp, vp, _i32, _i32p]
    L.lislam_orb_match.argtypes = [vp, vp, _i32, vp, _i32, vp, _i32p]
    L.lislam_intensity_tracker_create.argtypes = [vp, _i32, _i32, _i32, vp, ctypes.POINTER(vp)]
    L.lislam_intensity_tracker_destroy.argtypes = [vp]
    L.lislam_intensity_tracker_step.argtypes = [vp, vp, vp, vp, vp]
    L.lislam_batch_intensity_odometry.argtypes = [vp, _i32, _i32, vp]
    L.lislam_batch_orb_cascade_info.argtypes = [vp, _i32p]
    L.lislam_batch_ground.argtypes = [vp, _i32]
    L.lislam_lmap_create.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.POINTER(vp)]
    L.lislam_lmap_destroy.argtypes = [vp]
    L.lislam_lmap_step.argtypes = [vp, vp, _i32, vp, _i32, vp, vp, vp, vp]
    L.lislam_lmap_counts.argtypes = [vp, vp, vp]
    L.lislam_lmap_points.argtypes = [vp, _i32, vp, i64, i64p]
    L.lislam_ground_extract.argtypes = [vp, vp, ctypes.POINTER(PointLayout), vp, _i32, _i32p, vp, vp]
    L.lislam_batch_odometry_gated.argtypes = [vp, _i32, _i32, vp]
    L.lislam_odom_step_gated.argtypes = [vp, vp, _i32, vp, vp, vp]
    L.lislam_batch_mapopt.argtypes = [vp, vp, _i32, vp, vp, vp, vp]
    L.lislam_batch_mapopt_corner.argtypes = [vp, vp, vp, _i32, vp, vp, vp, vp]
    L.lislam_loop_icp.argtypes = [vp, ctypes.POINTER(IcpConfig), vp, _i32, vp, vp, vp, _i32, vp, vp, vp, vp, vp]
    L.lislam_odom_fuser_create.argtypes = [vp, ctypes.POINTER(vp)]
    L.lislam_odom_fuser_destroy.argtypes = [vp]
    L.lislam_odom_fuse.argtypes = [vp, vp, vp, vp, _i32, vp]
    L.lislam_map_set_timing.argtypes = [vp, _i32]
    L.lislam_map_kernel_times.argtypes = [vp, _fp, _i32p]
    for name in EXPORTED_SYMBOLS:
        getattr(L, name).restype = getattr(L, name).restype or ctypes.c_int
    L.lislam_last_error.restype = ctypes.c_char_p
    _LIB = L
    return L


class LislamError(RuntimeError):
    pass


def check(rc: int, ctx=None, what: str = ""):
    if rc != OK:
        msg = ""
        if ctx:
            raw = load().lislam_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise LislamError(f"{what} failed with status {rc}: {msg}")


def ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)
