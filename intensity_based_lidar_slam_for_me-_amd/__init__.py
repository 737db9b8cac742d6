"""lislam: MI355X-native intensity-LiDAR SLAM front-end hot path.

Import with ``importlib.import_module("intensity_based_lidar_slam_for_me-_amd")`` (the directory
name is not a Python identifier).  The compute path is the HIP library ``liblislam.so`` built by
``__graft_entry__.build()``; there is no CPU fallback.
"""
from . import intensity, loop, mapping, native, synth  # noqa: F401
from .frontend import Batch, Context, Features, ImageHandler, LaserOdometry, ScanRegistration, eval_factors  # noqa: F401

__all__ = ["intensity", "loop", "mapping", "native", "synth", "Batch", "Context", "Features", "ImageHandler", "LaserOdometry",
           "ScanRegistration", "eval_factors"]
