"""Host-side mirror of the reference's ORB intensity front end over the lislam C ABI.

``IntensityTracker.detectfeatures`` plays ``feature_tracker::detectfeatures``
(``src/intensity_feature_tracker.cpp:597-738``): ORB detect / describe on the intensity image
(``cv::ORB::create(1000, 1.2f, 8, 1)``), cloud-track lookup, Hamming cross-check matching
against the previous frame, selection of the best 30 % (20 % after re-detection with 2000
features) and the point-to-point Ceres solve ``p2p_calculateRandT`` -> ``T_s2s``.  ``orb_detect``
and ``orb_match`` expose the two OpenCV calls; ``set_mask`` is ``feature_tracker::setMask``.
All compute runs in ``liblislam.so`` on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native as nat

NUM_ORB_FEATURES = 1000  # spot.yaml:14
IMAGE_CROP = 3           # spot.yaml:9


def set_mask(H: int = 64, W: int = 1024, crop: int = IMAGE_CROP) -> np.ndarray:
    """feature_tracker::setMask (intensity_feature_tracker.cpp:1126-1136): 0 where j < crop or j > W - crop."""
    m = np.full((H, W), 255, np.uint8)
    j = np.arange(W)
    m[:, (j < crop) | (j > W - crop)] = 0
    return m


def _u8(a):
    return None if a is None else np.ascontiguousarray(a, np.uint8)


def _vp(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def orb_detect(ctx, image, cloud_track, nfeatures: int = NUM_ORB_FEATURES, mask=None):
    """detect + extractPointsAndFilterZeroValue + compute: (keypoints (n, 6), descriptors (n, 32), points (n, 4))."""
    img = _u8(image)
    H, W = img.shape
    tr = np.ascontiguousarray(cloud_track, np.float32).reshape(H * W, 4)
    m = _u8(mask)
    cap = 8 * nfeatures + 1024
    kp = np.zeros((cap, 6), np.float32)
    de = np.zeros((cap, 32), np.uint8)
    p3 = np.zeros((cap, 4), np.float32)
    n = ctypes.c_int32()
    nat.check(ctx.lib.lislam_orb_detect(ctx.h, _vp(img), _vp(tr), _vp(m), H, W, nfeatures, nat.ptr(kp), nat.ptr(de),
                                        nat.ptr(p3), cap, ctypes.byref(n)), ctx.h, "lislam_orb_detect")
    return kp[: n.value], de[: n.value], p3[: n.value]


def orb_match(ctx, qdesc, tdesc) -> np.ndarray:
    """BFMatcher(NORM_HAMMING, crossCheck).match: (m, 3) = query, train, distance in query order."""
    q, t = _u8(qdesc), _u8(tdesc)
    out = np.zeros((max(q.shape[0], 1), 3), np.int32)
    n = ctypes.c_int32()
    nat.check(ctx.lib.lislam_orb_match(ctx.h, _vp(q), q.shape[0], _vp(t), t.shape[0], nat.ptr(out), ctypes.byref(n)),
              ctx.h, "lislam_orb_match")
    return out[: n.value]


class IntensityTracker:
    """feature_tracker's per-frame front end (state = the previous frame) on the GPU."""

    def __init__(self, ctx, H: int = 64, W: int = 1024, nfeatures: int = NUM_ORB_FEATURES, mask=None):
        self.ctx = ctx
        self._mask = _u8(mask)
        h = ctypes.c_void_p()
        nat.check(ctx.lib.lislam_intensity_tracker_create(ctx.h, H, W, nfeatures, _vp(self._mask), ctypes.byref(h)),
                  ctx.h, "lislam_intensity_tracker_create")
        self.h = h
        self.T_s2m = np.eye(4)  # tfBroadcast accumulation (intensity_feature_tracker.cpp:819)

    def detectfeatures(self, image, cloud_track):
        """One frame: (T_s2s (7,) = q x,y,z,w, t; stats (8,))."""
        img = _u8(image)
        tr = np.ascontiguousarray(cloud_track, np.float32)
        T = np.zeros(7)
        st = np.zeros(8, np.int32)
        nat.check(self.ctx.lib.lislam_intensity_tracker_step(self.h, _vp(img), _vp(tr), nat.ptr(T), nat.ptr(st)),
                  self.ctx.h, "lislam_intensity_tracker_step")
        x, y, z, w = T[:4]
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        Ts = np.eye(4)
        Ts[:3, :3] = R
        Ts[:3, 3] = T[4:]
        self.T_s2m = self.T_s2m @ Ts
        return T, st

    def close(self):
        if self.h:
            self.ctx.lib.lislam_intensity_tracker_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
