"""Host-side mirror of the loop-closure ICP and the odometry fusion node
over the lislam C ABI.

``loop_closure_icp`` plays the ``USE_ICP`` block of ``feature_tracker::loopClosureThread``
(``src/intensity_feature_tracker.cpp:217-366``) with ``tranformCurrentScanToMap`` (``:167-172``)
and ``getSubmapOfhistory`` (``:174-193``); ``OdomHandler.callback`` plays ``odomHandler``'s
``callback`` (``src/odom_handler_node.cpp:44-132``).  ``get_transform_matrix`` is
``feature_tracker::getTransformMatrix`` (``:152-165``) on a ``PointTypePose`` (x, y, z, roll,
pitch, yaw).  All compute runs in ``liblislam.so`` on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from . import native as nat
from .mapping import _as_points

IcpConfig = nat.IcpConfig

ACCEPTED, REJECTED, EMPTY_SUBMAP, TOO_FEW_POINTS = 1, 0, -1, -2
CONVERGENCE_STATES = ("not_converged", "iterations", "transform", "abs_mse", "rel_mse", "no_correspondences")


def get_transform_matrix(x, y, z, roll, pitch, yaw) -> np.ndarray:
    """feature_tracker::getTransformMatrix (:152-165) of a PointTypePose: the reference builds
    ``gtsam::Rot3::RzRyRx(p.yaw, p.pitch, p.roll)``, i.e. Rz(roll) Ry(pitch) Rx(yaw) (RzRyRx(x, y, z)
    = Rz(z) Ry(y) Rx(x): the stored roll and yaw trade places), normalized through a quaternion."""
    def rz(a):
        c, s = math.cos(a), math.sin(a)
        return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])

    def ry(a):
        c, s = math.cos(a), math.sin(a)
        return np.array([[c, 0, s], [0, 1.0, 0], [-s, 0, c]])

    def rx(a):
        c, s = math.cos(a), math.sin(a)
        return np.array([[1.0, 0, 0], [0, c, -s], [0, s, c]])

    T = np.eye(4)
    T[:3, :3] = rz(roll) @ ry(pitch) @ rx(yaw)
    T[:3, 3] = (x, y, z)
    return T


def loop_closure_icp(ctx, cur, T_cur, hist, T_hist, cfg: IcpConfig | None = None):
    """ICP of the new keyframe's cloud_track ``cur`` (n, 4) at pose ``T_cur`` (4x4) against the
    history keyframes ``hist`` (list of (m, 4) clouds) at ``T_hist`` (list of 4x4).

    Returns ``(T_icp (4, 4), T_cur2map (4, 4), fitness, info (8,))``; ``info[0]`` is ACCEPTED when
    the loop factor would be added (``hasConverged() && getFitnessScore() <= FITNESS_SCORE``,
    :314)."""
    cfg = cfg or IcpConfig()
    pc, nc, stride, kc = _as_points(cur)
    if stride != 4:
        raise ValueError("cur must be (n, 4) x, y, z, intensity")
    hs = [np.ascontiguousarray(h, np.float32).reshape(-1, 4) for h in hist]
    counts = np.array([h.shape[0] for h in hs] or [0], np.int32)
    H = np.concatenate(hs) if hs else np.zeros((0, 4), np.float32)
    Tc = np.ascontiguousarray(T_cur, np.float64).reshape(16)
    Th = np.ascontiguousarray(np.array(T_hist, np.float64).reshape(-1, 16)) if hs else np.zeros((1, 16))
    T_icp = np.zeros(16)
    T_c2m = np.zeros(16)
    fit = np.zeros(1)
    info = np.zeros(8, np.int32)
    nat.check(ctx.lib.lislam_loop_icp(ctx.h, ctypes.byref(cfg), pc, nc, nat.ptr(Tc), nat.ptr(H) if H.size else None,
                                      nat.ptr(counts), len(hs), nat.ptr(Th), nat.ptr(T_icp), nat.ptr(T_c2m),
                                      nat.ptr(fit), nat.ptr(info)), ctx.h, "lislam_loop_icp")
    return T_icp.reshape(4, 4), T_c2m.reshape(4, 4), float(fit[0]), info


class OdomHandler:
    """odomHandler's callback (odom_handler_node.cpp:44-132) with its state on the device."""

    SKIP_FRAME_ID = "/odom_skip"

    def __init__(self, ctx):
        self.ctx = ctx
        h = ctypes.c_void_p()
        nat.check(ctx.lib.lislam_odom_fuser_create(ctx.h, ctypes.byref(h)), ctx.h, "lislam_odom_fuser_create")
        self.h = h

    def close(self):
        if self.h:
            self.ctx.lib.lislam_odom_fuser_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fuse(self, aloam, intensity, skip) -> np.ndarray:
        """n synchronized pairs ((n, 7) q x,y,z,w + t each; skip (n,) bool) -> fused (n, 7)."""
        a = np.ascontiguousarray(aloam, np.float64).reshape(-1, 7)
        b = np.ascontiguousarray(intensity, np.float64).reshape(-1, 7)
        s = np.ascontiguousarray(np.asarray(skip).reshape(-1), np.int32)
        if not (a.shape[0] == b.shape[0] == s.shape[0]):
            raise ValueError("aloam, intensity and skip must hold the same number of pairs")
        out = np.zeros_like(a)
        nat.check(self.ctx.lib.lislam_odom_fuse(self.h, nat.ptr(a), nat.ptr(b), nat.ptr(s), a.shape[0], nat.ptr(out)),
                  self.ctx.h, "lislam_odom_fuse")
        return out

    def callback(self, aloam_odom, intensity_odom, child_frame_id: str) -> np.ndarray:
        """One message pair; returns the published /laser_odom_to_init pose (7,)."""
        return self.fuse(aloam_odom, intensity_odom, [child_frame_id == self.SKIP_FRAME_ID])[0]
