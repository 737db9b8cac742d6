"""Synthetic loop-closure inputs shared by the oracle and GPU tests of the loop-closure ICP
(SURVEY.md §8(f) row 4).  The reference ships no data: a keyframe of the synthetic corridor drive
is re-observed with a drifted pose against the history keyframes around it."""
from __future__ import annotations

import math

import numpy as np


def pose_T(p) -> np.ndarray:
    c, s = math.cos(p.yaw), math.sin(p.yaw)
    T = np.eye(4)
    T[:2, :2] = [[c, -s], [s, c]]
    T[0, 3], T[1, 3] = p.x, p.y
    return T


def drift(dx, dy, dz, yaw_deg, roll_deg=0.0) -> np.ndarray:
    y, r = math.radians(yaw_deg), math.radians(roll_deg)
    Rz = np.array([[math.cos(y), -math.sin(y), 0], [math.sin(y), math.cos(y), 0], [0, 0, 1.0]])
    Rx = np.array([[1.0, 0, 0], [0, math.cos(r), -math.sin(r)], [0, math.sin(r), math.cos(r)]])
    T = np.eye(4)
    T[:3, :3] = Rz @ Rx
    T[:3, 3] = (dx, dy, dz)
    return T


def corridor_loop(synth, k=40, hist=(37, 38, 39), d=(0.3, -0.2, 0.05, 2.0, 0.5), n_scans=64, width=1024):
    """(cur (n, 4), T_cur, [hist clouds], [T_hist], T_true) for keyframe k re-observed with drift d."""
    cur = synth.make_scan(k, n_scans, width).reshape(-1, 4)
    hs = [synth.make_scan(j, n_scans, width).reshape(-1, 4) for j in hist]
    Th = [pose_T(synth.ground_truth_pose(j)) for j in hist]
    T_true = pose_T(synth.ground_truth_pose(k))
    return cur, drift(*d) @ T_true, hs, Th, T_true


def random_room(rng, n=3000):
    """Points on the 6 faces + a few boxes of a 10 x 8 x 3 m room (x, y, z, intensity)."""
    faces = rng.integers(0, 6, n)
    u, v = rng.random(n), rng.random(n)
    P = np.zeros((n, 4), np.float32)
    ext = np.array([10.0, 8.0, 3.0])
    for f in range(6):
        m = faces == f
        ax = f // 2
        o = [a for a in range(3) if a != ax]
        P[m, ax] = (f % 2) * ext[ax] - ext[ax] / 2
        P[m, o[0]] = (u[m] - 0.5) * ext[o[0]]
        P[m, o[1]] = (v[m] - 0.5) * ext[o[1]]
    box = rng.random((n // 5, 3)) * [1.0, 2.0, 1.5] + [1.0, -1.0, -1.5]
    P = np.concatenate([P, np.concatenate([box, np.zeros((box.shape[0], 1))], 1).astype(np.float32)])
    P[:, 3] = rng.random(P.shape[0]) * 255
    P[:, :3] += rng.normal(0, 0.005, (P.shape[0], 3))
    return P.astype(np.float32)
