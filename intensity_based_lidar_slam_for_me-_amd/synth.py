"""Seeded synthetic Ouster-style organized scans of a corridor.

The reference ships no data (its example bag is an external download,
``README.md:152-171``), so every benchmark and parity test runs on scans made
here.  The layout is the organized ring-by-ring cloud that
``ImageHandler::cloud_handler`` indexes as ``u * W + v``
(``src/image_handler.h_ouster:113-117``): ``H x W x 4`` float32 =
``(x, y, z, intensity)`` in the sensor frame.

Design choices that keep the reference's order-dependent logic well defined:

* Beam ``k`` sits at the centre of its ``scanID`` bin of
  ``scanRegistration.cpp:290-325`` so the bin assignment cannot flip on a
  1-ulp difference of ``atan``.
* Azimuth columns carry a fractional offset so no point lands exactly on an
  ``ori`` wrap boundary of ``scanRegistration.cpp:336-366``.
* Range noise N(0, 1 cm) makes exact curvature ties rare.
* 2 % dropouts are ``(0, 0, 0, 0)`` points, which exercise the ``range < 0.1``
  branch of ``cloud_handler`` and ``removeClosedPointCloud``.
* Pillar faces are retro-reflective (intensity up to 300) so the 255 clamp of
  ``image_handler.h_ouster:121`` is exercised.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

BASE_SEED = 20250204

# corridor geometry (metres, world frame)
WALL_Y = 1.5
FLOOR_Z = -0.6
CEIL_Z = 2.0
X_MIN = -20.0
X_MAX = 200.0
PILLAR_PITCH = 6.0
PILLAR_SIZE = 0.4
BEAM_PITCH = 4.0
BEAM_DEPTH = 0.3
BEAM_DROP = 0.35


def beam_elevations_deg(n_scans: int) -> np.ndarray:
    """Elevation of beam k at the centre of its scanID bin (scanRegistration.cpp:290-325)."""
    k = np.arange(n_scans, dtype=np.float64)
    if n_scans == 16:
        # scanID = int((angle + 15) / 2 + 0.5)
        return 2.0 * k - 15.0
    if n_scans == 32:
        # scanID = int((angle + 92/3) * 3/4)
        return (k + 0.5) / 0.75 - 92.0 / 3.0
    if n_scans == 64:
        # scanID = int((angle + 22.5) * 1.41 + 0.5) - 1
        return (k + 1.0) / 1.41 - 22.5
    if n_scans == 128:
        # scanID = int((angle + 22.5) * 2.83 + 0.5) - 1
        return (k + 1.0) / 2.83 - 22.5
    raise ValueError("only 16/32/64/128 scan lines are supported (scanRegistration.cpp:701)")


@dataclass
class Pose:
    x: float
    y: float
    yaw: float

    def as_qt(self):
        """(q[x,y,z,w], t[3]) of sensor->world."""
        h = 0.5 * self.yaw
        return (np.array([0.0, 0.0, math.sin(h), math.cos(h)]), np.array([self.x, self.y, 0.0]))


def ground_truth_pose(scan_idx: int, rate_hz: float = 10.0) -> Pose:
    t = scan_idx / rate_hz
    return Pose(x=1.0 * t, y=0.1 * math.sin(0.3 * t), yaw=0.05 * math.sin(0.2 * t))


def _pillars():
    """Wall pillars: full-height boxes (x-lo, x-hi, y-lo, y-hi) on alternating sides."""
    out = []
    for i, xc in enumerate(np.arange(PILLAR_PITCH, X_MAX - 1.0, PILLAR_PITCH)):
        ylo, yhi = (WALL_Y - PILLAR_SIZE, WALL_Y) if i % 2 == 0 else (-WALL_Y, -WALL_Y + PILLAR_SIZE)
        out.append((xc - PILLAR_SIZE / 2, xc + PILLAR_SIZE / 2, ylo, yhi))
    return np.array(out)


def _beams():
    """Transverse ceiling beams: full-width boxes (x-lo, x-hi, z-lo, z-hi)."""
    xs = np.arange(BEAM_PITCH / 2, X_MAX - 1.0, BEAM_PITCH)
    return np.stack([xs - BEAM_DEPTH / 2, xs + BEAM_DEPTH / 2, np.full_like(xs, CEIL_Z - BEAM_DROP),
                     np.full_like(xs, CEIL_Z)], axis=1)


_PILLARS = _pillars()
_BEAMS = _beams()


def _slab2(o0, o1, d0, d1, lo0, hi0, lo1, hi1):
    """Entry distance of 2-D rays (o + t d) into axis-aligned rectangles; inf if missed."""
    with np.errstate(divide="ignore", invalid="ignore"):
        i0, i1 = 1.0 / d0, 1.0 / d1
        a0, b0 = (lo0 - o0) * i0, (hi0 - o0) * i0
        a1, b1 = (lo1 - o1) * i1, (hi1 - o1) * i1
    tmin = np.maximum(np.minimum(a0, b0), np.minimum(a1, b1))
    tmax = np.minimum(np.maximum(a0, b0), np.maximum(a1, b1))
    hit = (tmax >= tmin) & (tmin > 1e-6)
    return np.where(hit, tmin, np.inf)


def _cast(origin, az_w, el):
    """Nearest hit distance and surface class of every (elevation row, azimuth column) ray from
    inside the corridor.  Surfaces: 0 end walls, 1 side walls, 2 floor/ceiling, 3 pillar/beam."""
    ce, se = np.cos(el)[:, None], np.sin(el)[:, None]              # (H, 1)
    ca, sa = np.cos(az_w)[None, :], np.sin(az_w)[None, :]          # (1, W)
    dx, dy, dz = ce * ca, ce * sa, np.broadcast_to(se, (el.size, az_w.size))
    box_lo = (X_MIN, -WALL_Y, FLOOR_Z)
    box_hi = (X_MAX, WALL_Y, CEIL_Z)
    ts = []
    for ax, d in enumerate((dx, dy, dz)):
        with np.errstate(divide="ignore", invalid="ignore"):
            t = np.where(d > 0, (box_hi[ax] - origin[ax]) / d, (box_lo[ax] - origin[ax]) / d)
        ts.append(np.where(np.abs(d) < 1e-12, np.inf, t))
    ts = np.stack(ts)                                               # (3, H, W)
    surf = np.argmin(ts, axis=0)
    t_hit = np.min(ts, axis=0)
    # pillars span floor to ceiling: a horizontal 2-D test per azimuth column, scaled by 1/cos(el)
    sp = _slab2(origin[0], origin[1], ca.ravel()[:, None], sa.ravel()[:, None], _PILLARS[None, :, 0],
                _PILLARS[None, :, 1], _PILLARS[None, :, 2], _PILLARS[None, :, 3]).min(axis=1)
    tp = sp[None, :] / ce
    # beams span wall to wall: a 2-D (x, z) test per ray
    tb = _slab2(origin[0], origin[2], dx[..., None], dz[..., None], _BEAMS[:, 0], _BEAMS[:, 1], _BEAMS[:, 2],
                _BEAMS[:, 3]).min(axis=2)
    tob = np.minimum(tp, tb)
    closer = tob < t_hit
    return np.where(closer, tob, t_hit).ravel(), np.where(closer, 3, surf).ravel(), \
        np.stack([dx, dy, dz], axis=-1).reshape(-1, 3)


def make_scan(scan_idx: int, n_scans: int = 64, width: int = 1024, seed_base: int = BASE_SEED,
              pose: Pose | None = None) -> np.ndarray:
    """One organized scan, ``(n_scans, width, 4)`` float32, row 0 = top beam (Ouster order)."""
    rng = np.random.default_rng(seed_base + scan_idx)
    pose = pose or ground_truth_pose(scan_idx)
    el = np.deg2rad(beam_elevations_deg(n_scans))[::-1]          # row u -> beam H-1-u
    col = np.arange(width, dtype=np.float64)
    az = -2.0 * math.pi * (col + 0.37) / width                   # clockwise sweep like an Ouster
    cel, sel = np.cos(el)[:, None], np.sin(el)[:, None]
    d_sensor = np.stack([np.broadcast_to(cel * np.cos(az)[None, :], (n_scans, width)),
                         np.broadcast_to(cel * np.sin(az)[None, :], (n_scans, width)),
                         np.broadcast_to(sel, (n_scans, width))], axis=-1).reshape(-1, 3)
    origin = np.array([pose.x, pose.y, 0.0])
    t_hit, surf, d_world = _cast(origin, az + pose.yaw, el)
    rng_noise = rng.normal(0.0, 0.01, size=t_hit.shape)
    r = t_hit + rng_noise
    p_world = origin + d_world * t_hit[:, None]
    # checker texture in surface coordinates (0.5 m period)
    u = np.where(surf == 0, p_world[:, 1], p_world[:, 0])
    v = np.where(surf == 2, p_world[:, 1], p_world[:, 2])
    checker = (np.floor(u / 0.5) + np.floor(v / 0.5)).astype(np.int64) & 1
    inten = np.where(surf == 3, 260.0 + 30.0 * checker, 40.0 + 180.0 * checker)
    inten = np.clip(inten + rng.normal(0.0, 5.0, size=inten.shape), 0.0, 300.0)
    pts = np.empty((n_scans * width, 4), dtype=np.float64)
    pts[:, :3] = d_sensor * r[:, None]
    pts[:, 3] = inten
    drop = rng.random(t_hit.shape) < 0.02
    pts[drop] = 0.0
    return pts.astype(np.float32).reshape(n_scans, width, 4)


def make_sequence(n: int, n_scans: int = 64, width: int = 1024, start: int = 0) -> np.ndarray:
    """``n`` consecutive scans of the 10 Hz corridor drive, ``(n, H, W, 4)`` float32."""
    out = np.empty((n, n_scans, width, 4), dtype=np.float32)
    for i in range(n):
        out[i] = make_scan(start + i, n_scans, width)
    return out


def relative_ground_truth(k: int):
    """Ground-truth T_{k-1 <- k} as (q[x,y,z,w], t)."""
    a, b = ground_truth_pose(k - 1), ground_truth_pose(k)
    dyaw = b.yaw - a.yaw
    ca, sa = math.cos(a.yaw), math.sin(a.yaw)
    dx, dy = b.x - a.x, b.y - a.y
    t = np.array([ca * dx + sa * dy, -sa * dx + ca * dy, 0.0])
    return np.array([0.0, 0.0, math.sin(dyaw / 2), math.cos(dyaw / 2)]), t


# ------------------------------------------------------------------ maps (config 5, a19-a21)
def make_corridor_map(n_points: int, spacing: float = 0.05, seed: int = BASE_SEED, x0: float = -10.0,
                      noise: float = 0.005) -> np.ndarray:
    """World-frame surface samples of the corridor (floor, ceiling, side walls, pillar faces) on a
    jittered ``spacing`` grid, extended along +x until ``n_points`` points exist; ``(n, 4)``
    float32 with w = 0 (PointXYZ as PCL stores it).  SURVEY.md §8(d) config 5: 5 cm sampling."""
    rng = np.random.default_rng(seed)
    s = spacing
    ny = int(round(2 * WALL_Y / s))
    nz = int(round((CEIL_Z - FLOOR_Z) / s))
    per_x = 2 * ny + 2 * nz  # floor + ceiling + two walls per x step
    nx = max(1, int(math.ceil(n_points / per_x)))
    xs = x0 + s * np.arange(nx)
    parts = []
    gy = -WALL_Y + s * (np.arange(ny) + 0.5)
    gz = FLOOR_Z + s * (np.arange(nz) + 0.5)
    X, Y = np.meshgrid(xs, gy, indexing="ij")
    for zc in (FLOOR_Z, CEIL_Z):
        parts.append(np.stack([X.ravel(), Y.ravel(), np.full(X.size, zc)], axis=1))
    X, Z = np.meshgrid(xs, gz, indexing="ij")
    for yc in (-WALL_Y, WALL_Y):
        parts.append(np.stack([X.ravel(), np.full(X.size, yc), Z.ravel()], axis=1))
    P = np.concatenate(parts)
    # in-plane jitter (no exact distance ties) and normal noise
    P += rng.uniform(-0.25 * s, 0.25 * s, size=P.shape) + rng.normal(0.0, noise, size=P.shape)
    P = P[:n_points]
    out = np.zeros((P.shape[0], 4), np.float32)
    out[:, :3] = P
    return out


def make_edge_map(n_lines: int = 40, spacing: float = 0.05, seed: int = BASE_SEED + 7, x0: float = 0.0) -> np.ndarray:
    """Vertical pillar edges (corner map of laserMapping): points every ``spacing`` along the four
    vertical edges of the first ``n_lines / 4`` pillars, jittered 5 mm.  ``(n, 4)`` float32."""
    rng = np.random.default_rng(seed)
    pts = []
    for i, (xl, xh, yl, yh) in enumerate(_PILLARS[: max(1, n_lines // 4)]):
        for ex, ey in ((xl, yl), (xl, yh), (xh, yl), (xh, yh)):
            z = np.arange(FLOOR_Z, CEIL_Z, spacing)
            e = np.stack([np.full(z.size, ex + x0), np.full(z.size, ey), z], axis=1)
            pts.append(e + rng.normal(0.0, 0.005, size=e.shape))
    P = np.concatenate(pts)
    out = np.zeros((P.shape[0], 4), np.float32)
    out[:, :3] = P
    return out


def perturb_pose(q, t, dt: float = 0.05, drot_deg: float = 0.5, seed: int = 1):
    """(q, t) perturbed by a random translation of |dt| and rotation of drot about a random axis;
    returned as x = (qx, qy, qz, qw, tx, ty, tz)."""
    rng = np.random.default_rng(seed)
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    h = 0.5 * math.radians(drot_deg)
    dq = np.array([*(math.sin(h) * ax), math.cos(h)])
    x1, y1, z1, w1 = dq
    x2, y2, z2, w2 = q
    qq = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                   w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
    dtv = rng.normal(size=3)
    dtv *= dt / np.linalg.norm(dtv)
    return np.concatenate([qq, np.asarray(t, np.float64) + dtv])
