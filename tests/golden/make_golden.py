"""Regenerates the golden fixtures under tests/golden/ (test infrastructure).

The reference ships no tests, fixtures or golden vectors and cannot be built here (SURVEY.md
§4, §8(c)), so the fixtures are produced by the C++ oracle restatement and cross-checked, when
generated, against the independent numpy / pure-Python restatement in tests/restate_np.py and
against scipy's exact kNN.  Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import importlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O  # noqa: E402
import restate_np as R  # noqa: E402

synth = importlib.import_module("intensity_based_lidar_slam_for_me-_amd.synth")


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def small_fixture():
    """Three consecutive 16 x 256 scans: every a1..a7 output and the odometry chain."""
    scans = synth.make_sequence(3, 16, 256)
    out = {"scans": scans}
    feats = [O.scan_registration(s) for s in scans]
    for k, f in enumerate(feats):
        cl, off = R.laser_cloud(scans[k], 16)
        assert np.array_equal(cl, f.laser_cloud), "numpy restatement disagrees with the oracle (laser_cloud)"
        assert np.array_equal(R.curvature(cl), f.curvature)
        sh, ls, fl, lf, lab = R.select_features(cl, off, f.curvature, 16)
        for a, b in ((sh, f.sharp), (ls, f.less_sharp), (fl, f.flat), (lf, f.less_flat), (lab, f.label)):
            assert np.array_equal(a, b), "pure-Python selection disagrees with the oracle"
        for name in ("img_range", "img_intensity", "cloud_track", "laser_cloud", "scan_start", "scan_end",
                     "curvature", "label", "sharp", "less_sharp", "flat", "less_flat"):
            out[f"s{k}_{name}"] = getattr(f, name)
    pose, rel, st = O.odometry_chain(feats)
    out["odom_pose"], out["odom_para"], out["odom_stats"] = pose, rel, st
    np.savez_compressed(os.path.join(HERE, "scan16x256_chain3.npz"), **out)


def full_size_digests():
    """64 x 1024 and 128 x 2048 scans: digests and counts of the oracle outputs (inputs are
    regenerated from the seeded generator; their digests guard against generator drift)."""
    rec = {}
    for (H, W, n) in ((64, 1024, 3), (128, 2048, 2)):
        scans = synth.make_sequence(n, H, W)
        feats = [O.scan_registration(s) for s in scans]
        pose, rel, st = O.odometry_chain(feats)
        entry = {"input_sha256": [digest(s) for s in scans], "scans": []}
        for f in feats:
            entry["scans"].append({name: {"n": int(getattr(f, name).shape[0]), "sha256": digest(getattr(f, name))}
                                   for name in ("laser_cloud", "curvature", "label", "sharp", "less_sharp", "flat",
                                                "less_flat")})
        entry["odom_para"] = rel.tolist()
        entry["odom_pose"] = pose.tolist()
        entry["odom_stats"] = st.tolist()
        rec[f"{H}x{W}"] = entry
    with open(os.path.join(HERE, "full_size_digests.json"), "w") as fh:
        json.dump(rec, fh, indent=1)


def knn_fixture():
    """Exact 1-NN vectors (scipy cKDTree) on a real less-flat target cloud."""
    from scipy.spatial import cKDTree

    scans = synth.make_sequence(2, 16, 256)
    f0, f1 = (O.scan_registration(s) for s in scans)
    tgt, q = f0.less_flat, f1.flat
    d, i = cKDTree(tgt[:, :3].astype(np.float64)).query(q[:, :3].astype(np.float64), k=1)
    np.savez_compressed(os.path.join(HERE, "nn1_scipy.npz"), target=tgt, queries=q, idx=i.astype(np.int32), dist=d)


if __name__ == "__main__":
    small_fixture()
    full_size_digests()
    knn_fixture()
    print("golden fixtures written to", HERE)
