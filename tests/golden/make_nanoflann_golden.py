"""Regenerates tests/golden/knn_nanoflann.npz (test infrastructure): exact k-NN neighbour sets from
the reference's OWN vendored kd-tree, nanoflann v1.3.2 (/root/reference/include/nanoflann.hpp:62,
through KDTreeVectorOfVectorsAdaptor.h), compiled where it lies by `make -C oracle ref`
(oracle/ref_nanoflann_knn.cpp -> oracle/_ref/nanoflann_knn).  Only this build container has
/root/reference; the GPU box reads the committed vectors.

Cases (inputs regenerated from the seeded generator and the oracle; their sha256 is stored so drift
is caught):
  corridor5  k = 5 over a 200k-point corridor map (config 5's map, 5 cm sampling) with 4000 queries
             jittered off its surfaces and 200 far outside it (laserMapping.cpp:673,753; the
             ikd-Tree's Nearest_Search, mapOptimization.cpp:393)
  lessflat1  k = 1 of scan 1's flat points in scan 0's less-flat cloud, 64 x 1024 (the surf
             association's KdTreeFLANN query, laserOdometry.cpp:574)
  lesssharp1 k = 1 of scan 1's sharp points in scan 0's less-sharp cloud (laserOdometry.cpp:452)
Usage:  python tests/golden/make_nanoflann_golden.py
"""
from __future__ import annotations

import hashlib
import importlib
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

synth = importlib.import_module("intensity_based_lidar_slam_for_me-_amd.synth")
EXE = os.path.join(ROOT, "oracle", "_ref", "nanoflann_knn")


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def cases():
    """The inputs of every case: name -> (target (n, 3) float32, queries (m, 3) float32, k)."""
    import oracle as O

    out = {}
    M = synth.make_corridor_map(200_000, spacing=0.05)[:, :3]
    rng = np.random.default_rng(61)
    near = M[rng.choice(M.shape[0], 4000, replace=False)] + rng.normal(0.0, 0.04, (4000, 3))
    far = rng.uniform(-40.0, 80.0, (200, 3))
    out["corridor5"] = (M, np.concatenate([near, far]).astype(np.float32), 5)
    f0, f1 = (O.scan_registration(s) for s in synth.make_sequence(2, 64, 1024, start=30))
    out["lessflat1"] = (f0.less_flat[:, :3], f1.flat[:, :3], 1)
    out["lesssharp1"] = (f0.less_sharp[:, :3], f1.sharp[:, :3], 1)
    return {k: (np.ascontiguousarray(t, np.float32), np.ascontiguousarray(q, np.float32), kk)
            for k, (t, q, kk) in out.items()}


def run_nanoflann(target: np.ndarray, queries: np.ndarray, k: int):
    """(found (m,), idx (m, k), dist_sq (m, k)) from oracle/_ref/nanoflann_knn."""
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as fh:
            np.array([target.shape[0], queries.shape[0], k], np.int32).tofile(fh)
            target.tofile(fh)
            queries.tofile(fh)
        subprocess.run([EXE, fin, fout], check=True)
        raw = np.fromfile(fout, np.int32)
    m = queries.shape[0]
    found = raw[:m].copy()
    idx = raw[m:m + m * k].reshape(m, k).copy()
    dist = raw[m + m * k:].view(np.float32).reshape(m, k).copy()
    return found, idx, dist


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    rec = {}
    for name, (t, q, k) in cases().items():
        found, idx, dist = run_nanoflann(t, q, k)
        rec[f"{name}_k"] = np.int32(k)
        rec[f"{name}_target_sha256"] = np.array(digest(t))
        rec[f"{name}_queries_sha256"] = np.array(digest(q))
        rec[f"{name}_found"], rec[f"{name}_idx"], rec[f"{name}_dist_sq"] = found, idx, dist
        print(f"{name}: {t.shape[0]} targets, {q.shape[0]} queries, k = {k}")
    np.savez_compressed(os.path.join(HERE, "knn_nanoflann.npz"), **rec)


if __name__ == "__main__":
    main()
