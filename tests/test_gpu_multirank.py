"""Config 4's sharded path on the GPU: `bench.py --gpus 2 --total-scans T` starts two ranks
(they share the box's one GPU round-robin), each runs its contiguous shard with chains restarting
at the shard boundary (laserOdometry.cpp:130-135 within a shard), and every
rank's poses, stats and feature counts equal the oracle's chains over the same shard.  The line
itself carries the CPU baseline and every rank's pose delta (bench.py's CPU stage runs on every rank
before it touches the GPU)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POSE_TOL = 1e-4


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_ranks_config4_shards_match_oracle(tmp_path, oracle, synth):
    T, L = 14, 4
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--total-scans", str(T),
                          "--chain", str(L), "--steps", "2", "--warmup", "1", "--cpu-budget", "2", "--cpu-workers", "2",
                          "--sustain-s", "0", "--workers", "1", "--dump-dir", str(tmp_path)],
                         capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.strip()][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["total_scans_per_step"] == T
    # the multi-GPU line carries the CPU baseline (rank 0's shard, timed before it touched the GPU)
    # and every rank's pose delta against the oracle over its own shard
    cpu, pd = line["cpu_baseline"], line["pose_delta_vs_cpu"]
    assert cpu is not None and cpu["kind"] == "port" and cpu["value"] > 0
    assert pd is not None and pd["ranks_compared"] == 2 and pd["within_tolerance"], pd
    assert pd["stats_mismatches"] == 0 and pd["pairs_compared"] >= 2 * (7 - 1), pd
    for r in range(2):
        d = np.load(tmp_path / f"rank{r}.npz")
        start, n = int(d["start"]), int(d["n"])
        assert (start, n) == (7 * r, 7)
        scans = synth.make_sequence(n, start=start)
        feats = [oracle.scan_registration(s) for s in scans]
        for k, f in enumerate(feats):
            ref = [f.laser_cloud.shape[0], f.sharp.shape[0], f.less_sharp.shape[0], f.flat.shape[0], f.less_flat.shape[0]]
            assert list(d["counts"][k]) == ref, (r, k)
        for c0 in range(0, n - 1, L):
            chain = feats[c0:min(c0 + L, n - 1) + 1]
            pose, rel, st = oracle.odometry_chain(chain)
            for j in range(1, len(chain)):
                k = c0 + j
                assert np.max(np.abs(d["pose"][k] - pose[j])) < POSE_TOL, (r, k)
                assert np.max(np.abs(d["para"][k] - rel[j])) < POSE_TOL, (r, k)
                assert np.array_equal(d["stats"][k][:4], st[j][:4]), (r, k)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_eight_ranks_config4_full_shape(tmp_path, oracle, synth):
    """Config 4 at its full shape on the one GPU: `bench.py --gpus 8 --total-scans 1000` (eight
    rank processes round-robin on the card, 125 contiguous scans each, one continuous odometry chain
    per shard).  The line carries n_gpus 8 and total_scans_per_step 1000; every rank's feature counts
    match the oracle on its whole shard, and its poses / para / stats on every one of the 124 pairs
    of its chain."""
    T, W = 1000, 8
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(W), "--total-scans", str(T),
                          "--steps", "1", "--warmup", "1", "--cpu-budget", "0", "--sustain-s", "0", "--segmented", "0",
                          "--workers", "1", "--dump-dir", str(tmp_path)],
                         capture_output=True, text=True, timeout=560, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.strip()][-1])
    assert line["n_gpus"] == W and line["scaling"] == "strong"
    assert line["config"]["total_scans_per_step"] == T
    per = T // W
    for r in range(W):
        d = np.load(tmp_path / f"rank{r}.npz")
        start, n = int(d["start"]), int(d["n"])
        assert (start, n) == (per * r, per)
        assert int(d["chain"]) == n - 1  # one continuous chain over the shard
        print(f"rank {r}: shard [{start}, {start + n}) checking", flush=True)
        scans = synth.make_sequence(n, start=start)
        feats = [oracle.scan_registration(s) for s in scans]
        for k, f in enumerate(feats):
            ref = [f.laser_cloud.shape[0], f.sharp.shape[0], f.less_sharp.shape[0], f.flat.shape[0], f.less_flat.shape[0]]
            assert list(d["counts"][k]) == ref, (r, k)
        pose, rel, st = oracle.odometry_chain(feats)
        for k in range(1, n):
            assert np.max(np.abs(d["pose"][k] - pose[k])) < POSE_TOL, (r, k)
            assert np.max(np.abs(d["para"][k] - rel[k])) < POSE_TOL, (r, k)
            assert np.array_equal(d["stats"][k][:6], st[k][:6]), (r, k)  # correspondences + LM iterations
