"""Counter passes of the chain engine (run under rocprofv3 --pmc / --kernel-trace, program right
after --): config 2's batch (300 synthetic 64x1024 scans, one continuous 299-pair chain) extracted
once, then `--launches` odometry calls, each synchronized and followed by the batch's abort count.

The split engine's two launches must run together, and dispatch-counter collection serializes
dispatches, so under --pmc every split launch gives up (and is re-run on the per-round schedule).
The counters are therefore taken on the single-launch engine (LISLAM_ENGINE_SINGLE=1, k_odom_chain:
the same association items and solve as the split engine, in one grid).  Its launches can also give
up under the profiler; the JSON line lists which did, and scripts/summarize_engine_pmc.py averages
the counters over the launches that did not.

Usage: python3 scripts/engine_pmc.py [--launches N] [--scan-cache PREFIX]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--scan-cache", default="/tmp/lislam_scans")
    ap.add_argument("--batch", type=int, default=300)
    args = ap.parse_args()
    import bench

    B, H, W = args.batch, 64, 1024
    cache = f"{args.scan_cache}.0_{B}_{H}x{W}.npy"
    if os.path.exists(cache):
        scans = np.load(cache)
    else:
        scans = bench.generate(0, B, H, W, 16)
        np.save(cache, scans)
    pkg = importlib.import_module(bench.PKG)
    if os.environ.get("LISLAM_ALT_LIB"):  # developer A/B: a variant build of the library
        pkg.native.load(os.environ["LISLAM_ALT_LIB"])
    ctx = pkg.Context(n_scans=H, width=W)
    b = pkg.Batch(ctx, B)
    b.upload(scans)
    b.extract(B)
    ctx.synchronize()
    aborted, ms = [], []
    for i in range(args.launches):
        t0 = time.perf_counter()
        b.odometry(B, B - 1)
        ctx.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
        aborted.append(b.odometry_status())
    print(json.dumps({"launches": args.launches, "engine": b.ENGINES[b.odometry_engine()], "aborted": aborted,
                      "host_ms": [round(v, 3) for v in ms],
                      "config": {"lines": H, "width": W, "scans_per_step_per_gpu": B, "chain_len": B - 1}}), flush=True)
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
