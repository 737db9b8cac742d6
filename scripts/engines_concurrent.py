"""Developer tool (GPU box): K engines at once with nothing else on the GPU.  K contexts, each with
its own 300-scan batch already extracted; every rep queues one continuous chain per context at the
throughput shape and waits for all of them.  Prints each context's engine time (its t0/t1 events)
per rep and the wall time per rep, so the spread between concurrent chains is visible without the
extraction beside them.
usage: python scripts/engines_concurrent.py [K ...]   (default 1 2 3 4 5)"""
import ctypes
import os
import sys
import time

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
if os.environ.get("LISLAM_ALT_LIB"):
    pkg.native.load(os.environ["LISLAM_ALT_LIB"])
S = 300
REPS = int(os.environ.get("REPS", "4"))
cache = f"/tmp/lislam_scans.0_{S}_64x1024.npy"
scans = np.load(cache) if os.path.exists(cache) else pkg.synth.make_sequence(S)
ks = [int(x) for x in sys.argv[1:]] or [1, 2, 3, 4, 5]
shape = os.environ.get("SHAPE", "throughput")
ctxs, bats = [], []
for i in range(max(ks)):
    c = pkg.Context()
    c.set_odometry_schedule(c.ENGINE_ON)
    c.set_engine_shape(*(c.SHAPE_THROUGHPUT if shape == "throughput" else c.SHAPE_LATENCY))
    b = pkg.Batch(c, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, S - 1)
    c.synchronize()
    ctxs.append(c)
    bats.append(b)
ref = bats[0].download(pkg.native.OUT_POSE, S - 1)
# EXTRA=n idle contexts: n more hardware queues (each context's stream is CU-masked)
idle = [pkg.Context() for _ in range(int(os.environ.get("EXTRA", "0")))]
print(f"masked queues: {ctxs[0].masked_queues()}", flush=True)
# a LISLAM_ENG_STAMPS build (scripts/build_variant.sh stamps lislam_odometry.hip -DLISLAM_ENG_STAMPS=1,
# LISLAM_ALT_LIB=scripts/_ab/liblislam_stamps.so): each launch's role / item start and end
lib = ctxs[0].lib
stamps = hasattr(lib, "lislam_debug_engine_stamps")
st_buf = np.zeros((64, 12), np.uint64)
if stamps:
    lib.lislam_debug_engine_stamps.argtypes = [ctypes.c_void_p]
    lib.lislam_debug_engine_stamps(st_buf.ctypes.data)
for k in ks:
    walls, per, stamp_rows = [], [], []
    for r in range(REPS):
        for b in bats[:k]:
            b.set_timing(True)
        t = time.perf_counter()
        if stamps:
            print(f"rep {r} submit at {time.monotonic() * 1e3:.3f} ms", file=sys.stderr, flush=True)
        for b in bats[:k]:
            b.odometry(S, S - 1)
        for c in ctxs[:k]:
            c.synchronize()
        walls.append((time.perf_counter() - t) * 1e3)
        if stamps:
            lib.lislam_debug_engine_stamps(st_buf.ctypes.data)
            rows = st_buf[st_buf[:, 5] > 0]
            t0 = int(rows[:, 3].min()) if len(rows) else 0
            desc = []
            for r_ in rows:  # ms from the first item start: role start-end @xcd, items first/last start, end
                f = lambda v: (int(v) - t0) / 1e5
                desc.append(f"[zero {f(r_[7]):.1f}@x{int(r_[8]) - 1} rwg {f(r_[10]):.1f}/{f(r_[9]):.1f} role {f(r_[0]):.1f}-{f(r_[1]):.1f} x{int(r_[2]) - 1} items {f(r_[3]):.1f}/{f(r_[4]):.1f} n{int(r_[5])} end {f(r_[6]):.1f}]")
            stamp_rows.append(" ".join(desc))
        row = []
        for b in bats[:k]:
            ms, _, _ = b.kernel_times()
            b.set_timing(False)
            row.append(float(ms[6]))
        per.append(row)
    bad = sum(int(np.max(np.abs(b.download(pkg.native.OUT_POSE, S - 1) - ref)) > 1e-9) for b in bats[:k])
    aborts = sum(b.odometry_status() for b in bats[:k])
    print(f"K={k}: wall ms per rep {' '.join(f'{w:.1f}' for w in walls)}; chains/s {k * REPS * 1e3 / sum(walls):.1f}; "
          f"aborts {aborts}; pose mismatches {bad}", flush=True)
    for r, row in enumerate(per):
        print(f"   rep {r}: chain ms " + " ".join(f"{x:.1f}" for x in row), flush=True)
        if stamps:
            print("      " + stamp_rows[r], flush=True)
for b in bats:
    b.close()
for c in ctxs + idle:
    c.close()
