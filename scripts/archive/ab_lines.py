"""A/B timing of library variants (developer tool, GPU box).

    python scripts/archive/ab_lines.py [--scans 300] [--chain 10] [--odometry] main scripts/_ab/liblislam_x.so ...

Generates the seeded 300-scan batch once (spawn pool, cached in /tmp), then runs each library in
its own child process: extraction (and odometry with --odometry) repeated, per-kernel HIP-event
times printed, and the less-flat / sharp clouds and odometry outputs compared with the first
library's (bit-exact)."""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

CACHE = "/tmp/lislam_ab_scans.npy"


def child(lib: str, n: int, chain: int, odo: bool, reps: int, out: str):
    import __graft_entry__ as g
    pkg = g.package()
    if lib != "main":
        pkg.native.load(lib)
    scans = np.load(CACHE, mmap_mode="r")[:n]
    ctx = pkg.Context()
    if os.environ.get("LISLAM_AB_TIES") == "index":
        ctx.set_tie_order(ctx.TIES_INDEX)
    b = pkg.Batch(ctx, n)
    b.upload(np.ascontiguousarray(scans))
    b.extract(n)
    if odo:
        b.odometry(n, chain)
    ctx.synchronize()
    b.set_timing(True)
    t = time.perf_counter()
    for _ in range(reps):
        b.extract(n)
        if odo:
            b.odometry(n, chain)
    ctx.synchronize()
    el = (time.perf_counter() - t) / reps
    ms, la, _ = b.kernel_times()
    line = f"{os.path.basename(lib):28s} step {el * 1e3:7.3f} ms |"
    for k, m, l in zip(pkg.native.KERNELS, ms, la):
        if l:
            line += f" {k} {m:.3f}"
    print(line, flush=True)
    nat = pkg.native
    if hasattr(ctx.lib, "lislam_debug_heap_counts"):  # the counting variant (scripts/build_variant.sh)
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        ctx.lib.lislam_debug_heap_counts(buf)
        calls = reps + 1
        print(f"  heap fallbacks per batch: LDS {buf[0] / calls:.0f} calls, {buf[1] / calls:.0f} elements; "
              f"register {buf[2] / calls:.0f} calls, {buf[3] / calls:.0f} elements", flush=True)
    res = {}
    for k in range(0, n, max(1, n // 16)):
        for what in (nat.OUT_LESS_FLAT, nat.OUT_SHARP, nat.OUT_LESS_SHARP, nat.OUT_FLAT):
            res[f"f{what}_{k}"] = b.download(what, k)
        if odo:
            res[f"pose_{k}"] = b.download(nat.OUT_POSE, k)
    np.savez(out, **res)
    b.close()
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--scans", type=int, default=300)
    ap.add_argument("--chain", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--odometry", action="store_true")
    ap.add_argument("--child", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.scans, a.chain, a.odometry, a.reps, a.out)
        return
    if not os.path.exists(CACHE) or np.load(CACHE, mmap_mode="r").shape[0] < a.scans:
        import bench
        np.save(CACHE, bench.generate(0, a.scans, 64, 1024, 16))
    first = None
    for i, lib in enumerate(a.libs):
        out = f"/tmp/lislam_ab_{i}.npz"
        cmd = [sys.executable, __file__, "--child", lib, "--out", out, "--scans", str(a.scans), "--chain", str(a.chain),
               "--reps", str(a.reps)] + (["--odometry"] if a.odometry else [])
        r = subprocess.run(cmd, timeout=300)
        if r.returncode != 0:
            print(f"{lib}: exit {r.returncode}", flush=True)
            sys.exit(r.returncode)
        got = np.load(out)
        if first is None:
            first = got
            continue
        bad = [k for k in first.files if not np.array_equal(first[k], got[k])]
        print(f"  vs first: {'identical' if not bad else 'DIFFERS in ' + ','.join(bad[:6])}", flush=True)


if __name__ == "__main__":
    main()
