"""Time the odometry stage alone (a12-a18) on a 300-scan synthetic batch (developer tool, GPU box):
extraction once, then REPS x lislam_batch_odometry(S, 10) with per-kernel event timing.
LISLAM_ALT_LIB selects a developer variant of the library."""
import os
import sys
import time

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
if os.environ.get("LISLAM_ALT_LIB"):
    pkg.native.load(os.environ["LISLAM_ALT_LIB"])
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
scans = pkg.synth.make_sequence(S)
with pkg.Context() as ctx:
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, 10)
    ctx.synchronize()
    b.set_timing(True) if hasattr(b, "set_timing") else None
    t = time.perf_counter()
    for _ in range(REPS):
        b.odometry(S, 10)
    ctx.synchronize()
    el = (time.perf_counter() - t) / REPS
    print(f"odometry {el * 1e3:.3f} ms per {S}-scan batch", flush=True)
    if hasattr(b, "kernel_times"):
        print(b.kernel_times(), flush=True)
    b.close()
