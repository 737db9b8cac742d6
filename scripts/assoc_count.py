"""Round-trip counters of k_odom_assoc (developer tool): builds a -DLISLAM_ASSOC_COUNT variant into
scripts/_prof/liblislam_count.so (`build`, on the CPU container), then `run S` on the GPU box runs
one odometry pass over S synthetic scans and prints the per-query averages of each counter."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

OUT = os.environ.get("LISLAM_COUNT_LIB", os.path.join(ROOT, "scripts", "_prof", "liblislam_count.so"))
NAMES = ["nn: candidate super-chunk", "nn: super-chunk rounds", "nn: chunk rounds", "nn: speculative bounds", "ls: windows",
         "ls: first batch", "ls corner: batch rounds", "ls surf: batch rounds", "corner queries", "surf queries",
         "corner with closest", "surf with closest"]

if sys.argv[1] == "build":
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    srcs = [os.path.join(g.CSRC, s) for s in g.HIP_SOURCES]
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *g.HIPCC_FLAGS, "-DLISLAM_PHASE_PROF", "-DLISLAM_ASSOC_COUNT", "-o", OUT,
                    *srcs], check=True, cwd=g.CSRC)
    sys.exit(0)

pkg = g.package()
L = pkg.native.load(OUT)
S = int(sys.argv[2]) if len(sys.argv) > 2 else 300
scans = pkg.synth.make_sequence(S)
buf = (ctypes.c_ulonglong * 16)()
with pkg.Context() as ctx:
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    ctx.synchronize()
    L.lislam_debug_assoc_stats(buf)
    b.odometry(S, 10)
    ctx.synchronize()
    L.lislam_debug_assoc_stats(buf)
nq = buf[8] + buf[9]
for i, n in enumerate(NAMES):
    if n != "-":
        print(f"{n:28s} {buf[i]:12d}  per query {buf[i] / max(nq, 1):8.3f}")
