"""Per-phase cycle breakdown of k_scan_lines (developer tool).

Builds a variant of liblislam with -DLISLAM_PHASE_PROF into scripts/_prof/ (run the build step
on the CPU container: `python scripts/phase_prof.py build`), then on the GPU box
`python scripts/phase_prof.py run S` extracts S synthetic scans and prints the summed cycles of
each phase over all lines.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

OUT = os.path.join(ROOT, "scripts", "_prof", "liblislam_prof.so")
PHASES = ["curv+links", "seg sort", "sharp walk", "flat walk", "lessflat list", "label/feature writes",
          "voxel keys", "voxel sort", "voxel centroids"]

if sys.argv[1] == "build":
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    srcs = [os.path.join(g.CSRC, s) for s in g.HIP_SOURCES]
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *g.HIPCC_FLAGS, "-DLISLAM_PHASE_PROF", "-o", OUT,
                    *srcs], check=True, cwd=g.CSRC)
    sys.exit(0)

pkg = g.package()
L = pkg.native.load(OUT)
S = int(sys.argv[2]) if len(sys.argv) > 2 else 100
scans = pkg.synth.make_sequence(S)
buf = (ctypes.c_ulonglong * 16)()
with pkg.Context() as ctx:
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    ctx.synchronize()
    L.lislam_debug_phase_cycles(buf)  # reset after the warm-up
    b.extract(S)
    ctx.synchronize()
    L.lislam_debug_phase_cycles(buf)
    tot = sum(buf[i] for i in range(len(PHASES)))
    nl = S * 64
    for i, n in enumerate(PHASES):
        print(f"{n:22s} {buf[i] / nl:12.0f} cycles/line  {100 * buf[i] / max(tot, 1):5.1f}%")
    # association search statistics over one odometry pass
    b.odometry(S, 10)
    ctx.synchronize()
    L.lislam_debug_assoc_stats(buf)
    b.odometry(S, 10)
    ctx.synchronize()
    L.lislam_debug_assoc_stats(buf)
    names = ["nn queries (>=1 super in range)", "nn extra super batches", "nn chunk batches", "-", "ls windows",
             "ls first batches", "ls corner batches", "ls surf batches", "corner queries", "surf queries",
             "corner with closest", "surf with closest"]
    for i, n in enumerate(names):
        print(f"{n:34s} {buf[i]}")
    b.close()
