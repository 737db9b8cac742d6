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

OUT = os.environ.get("LISLAM_PROF_LIB", os.path.join(ROOT, "scripts", "_prof", "liblislam_prof.so"))
PHASES = ["curv+links", "seg sort", "sharp walk", "flat walk", "lessflat list", "label/feature writes",
          "voxel keys", "voxel sort", "voxel centroids", "voxel numbering sort", "voxel numbering",
          "voxel final positions + permutation", "voxel introsort loop",
          "(count) introsort heap-sort fallbacks", "(count) register partitions", "(count) LDS partitions"]

if sys.argv[1] == "build":
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    srcs = [os.path.join(g.CSRC, s) for s in g.HIP_SOURCES]
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *g.HIPCC_FLAGS, "-DLISLAM_PHASE_PROF", "-o", OUT,
                    *srcs], check=True, cwd=g.CSRC)
    sys.exit(0)

if sys.argv[1] == "lm":  # k_odom_lm: first evaluation + start, later evaluations, step logic
    pkg = g.package()
    L = pkg.native.load(OUT)
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    scans = pkg.synth.make_sequence(S)
    buf = (ctypes.c_ulonglong * 8)()
    with pkg.Context() as ctx:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, 10)
        ctx.synchronize()
        L.lislam_debug_lm_phases(buf)
        b.odometry(S, 10)
        ctx.synchronize()
        L.lislam_debug_lm_phases(buf)
        nwg = 2 * 10 * ((S - 1 + 9) // 10)
        names = ["first eval (+ start, v1)", "evaluations", "steps (thread 0)", "record load + counts (v2)"]
        for i, nm in enumerate(names):
            print(f"{nm:26s} {buf[i] / 100.0 / nwg:9.1f} us per workgroup")
        print(f"{'later evaluations':26s} {buf[5] / nwg:9.2f} per workgroup")
        b.close()
    sys.exit(0)

if sys.argv[1] == "lines":  # per-wave timeline of one k_scan_lines launch
    import numpy as np
    import torch

    pkg = g.package()
    L = pkg.native.load(OUT)
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    scans = pkg.synth.make_sequence(S)
    with pkg.Context() as ctx:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        ctx.synchronize()
        H = 64
        log = torch.zeros(S * H * 4, dtype=torch.int64, device="cuda")
        L.lislam_debug_line_log(ctypes.c_void_p(log.data_ptr()))
        buf = (ctypes.c_ulonglong * 16)()
        L.lislam_debug_phase_cycles(buf)
        b.extract(S)
        ctx.synchronize()
        L.lislam_debug_line_log(ctypes.c_void_p(0))
        L.lislam_debug_phase_cycles(buf)
        a = log.view(-1, 4).cpu().numpy()
        t0 = a[:, 0].min()
        st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0
        d = en - st
        print(f"waves {len(a)}  span {en.max():.1f} us  duration us: p50 {np.median(d):.1f} p90 "
              f"{np.percentile(d, 90):.1f} p99 {np.percentile(d, 99):.1f} max {d.max():.1f}  mean {d.mean():.1f}")
        print(f"start us: p50 {np.median(st):.1f} p90 {np.percentile(st, 90):.1f} max {st.max():.1f}")
        print(f"sum of wave durations {d.sum() / 1e3:.1f} ms; waves alive at t: " +
              " ".join(f"{t:.0f}:{int(((st <= t) & (en > t)).sum())}" for t in np.linspace(0, en.max(), 12)))
        order = np.argsort(-d)[:12]
        print("longest waves (us, len, start):", [(round(float(d[i]), 1), int(a[i, 2]), round(float(st[i]), 1))
                                                  for i in order])
        sc = np.arange(len(a)) // H
        print("by scan (30-scan bins): mean / p90 us:",
              [(int(b0), round(float(d[(sc >= b0) & (sc < b0 + 30)].mean()), 1),
                round(float(np.percentile(d[(sc >= b0) & (sc < b0 + 30)], 90)), 1)) for b0 in range(0, S, 30)])
        print("by line (8-line bins): mean us:",
              [(int(l0), round(float(d[(np.arange(len(a)) % H >= l0) & (np.arange(len(a)) % H < l0 + 8)].mean()), 1))
               for l0 in range(0, H, 8)])
        sb = np.linspace(0, st.max() + 1e-6, 9)
        print("by start time: mean us:", [(round(float(x0)), round(float(d[(st >= x0) & (st < x1)].mean()), 1))
                                          for x0, x1 in zip(sb, sb[1:]) if ((st >= x0) & (st < x1)).any()])
        lens = a[:, 2]
        for lo_, hi_ in ((0, 600), (600, 800), (800, 950), (950, 1024), (1024, 5000)):
            m = (lens >= lo_) & (lens < hi_)
            if m.any():
                print(f"len [{lo_},{hi_}): {m.sum()} waves, mean {d[m].mean():.1f} us, max {d[m].max():.1f} us")
        tot = sum(buf[i] for i in range(min(len(PHASES), 13)))
        for i, nm in enumerate(PHASES):
            print(f"{nm:28s} {buf[i] / (S * H):10.0f} cycles/line {100.0 * buf[i] / max(tot, 1):5.1f}%")
        b.close()
    sys.exit(0)

if sys.argv[1] == "waves":  # per-wave timeline of one association launch (round R, outer pass 1)
    import numpy as np
    import torch

    pkg = g.package()
    L = pkg.native.load(OUT)
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    scans = pkg.synth.make_sequence(S)
    with pkg.Context() as ctx:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, 10)
        ctx.synchronize()
        log = torch.zeros(4 * 4 * 2000 * 1000, dtype=torch.int64, device="cuda")
        L.lislam_debug_wave_log(ctypes.c_void_p(log.data_ptr()), R)
        b.odometry(S, 10)
        ctx.synchronize()
        L.lislam_debug_wave_log(ctypes.c_void_p(0), -1)
        a = log.view(-1, 4).cpu().numpy()
        a = a[a[:, 0] != 0]
        t0 = a[:, 0].min()
        st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # 100 MHz -> us
        d = en - st
        kind = a[:, 2] & 0xff
        print(f"waves {len(a)}  span {en.max():.1f} us  start: p50 {np.median(st):.1f} p99 {np.percentile(st, 99):.1f} "
              f"max {st.max():.1f}")
        for k, nm in ((1, "corner"), (2, "surf")):
            dk = d[kind == k]
            print(f"  {nm:6s} n={len(dk)} dur us: p50 {np.median(dk):.1f} p90 {np.percentile(dk, 90):.1f} "
                  f"p99 {np.percentile(dk, 99):.1f} max {dk.max():.1f}  sum {dk.sum():.0f}")
        top = np.argsort(-d)[:10]
        for i in top:
            print(f"    slow: kind {kind[i]} chain {(a[i, 2] >> 8) & 0xffffff} q {a[i, 2] >> 32} start {st[i]:.1f} "
                  f"dur {d[i]:.1f} nL {a[i, 3]}")
        hist, edges = np.histogram(en, bins=20)
        print("  end-time histogram:", list(hist))
        b.close()
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
