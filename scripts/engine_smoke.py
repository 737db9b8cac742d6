"""Developer tool (GPU box): the chain engine on growing continuous chains, with progress lines,
the engine status word and the oracle comparison.  usage: python scripts/engine_smoke.py S1 S2 ..."""
import os
import sys
import time

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, os.path.join(_R, "oracle"))
import __graft_entry__ as g  # noqa: E402
import oracle as O  # noqa: E402  checker only

pkg = g.package()
t0 = time.time()


def log(*a):
    print(f"[{time.time() - t0:7.2f}s]", *a, flush=True)


sizes = [int(v) for v in sys.argv[1:]] or [3, 12]
with pkg.Context() as ctx:
    for S in sizes:
        scans = pkg.synth.make_sequence(S, start=100)
        log(f"S={S}: synth done")
        feats = [O.scan_registration(s) for s in scans]
        pose, rel, st = O.odometry_chain(feats)
        log("oracle done")
        for name, mode in (("engine", ctx.ENGINE_ON), ("rounds", ctx.ENGINE_OFF)):
            ctx.set_odometry_schedule(mode)
            b = pkg.Batch(ctx, S)
            b.upload(scans)
            b.extract(S)
            ctx.synchronize()
            t = time.perf_counter()
            b.odometry(S, S - 1)
            ctx.synchronize()
            el = time.perf_counter() - t
            status = b.odometry_status()
            worst, nst = 0.0, 0
            for k in range(1, S):
                d = max(np.max(np.abs(b.download(pkg.native.OUT_PARA, k) - rel[k])),
                        np.max(np.abs(b.download(pkg.native.OUT_POSE, k) - pose[k])))
                worst = max(worst, d)
                nst += int(not np.array_equal(b.download(pkg.native.OUT_STATS, k)[:6], st[k][:6]))
            log(f"  {name}: {el * 1e3:.2f} ms, status {status}, max |delta| {worst:.3g}, stats mismatches {nst}")
            b.close()
