"""Developer tool (GPU box): time one continuous odometry chain over a synthetic batch with both
schedules (per-round launches / persistent engine) and compare their outputs.
usage: python scripts/chain_quick.py [S] [REPS]"""
import os
import sys
import time

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
if os.environ.get("LISLAM_ALT_LIB"):
    pkg.native.load(os.environ["LISLAM_ALT_LIB"])  # a developer variant of the library
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cache = f"/tmp/lislam_chain_scans_{S}.npy"
if os.path.exists(cache):
    scans = np.load(cache)
else:
    scans = pkg.synth.make_sequence(S)
    np.save(cache, scans)
with pkg.Context() as ctx:
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    ctx.synchronize()
    res = {}
    modes = (("engine", ctx.ENGINE_ON),) if os.environ.get("CHAIN_ENGINE_ONLY") else (("engine", ctx.ENGINE_ON), ("rounds", ctx.ENGINE_OFF))
    for name, mode in modes:
        ctx.set_odometry_schedule(mode)
        b.odometry(S, S - 1)
        ctx.synchronize()
        b.set_timing(True)
        t = time.perf_counter()
        for _ in range(REPS):
            b.odometry(S, S - 1)
        ctx.synchronize()
        el = (time.perf_counter() - t) / REPS
        ms, la, calls = b.kernel_times()
        b.set_timing(False)
        print(f"{name}: {el * 1e3:.3f} ms per {S}-scan chain = {S / el:.0f} scans/s; "
              + ", ".join(f"{k} {m:.3f} ms x{l}" for k, m, l in zip(pkg.native.KERNELS, ms, la) if l), flush=True)
        res[name] = np.array([np.concatenate([b.download(pkg.native.OUT_PARA, k), b.download(pkg.native.OUT_POSE, k)])
                              for k in range(S)])
        st = np.array([b.download(pkg.native.OUT_STATS, k) for k in range(S)])
        res[name + "_st"] = st
    if "rounds" not in res:
        ref = os.environ.get("CHAIN_REF")
        if ref and os.path.exists(ref):
            z = np.load(ref)
            print(f"engine vs {ref}: max |para/pose delta| {np.max(np.abs(res['engine'] - z['p'])):.3g}, "
                  f"stats mismatches {int(np.sum(np.any(res['engine_st'][:, :6] != z['st'][:, :6], axis=1)))}", flush=True)
        elif ref:
            np.savez(ref, p=res["engine"], st=res["engine_st"])
        b.close()
        sys.exit(0)
    d = np.max(np.abs(res["engine"] - res["rounds"]))
    nst = int(np.sum(np.any(res["engine_st"][:, :6] != res["rounds_st"][:, :6], axis=1)))
    print(f"engine vs rounds: max |para/pose delta| {d:.3g}, stats mismatches {nst}", flush=True)
    b.close()
