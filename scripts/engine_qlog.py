"""Developer tool (GPU box): per-query 1-NN / line-search times of one pair of a continuous chain
through the engine, and what the slow queries have in common.  usage: engine_qlog.py [S] [pair]"""
import ctypes
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
PAIR = int(sys.argv[2]) if len(sys.argv) > 2 else 150
cache = f"/tmp/lislam_chain_scans_{S}.npy"
scans = np.load(cache) if os.path.exists(cache) else pkg.synth.make_sequence(S)
if not os.path.exists(cache):
    np.save(cache, scans)
cap = 12 * 64 + 24 * 64
with pkg.Context() as ctx:
    lib = ctx.lib
    lib.lislam_debug_engine_qlog.argtypes = [ctypes.c_void_p, ctypes.c_int]
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(2 * cap * 16)) == 0
    hip.hipMemset(buf, ctypes.c_int(0xff), ctypes.c_size_t(2 * cap * 16))
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    ctx.synchronize()
    assert lib.lislam_debug_engine_qlog(buf, PAIR) == 0
    b.odometry(S, S - 1)
    ctx.synchronize()
    lib.lislam_debug_engine_qlog(None, -1)
    q = np.zeros(2 * cap * 4, np.int32)
    hip.hipMemcpy(q.ctypes.data_as(ctypes.c_void_p), buf, ctypes.c_size_t(q.nbytes), ctypes.c_int(2))
    q = q.reshape(2, cap, 4)
    n = pkg.native
    ns, nf = b.count(n.OUT_SHARP, PAIR), b.count(n.OUT_FLAT, PAIR)
    for outer in (0, 1):
        v = q[outer, :ns + nf]
        t = (v[:, 0] + v[:, 1]) * 0.01
        print(f"pair {PAIR} outer {outer}: {ns} corner + {nf} surf queries; query time us: p50 {np.median(t):.2f} "
              f"p90 {np.percentile(t, 90):.2f} p99 {np.percentile(t, 99):.2f} max {t.max():.2f}")
        print(f"  1-NN p50 {np.median(v[:, 0]) * 0.01:.2f} max {v[:, 0].max() * 0.01:.2f}; line p50 "
              f"{np.median(v[:, 1]) * 0.01:.2f} max {v[:, 1].max() * 0.01:.2f}")
        slow = np.argsort(-t)[:12]
        for i in slow:
            print(f"   query {i}: {'corner' if i < ns else 'surf'} nn {v[i, 0] * 0.01:.2f} ls {v[i, 1] * 0.01:.2f} "
                  f"closest {v[i, 2]} kind {v[i, 3]}")
        nokind = np.sum(v[:, 2] < 0)
        print(f"  queries without a 1-NN: {nokind}; their time p50 {np.median(t[v[:, 2] < 0]) if nokind else 0:.2f}")
    b.close()
