"""Developer diagnostic (GPU box): tests/test_gpu_parity.py::test_odometry_node_stream_api step by
step — each frame's para / stats against the oracle chain, and the batch path over the same 5 scans
(one chain of 4 pairs) for comparison."""
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, os.path.join(_R, "oracle"))
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
import oracle  # noqa: E402

ctx = pkg.Context(n_scans=64, width=1024)
scans = pkg.synth.make_sequence(5, start=40)
feats = [oracle.scan_registration(s) for s in scans]
pose, rel, st = oracle.odometry_chain(feats)
node = pkg.LaserOdometry(ctx)
for k, f in enumerate(feats):
    para, pw, gst = node.step(f)
    print("node k", k, "dpara %.3g" % np.max(np.abs(para - rel[k])), "gpu stats", list(gst[:8]), "oracle", list(st[k][:8]))
b = pkg.Batch(ctx, 5)
b.upload(scans)
b.extract(5)
b.odometry(5, 4)
ctx.synchronize()
for k in range(1, 5):
    para = b.download(pkg.native.OUT_PARA, k)
    gst = b.download(pkg.native.OUT_STATS, k)
    print("batch k", k, "dpara %.3g" % np.max(np.abs(para - rel[k])), "gpu stats", list(gst[:8]), "engine", b.odometry_engine())
