"""Developer tool (GPU box): per-line label differences between the GPU extraction and the oracle's
tie modes on a snapped synthetic scan.  usage: python scripts/ties_debug.py [start] [quantum]"""
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, os.path.join(_R, "oracle"))
import __graft_entry__ as g  # noqa: E402
import oracle as O  # noqa: E402

pkg = g.package()
start = int(sys.argv[1]) if len(sys.argv) > 1 else 40
q = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
scans = pkg.synth.make_sequence(2, start=start).copy()
xyz = scans[..., :3]
nz = np.abs(xyz).sum(-1) > 0
xyz[nz] = np.round(xyz[nz] / q) * q
with pkg.Context() as ctx:
    b = pkg.Batch(ctx, 2)
    b.upload(scans)
    b.extract(2)
    for k in range(2):
        lab = b.download(pkg.native.OUT_LABEL, k)
        lo = b.download(pkg.native.OUT_LINE_OFFSETS, k)
        r0 = O.scan_registration(scans[k], ties=0)
        r1 = O.scan_registration(scans[k], ties=1)
        print(f"scan {k}: label diffs vs ties0 {int(np.sum(lab != r0.label))}, vs ties1 {int(np.sum(lab != r1.label))}")
        for ln in range(len(lo) - 1):
            a, e = lo[ln], lo[ln + 1]
            d0 = int(np.sum(lab[a:e] != r0.label[a:e]))
            d1 = int(np.sum(lab[a:e] != r1.label[a:e]))
            if d0:
                idx = np.nonzero(lab[a:e] != r0.label[a:e])[0]
                print(f"  line {ln} len {e - a}: diffs vs ties0 {d0} (first at {idx[:8]}), vs ties1 {d1}")
    b.close()

# the feature clouds, first differing rows; the batch's scratch first holds another extraction
with pkg.Context() as ctx:
    b = pkg.Batch(ctx, 2)
    if os.environ.get("DIRTY"):
        b.upload(pkg.synth.make_sequence(2, start=70))
        b.extract(2)
    b.upload(scans)
    b.extract(2)
    for k in range(2):
        gf = b.features(k)
        r0 = O.scan_registration(scans[k], ties=0)
        for name in ("sharp", "less_sharp", "flat", "less_flat"):
            a_, r_ = getattr(gf, name), getattr(r0, name)
            if a_.shape != r_.shape:
                print(k, name, "shape", a_.shape, r_.shape)
                continue
            bad = np.nonzero(np.any(a_ != r_, axis=1))[0]
            print(k, name, "rows differing", len(bad), bad[:10])
            for i in bad[:4]:
                print("   gpu", a_[i], "oracle", r_[i])
    b.close()
