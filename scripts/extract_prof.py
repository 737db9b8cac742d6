"""Developer tool (GPU box): the feature extraction + target index of one synthetic batch, a few
times, for rocprofv3 kernel traces / PMC passes of the streaming kernels alone.
usage: python scripts/extract_prof.py [S] [REPS] [H] [W]"""
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
if os.environ.get("LISLAM_ALT_LIB"):  # a developer variant of the library (A/B)
    pkg.native.load(os.environ["LISLAM_ALT_LIB"])
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
W = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
cache = f"/tmp/lislam_extract_scans_{S}_{H}_{W}.npy"
if os.path.exists(cache):
    scans = np.load(cache)
else:
    scans = pkg.synth.make_sequence(S, H, W)
    np.save(cache, scans)
with pkg.Context(n_scans=H, width=W) as ctx:
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    for _ in range(REPS):
        b.extract(S)
    ctx.synchronize()
    n = pkg.native
    lf = [b.count(n.OUT_LESS_FLAT, k) for k in range(S)]
    ls = [b.count(n.OUT_LESS_SHARP, k) for k in range(S)]
    print(f"{S} scans x {REPS}: less-flat per scan mean {np.mean(lf):.0f} max {max(lf)}, less-sharp mean {np.mean(ls):.0f}")
    b.close()
