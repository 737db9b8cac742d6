import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import __graft_entry__ as g
pkg = g.package()
if os.environ.get('LISLAM_ALT_LIB'):
    pkg.native.load(os.environ['LISLAM_ALT_LIB'])  # a developer variant of the library
S = int(sys.argv[1]) if len(sys.argv) > 1 else 8
L = int(sys.argv[2]) if len(sys.argv) > 2 else 4
scans = pkg.synth.make_sequence(S)
ctx = pkg.Context()
b = pkg.Batch(ctx, S)
b.upload(scans)
b.extract(S); b.odometry(S, L); ctx.synchronize()
b.set_timing(True)
t=time.perf_counter()
for _ in range(3):
    b.extract(S); b.odometry(S, L)
ctx.synchronize(); el=(time.perf_counter()-t)/3
ms, la, calls = b.kernel_times()
print(f'S={S} L={L} step {el*1e3:.2f} ms -> {S/el:.0f} scans/s', flush=True)
for k, m, l in zip(pkg.native.KERNELS, ms, la): print(f'  {k:16s} {m:9.3f} ms/step {l:5d} launches', flush=True)
