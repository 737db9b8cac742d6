"""Time the batch ground extraction and (profiling build) the k_ground_ransac phase split."""
import ctypes, os, sys, time
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, _R)
import __graft_entry__ as g
pkg = g.package()
if os.environ.get('LISLAM_ALT_LIB'):
    pkg.native.load(os.environ['LISLAM_ALT_LIB'])
L = pkg.native.load()
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
scans = pkg.synth.make_sequence(S)
ctx = pkg.Context()
b = pkg.Batch(ctx, S)
b.upload(scans)
b.ground(S)
ctx.synchronize()
buf = (ctypes.c_ulonglong * 8)()
if hasattr(L, 'lislam_debug_ground_phases'):
    L.lislam_debug_ground_phases(buf)
t = time.perf_counter()
b.ground(S)
ctx.synchronize()
print(f'S={S} ground {1e3 * (time.perf_counter() - t):.3f} ms')
if hasattr(L, 'lislam_debug_ground_phases'):
    L.lislam_debug_ground_phases(buf)
    for i, nm in enumerate(['sampling', 'counting', 'replay+refit sums', 'eigen33']):
        print(f'  {nm:18s} {buf[i] / 100.0 / S:9.1f} us per WG')
