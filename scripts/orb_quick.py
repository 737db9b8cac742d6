"""Time the ORB batch path (a8-a11) on a 300-scan synthetic batch, per kernel (GPU box)."""
import sys, time
import os; _R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, 'oracle'))
import numpy as np
import __graft_entry__ as g
pkg = g.package()
if os.environ.get('LISLAM_ALT_LIB'):
    pkg.native.load(os.environ['LISLAM_ALT_LIB'])  # a developer variant of the library
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
scans = np.load('/tmp/lislam_scans.r0.npy')[:S] if len(sys.argv) > 2 else pkg.synth.make_sequence(S)
ctx = pkg.Context()
b = pkg.Batch(ctx, S)
b.upload(scans)
b.extract(S)
mask = pkg.intensity.set_mask()
b.intensity_odometry(S, 1000, mask)
ctx.synchronize()
pkg.mapping.kernel_times(ctx)
pkg.mapping.set_timing(ctx, True)
t = time.perf_counter()
for _ in range(3):
    b.intensity_odometry(S, 1000, mask)
ctx.synchronize()
el = (time.perf_counter() - t) / 3
kt = pkg.mapping.kernel_times(ctx)
print(f'S={S} intensity odometry {el*1e3:.2f} ms/batch -> {S/el:.0f} scans/s', flush=True)
for k, (ms, n) in kt.items():
    if n: print(f'  {k:16s} {ms/3:9.3f} ms/batch {n/3:6.1f} launches', flush=True)
st = np.stack([b.download(pkg.native.OUT_ORB_STATS, k) for k in range(S)])
print('good', (st[:, 0] == 1).sum(), 'redetect', st[:, 1].sum(), 'kp mean', st[:, 2].mean(), 'good matches', st[1:, 4].mean())
L = pkg.native.load()
if hasattr(L, 'lislam_debug_sel_phases'):  # profiling build: k_orb_select phase split (WG-summed us)
    import ctypes
    buf = (ctypes.c_ulonglong * 8)()
    L.lislam_debug_sel_phases(buf)
    L.lislam_debug_sel_phases(buf)  # (cleared above; read what the next batch adds)
    b.intensity_odometry(S, 1000, mask)
    ctx.synchronize()
    L.lislam_debug_sel_phases(buf)
    names = ['compact', 'retain2n', 'harris', 'retainN', 'angles']
    tot = sum(buf[i] for i in range(5))
    for i, nm in enumerate(names):
        print(f'  select {nm:9s} {buf[i] / 100.0:12.0f} WG-us  {100 * buf[i] / max(1, tot):5.1f}%')
if hasattr(L, 'lislam_debug_pyr_phases'):  # profiling build: k_orb_pyramid phase split (per-WG us)
    import ctypes
    buf = (ctypes.c_ulonglong * 32)()
    L.lislam_debug_pyr_phases(buf)
    b.intensity_odometry(S, 1000, mask)
    ctx.synchronize()
    L.lislam_debug_pyr_phases(buf)
    print(f'  pyramid load        {buf[0] / 100.0 / S:8.2f} us per WG')
    for p, nm in ((1, 'resize'), (2, 'padded'), (3, 'blur')):
        row = ' '.join(f'{buf[8 * p + l] / 100.0 / S:6.2f}' for l in range(8))
        tot = sum(buf[8 * p + l] for l in range(8)) / 100.0 / S
        print(f'  pyramid {nm:8s} {tot:8.2f} us per WG  (levels: {row})')
