import sys, time, os
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import numpy as np
import __graft_entry__ as g
pkg = g.package()
import oracle as O
t=time.time()
g.smoke()
print('smoke time', time.time()-t, flush=True)
S=8
scans = pkg.synth.make_sequence(S)
ctx = pkg.Context()
b = pkg.Batch(ctx, S)
b.upload(scans)
b.set_timing(True)
b.extract(S); b.odometry(S, 4)
ctx.synchronize()
print('kernel ms', b.kernel_times(), flush=True)
feats=[O.scan_registration(s) for s in scans]
bad=0
for k in range(S):
    gf=b.features(k); r=feats[k]
    for name in ("laser_cloud","sharp","less_sharp","flat","less_flat"):
        a, rr = getattr(gf,name), getattr(r,name)
        same = a.shape==rr.shape and np.array_equal(a[:,:3], rr[:,:3])
        di = np.max(np.abs(a[:,3]-rr[:,3])) if a.shape==rr.shape and a.size else 0
        if not same or di>1e-6: bad+=1; print('MISMATCH', k, name, a.shape, rr.shape, di)
    c=b.download(pkg.native.OUT_CURVATURE,k); 
    if not np.array_equal(c, r.curvature): print('curv mismatch', k, np.abs(c-r.curvature).max())
    l=b.download(pkg.native.OUT_LABEL,k)
    if not np.array_equal(l, r.label): print('label mismatch', k, (l!=r.label).sum())
    ir=b.download(pkg.native.OUT_IMAGE_RANGE,k); ii=b.download(pkg.native.OUT_IMAGE_INTENSITY,k); tr=b.download(pkg.native.OUT_CLOUD_TRACK,k)
    if not (np.array_equal(ir, r.img_range.ravel()) and np.array_equal(ii, r.img_intensity.ravel()) and np.array_equal(tr, r.cloud_track.reshape(-1,4))): print('image mismatch', k)
print('feature mismatches', bad)
for c0 in range(0, S-1, 4):
    ch = feats[c0:c0+5]
    pose, rel, st = O.odometry_chain(ch)
    for j in range(1, len(ch)):
        k=c0+j
        para=b.download(pkg.native.OUT_PARA,k); gst=b.download(pkg.native.OUT_STATS,k)
        print(k, 'dpara', np.abs(para-rel[j]).max(), 'stats gpu', gst, 'cpu', st[j])
