"""Developer tool (GPU box): the latency workload's per-call host times (bench.py --workload
latency): scan registration, the ORB tracker, the odometry node step, over 60 scans."""
import os
import sys
import time

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
H, W = 64, 1024
scans = pkg.synth.make_sequence(70)
ctx = pkg.Context(n_scans=H, width=W)
reg = pkg.ScanRegistration(ctx)
odo = pkg.LaserOdometry(ctx)
trk = pkg.intensity.IntensityTracker(ctx, H, W, 1000, pkg.intensity.set_mask(H, W))
t = {"reg": [], "orb": [], "odo": []}
for k, s in enumerate(scans):
    a = time.perf_counter()
    f = reg.laser_cloud_handler(s)
    b = time.perf_counter()
    trk.detectfeatures(f.image_intensity, f.cloud_track)
    c = time.perf_counter()
    odo.step(f)
    d = time.perf_counter()
    if k >= 10:
        t["reg"].append(b - a)
        t["orb"].append(c - b)
        t["odo"].append(d - c)
print({k: round(float(np.median(v)) * 1e3, 3) for k, v in t.items()}, "engine env", os.environ.get("LISLAM_ENGINE"))
