"""Timeline summary of a rocprofv3 kernel trace (developer tool): where the blit copies fall and how
busy the device is between extract calls.  Usage: python scripts/trace_timeline.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
t0 = ev[0][0]
fc = [e for e in ev if "k_front_count" in e[2]]
print("k_front_count starts (ms):", [round((e[0] - t0) / 1e6, 2) for e in fc])
cp = [e for e in ev if "copyBuffer" in e[2]]
b = collections.Counter(int((e[0] - t0) / 1e6 // 50) for e in cp)
print("copies per 50 ms bucket:", sorted(b.items()))
print("span ms", round((ev[-1][1] - t0) / 1e6, 2))
# busy fraction (union of kernel intervals) between consecutive k_front_count launches
for a, z in zip(fc, fc[1:]):
    iv = sorted((s, e) for s, e, n in ev if s >= a[0] and s < z[0])
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = z[0] - a[0]
    ncp = sum(1 for s, e, n in ev if s >= a[0] and s < z[0] and "copyBuffer" in n)
    print(f"window {round((a[0] - t0) / 1e6, 2)} ms: span {span / 1e6:.2f} ms busy {busy / 1e6:.2f} ms copies {ncp}")
