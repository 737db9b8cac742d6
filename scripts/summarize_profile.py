"""Summarize a profile_round.sh run (gpurun_out/<tag>) into profiles/<tag>_*.

Traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB from the
L2's memory-side request counters; on gfx950 FETCH_SIZE reads half the bytes of a wide (16 B/lane)
read stream, so it is doubled; WRITE_SIZE is taken as is.  Both come from separate --pmc passes.
"""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", tag)
dst = "profiles"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, f"{tag}_rocprof_kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))


def short(name):
    return name.split("(")[0].replace("lislam::", "")


# rocprof kernel (base name, no "void", namespaces or template arguments) -> the bench's logical
# kernel (native.KERNELS / the ORB timers); kernels of one logical name are summed per step
LOGICAL = [("k_front_", "k_scan_front"), ("k_scan_lines", "k_scan_lines"), ("k_scan_compact", "k_scan_compact"),
           ("k_target_index", "k_target_index"), ("k_odom_assoc", "k_odom_assoc"), ("k_odom_lm", "k_odom_lm"),
           ("k_odom_chain", "k_odom_chain"), ("k_odom_items", "k_odom_chain"), ("k_odom_roles", "k_odom_chain+"),
           ("k_knn", "k_knn"), ("k_fit", "k_fit"), ("k_lm_eval", "k_lm_eval"), ("k_lm_step", "k_lm_step")]


def logical(name):
    base = short(name).replace("void ", "").split("::")[-1].split("<")[0]
    for pre, lg in LOGICAL:
        if base.startswith(pre):
            return lg
    return None


def pmc(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        a = agg.setdefault(k, [0.0, 0])
        a[0] += float(r["Counter_Value"])
        a[1] += 1
    return agg


def pmc_multi(path):  # several counters in one pass: kernel -> counter -> [sum, launches]
    agg = {}
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        a = agg.setdefault(k, {}).setdefault(r["Counter_Name"], [0.0, 0])
        a[0] += float(r["Counter_Value"])
        a[1] += 1
    return agg


fetch = pmc(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"))
sq = pmc_multi(os.path.join(src, "pmc_sq", "pmc_counter_collection.csv"))
write = pmc(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"))
stats = {short(r["Name"]): r for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv")))}
bench = json.load(open(os.path.join(src, "trace_bench.json")))
bc = bench["config"]
# the odometry schedule the PMC passes ran (bench.py matches it before citing the odometry's counters)
pmc_cfg = json.load(open(os.path.join(src, "pmc_fetch.json"))).get("config", {})
out = {"tag": tag, "config": {k: bc[k] for k in ("lines", "width", "scans_per_step_per_gpu", "chain_len") if k in bc},
       "workload": bc.get("workload"), "odometry_engine": pmc_cfg.get("odometry_schedule"),
       "trace_odometry_schedule": bc.get("odometry_schedule"),
       "correction": "traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (gfx950 FETCH_SIZE "
                                 "half-count of wide reads, MI355X_MICROARCH.md HBM section)", "kernels": {}}
for k in fetch:
    if k.startswith("__amd"):
        continue
    f, nf = fetch[k]
    w, nw = write.get(k, [0.0, 1])
    per = (2 * f / nf + w / nw) * 1024
    s = stats.get(k, {})
    out["kernels"][k] = {"launches_profiled": nf, "fetch_kib_per_launch": f / nf, "write_kib_per_launch": w / nw,
                         "traffic_bytes_per_launch": per,
                         "avg_ns": float(s.get("AverageNs", 0) or 0), "calls": int(s.get("Calls", 0) or 0)}
# per logical kernel: traffic per launch of the logical kernel (its rocprof kernels' traffic per
# step / its launches per step), what bench.py's roofline line looks up.  The split chain engine is
# two concurrent launches: k_odom_items counts the launches (and sets the duration), k_odom_roles'
# traffic is added to the same engine launch ("k_odom_chain+").
steps_pmc = 1  # profile_round.sh's PMC passes run one step
lg = {}
for k in fetch:
    name = logical(k)
    if not name:
        continue
    f, nf = fetch[k]
    w, nw = write.get(k, [0.0, 1])
    a = lg.setdefault(name.rstrip("+"), [0.0, 0])
    a[0] += (2 * f + w) * 1024
    a[1] += 0 if name.endswith("+") else nf
out["kernels_logical"] = {k: {"launches_profiled": v[1], "traffic_bytes_per_launch": v[0] / max(1, v[1])}
                          for k, v in lg.items()}
# SQ counters per launch (summed over the dispatch's shader engines); the fractions of the wave
# cycles spent waiting (SQ_WAIT_ANY), waiting for instruction issue (SQ_WAIT_INST_ANY) and with an
# instruction active (SQ_ACTIVE_INST_ANY) name the bound that applies to a latency-bound kernel
for k, cs in sq.items():
    name = logical(k) or k
    if name.endswith("+"):
        name = k.replace("void ", "").split("::")[-1].split("<")[0]
    per = {c: v[0] / max(1, v[1]) for c, v in cs.items()}
    wc = per.get("SQ_WAVE_CYCLES", 0.0)
    if wc > 0:
        per.update({"wait_any_frac": per.get("SQ_WAIT_ANY", 0.0) / wc,
                    "wait_inst_any_frac": per.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                    "active_inst_any_frac": per.get("SQ_ACTIVE_INST_ANY", 0.0) / wc})
    out.setdefault("sq_logical", {})[name] = per
# The roofline's launch time: bench.py measures the dominant kernel in its final isolated stage
# pass (no other stream active); the same launches are the last `isolated_launches` of that kernel
# in the kernel trace, so rocprof's average over them is the cross-check of the line's avg_launch_ms.
rl = bench.get("roofline") or {}
dom, n_iso = rl.get("kernel"), int(rl.get("isolated_launches", 0) or 0)
durs = []
trace_csv = os.path.join(src, "trace", "trace_kernel_trace.csv")
if n_iso and os.path.exists(trace_csv):
    rows = [r for r in csv.DictReader(open(trace_csv)) if logical(r["Kernel_Name"]) == dom]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if "isolated_after_steps" in rl:  # since r06: the isolated pass follows the warmup + timed steps
        first = int(rl["isolated_after_steps"]) * int(rl.get("launches_per_step", {}).get(dom, 1) or 1)
        sel = rows[first:first + n_iso]
    else:  # before r06 the isolated pass was the run's last
        sel = rows[-n_iso:]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel]
if durs:
    avg_ms = sum(durs) / len(durs) / 1e6
    ach = rl["algorithmic_bytes_per_launch"] / (avg_ms * 1e-3) / 1e9
    out["roofline_check"] = {"kernel": dom, "launches": len(durs), "rocprof_avg_ms": avg_ms,
                             "bench_avg_launch_ms": rl["avg_launch_ms"], "ratio": avg_ms / rl["avg_launch_ms"],
                             "algorithmic_bytes_per_launch": rl["algorithmic_bytes_per_launch"],
                             "achieved_GBps_from_rocprof": ach, "frac_from_rocprof": ach / 8000.0}
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
