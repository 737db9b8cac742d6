"""Summarize an engine_pmc.sh run (gpurun_out/<tag>) into profiles/<tag>_pmc_traffic.json and
profiles/<tag>_engine_kernel_stats.csv: the chain engine's HBM traffic and SQ stall fractions per
launch, over the launches that did not give up under the profiler (engine_pmc.py lists them).

Traffic per launch follows MI355X_MICROARCH.md §HBM, as scripts/summarize_profile.py: FETCH_SIZE and
WRITE_SIZE are KiB from the L2's memory-side request counters, separate passes; FETCH_SIZE is doubled
on gfx950 (half-count of wide reads), WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r05c"
src = os.path.join("gpurun_out", tag)
KERNEL = "k_odom_chain"


def runs(path):  # the per-launch counter values of the engine, in dispatch order: counter -> [values]
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = {}
    for r in rows:
        out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return out


def ok_mask(name):
    d = json.loads(open(os.path.join(src, name)).read().strip().splitlines()[-1])
    return [a == 0 for a in d["aborted"]], d


def mean_ok(vals, ok):
    v = [x for x, good in zip(vals, ok) if good]
    return sum(v) / len(v) if v else None


fetch_ok, meta = ok_mask("fetch.json")
write_ok, _ = ok_mask("write.json")
sq_ok, _ = ok_mask("sq.json")
fetch = mean_ok(runs(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"))["FETCH_SIZE"], fetch_ok)
write = mean_ok(runs(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"))["WRITE_SIZE"], write_ok)
sq_raw = runs(os.path.join(src, "pmc_sq", "pmc_counter_collection.csv"))
sq = {c: mean_ok(v, sq_ok) for c, v in sq_raw.items()}
wc = sq.get("SQ_WAVE_CYCLES") or 0.0
if wc > 0:
    sq.update({"wait_any_frac": sq["SQ_WAIT_ANY"] / wc, "wait_inst_any_frac": sq["SQ_WAIT_INST_ANY"] / wc,
               "active_inst_any_frac": sq["SQ_ACTIVE_INST_ANY"] / wc})
trace_ok, _ = ok_mask("trace.json")
durs = []
for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv"))):
    if KERNEL in r["Kernel_Name"]:
        durs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
durs = [d for _, d in sorted(durs)]
avg_ms = mean_ok(durs, trace_ok) / 1e6
traffic = (2 * fetch + write) * 1024
out = {"tag": tag, "config": meta["config"], "workload": None, "odometry_engine": meta["engine"],
       "correction": "traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (gfx950 FETCH_SIZE half-count of "
                     "wide reads, MI355X_MICROARCH.md HBM section)",
       "launches_counted": {"fetch": sum(fetch_ok), "write": sum(write_ok), "sq": sum(sq_ok), "trace": sum(trace_ok)},
       "note": "the chain engine alone (scripts/engine_pmc.py: config 2's batch extracted once, then one continuous "
               "299-pair chain per launch) on the single-launch engine: the split engine's two launches must run "
               "together and dispatch-counter collection serializes dispatches, so its launches give up under --pmc "
               "(scripts/archive/pmc_engine_probe.sh, gpurun_out/r05b)",
       "kernels_logical": {KERNEL: {"launches_profiled": sum(fetch_ok), "fetch_kib_per_launch": fetch,
                                    "write_kib_per_launch": write, "traffic_bytes_per_launch": traffic,
                                    "rocprof_avg_ms": avg_ms}},
       "sq_logical": {KERNEL: sq}}
os.makedirs("profiles", exist_ok=True)
json.dump(out, open(os.path.join("profiles", f"{tag}_pmc_traffic.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join("profiles", f"{tag}_engine_kernel_stats.csv"))
print(json.dumps(out, indent=1))
