"""Developer tool: merge the device timeline (LISLAM_TIMELINE=1) and the host call log
(LISLAM_BENCH_HOSTLOG=1) a bench run wrote to stderr into one listing, plus the chain summary
(duration of each chain, gap to the previous one).  Usage: python scripts/timeline.py bench.err"""
import json
import sys

ORB = {6: "orb_pyramid", 7: "orb_fast", 8: "orb_select", 9: "orb_finish", 10: "orb_blur", 11: "orb_desc",
       12: "orb_match", 13: "orb_lm"}


def main(path):
    rows, host = [], []
    for line in open(path):
        if line.startswith("timeline "):
            _, who, obj, k, a, b = line.split()
            k = int(k)
            name = ORB.get(k, f"ctx{k}") if who == "ctx" else ("chain" if who == "odometry" else "extract")
            rows.append((float(a), float(b), "dev", obj[-4:], name))
        elif line.startswith("hostlog "):
            host = json.loads(line[8:])
    for n, st, a, b in host:
        rows.append((a, b, "host", str(st), n))
    rows.sort()
    for a, b, kind, who, name in rows:
        print(f"{a:10.3f} {b:10.3f} {b - a:8.3f}  {kind:4s} {who:5s} {name}")
    chains = sorted((a, b) for a, b, kind, _, name in rows if name == "chain")
    print("\nchains (start, ms, gap to the previous end):")
    for i, (a, b) in enumerate(chains):
        gap = a - chains[i - 1][1] if i else 0.0
        print(f"  {a:10.3f} {b - a:8.3f} {gap:8.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
