"""Developer tool: per-batch critical path of a LISLAM_TIMELINE=1 bench run (bench.err): for every
step of a batch, its extraction, chain and ORB spans (ORB = the batch's ORB events between its
extraction and its next one), and the gap between the later of chain / ORB end and the batch's next
extraction start (host latency + the context stream).  Usage: python scripts/timeline_ctx.py bench.err"""
import collections
import sys


def main(path):
    ev = []
    for line in open(path):
        if line.startswith("timeline "):
            _, who, obj, k, a, b = line.split()
            ev.append((float(a), float(b), who, obj, int(k)))
    ev.sort()
    bat = collections.defaultdict(lambda: {"extract": [], "odometry": []})
    orb = collections.defaultdict(list)
    for a, b, who, o, k in ev:
        if who in ("extract", "odometry"):
            bat[o][who].append((a, b))
        elif 6 <= k <= 13:
            orb[o].append((a, b))
    # an ORB object belongs to a batch: match them in the order of their first ORB event / first
    # extraction end (each batch's ORB follows its extraction)
    ob_order = sorted(orb, key=lambda o: orb[o][0][0])
    ba_order = sorted((bo for bo in bat if bat[bo]["extract"]), key=lambda bo: bat[bo]["extract"][0][1])
    owner = dict(zip(ob_order, ba_order))
    gaps, crit = [], collections.Counter()
    for bo, d in bat.items():
        ex, ch = d["extract"], d["odometry"]
        ospans = [s for o, sp in orb.items() if owner.get(o) == bo for s in sp]
        for i in range(len(ex) - 1):
            e0, e1 = ex[i], ex[i + 1]
            c = [x for x in ch if e0[1] <= x[0] + 1e-3 and x[0] < e1[0]]
            ob = [x for x in ospans if e0[1] <= x[0] + 1e-3 and x[0] < e1[0]]
            cend = max((x[1] for x in c), default=e0[1])
            oend = max((x[1] for x in ob), default=e0[1])
            last = max(cend, oend)
            crit["chain" if cend >= oend else "orb"] += 1
            gaps.append(e1[0] - last)
            print(f"{bo[-4:]} step {i}: extract {e0[1] - e0[0]:6.1f}  chain {cend - e0[1]:6.1f}  orb {oend - e0[1]:6.1f}  "
                  f"-> next extract after {e1[0] - last:6.2f} ms")
    if gaps:
        print(f"later of chain / ORB: {dict(crit)}; gap to the next extraction mean {sum(gaps) / len(gaps):.2f} ms, max {max(gaps):.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
