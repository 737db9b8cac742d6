"""Developer tool: summary of a LISLAM_TIMELINE=1 bench run's device timeline (bench.err): over the
pipelined chains (those before the single-sequence leg's back-to-back chains), the mean chain
duration, the mean number of chains in flight, and the mean extraction span.
Usage: python scripts/timeline_summary.py bench.err [...]"""
import sys


def summary(path):
    ch, ex = [], []
    for line in open(path):
        if line.startswith("timeline "):
            _, who, obj, k, a, b = line.split()
            (ch if who == "odometry" else ex if who == "extract" else []).append((float(a), float(b), obj))
    ch.sort()
    ex.sort()
    # the single-sequence leg: one context, chains back to back after the pipelined ones
    objs = [o for _, _, o in ch]
    n = len(ch)
    while n > 1 and objs[n - 1] == objs[-1] and ch[n - 1][0] >= max(b for _, b, _ in ch[:n - 1]):
        n -= 1
    pipe = ch[:n]
    t0, t1 = pipe[0][0], max(b for _, b, _ in pipe)
    busy = sum(b - a for a, b, _ in pipe)
    exp = [(a, b) for a, b, _ in ex if a < t1]
    print(f"{path}: {len(pipe)} pipelined chains over {t1 - t0:.1f} ms: mean {busy / len(pipe):.1f} ms, "
          f"in flight {busy / (t1 - t0):.2f}; {len(exp)} extractions, mean {sum(b - a for a, b in exp) / max(1, len(exp)):.1f} ms; "
          f"chain-bound rate {len(pipe) * 299 / (t1 - t0) * 1e3:.0f} pairs/s")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        summary(p)
