"""Developer tool (GPU box): the chain engine's device waits counted per wait code over one
continuous 299-pair chain (config 2's batch): polls, waits, and the agent-scope load bytes they
cost (each poll loads the waited word and the abort word: two requests of 64 B as FETCH_SIZE counts
them).  The counters exist only in a developer build:
  bash scripts/build_variant.sh prof lislam_odometry.hip -DLISLAM_ENG_PROF=1
  LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so python scripts/engine_polls.py [latency|throughput]
LISLAM_ENGINE_SINGLE=1 counts the single-launch engine (the PMC stand-in) instead of the split one.
Wait codes: 1 an item waiting for the previous pass's items (second outer pass), 2 an item waiting
for its pass's x, 3 a solve role waiting for its pass's items."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "latency"
    pkg = g.package()
    if os.environ.get("LISLAM_ALT_LIB"):
        pkg.native.load(os.environ["LISLAM_ALT_LIB"])
    S = 300
    cache = f"/tmp/lislam_scans.0_{S}_64x1024.npy"
    scans = np.load(cache) if os.path.exists(cache) else pkg.synth.make_sequence(S)
    with pkg.Context() as ctx:
        lib = ctx.lib
        lib.lislam_debug_engine_polls.argtypes = [ctypes.c_void_p]
        ctx.set_odometry_schedule(ctx.ENGINE_ON)
        ctx.set_engine_shape(*(ctx.SHAPE_THROUGHPUT if shape == "throughput" else ctx.SHAPE_LATENCY))
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, S - 1)
        ctx.synchronize()
        buf = np.zeros(16, np.uint64)
        assert lib.lislam_debug_engine_polls(buf.ctypes.data) == 0  # clear
        b.odometry(S, S - 1)
        ctx.synchronize()
        assert lib.lislam_debug_engine_polls(buf.ctypes.data) == 0
        aborted = b.odometry_status()
        names = {1: "item: previous pass's items", 2: "item: its pass's x", 3: "role: its pass's items"}
        out = {"shape": shape, "engine": b.ENGINES[b.odometry_engine()], "aborted": aborted, "waits": {}}
        tot = 0
        for code, name in names.items():
            polls, waits = int(buf[code]), int(buf[8 + code])
            out["waits"][name] = {"polls": polls, "waits": waits, "polls_per_wait": round(polls / max(1, waits), 1),
                                  "load_bytes": polls * 2 * 64}
            tot += polls * 2 * 64
        out["load_bytes_total"] = tot
        print(json.dumps(out), flush=True)
        b.close()


if __name__ == "__main__":
    main()
