"""Developer tool (GPU box): phase profile of the chain engine on one continuous chain — per round
and outer pass, from the device's own clock (s_memrealtime, 10 ns ticks): association span,
association -> solve hand-off, record load, evaluations, steps, solve -> association hand-off.
usage: python scripts/engine_prof.py [S]
The stamps are compiled out of the production library: build a variant first,
  bash scripts/build_variant.sh prof lislam_odometry.hip -DLISLAM_ENG_PROF=1
and run with LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so."""
import ctypes
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
if os.environ.get("LISLAM_ALT_LIB"):
    pkg.native.load(os.environ["LISLAM_ALT_LIB"])  # a developer variant of the library
S = int(sys.argv[1]) if len(sys.argv) > 1 else 300
cache = f"/tmp/lislam_chain_scans_{S}.npy"
if os.path.exists(cache):
    scans = np.load(cache)
else:
    scans = pkg.synth.make_sequence(S)
    np.save(cache, scans)
if len(sys.argv) > 2:
    os.environ["LISLAM_ENGINE_PREFETCH"] = sys.argv[2]
with pkg.Context() as ctx:
    lib = ctx.lib
    lib.lislam_debug_engine_prof.argtypes = [ctypes.c_int]
    lib.lislam_debug_engine_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, S - 1)
    ctx.synchronize()
    I = lib.lislam_debug_engine_items(12 * 64 + 24 * 64, int(os.environ.get("LISLAM_ENGINE_QPW", "1")),
                                      int(os.environ.get("LISLAM_ENGINE_DEPTH", "1")))
    R = S - 1
    T = 2 * R * (I + 1)
    assert lib.lislam_debug_engine_prof(T) == 0
    b.odometry(S, S - 1)
    ctx.synchronize()
    nq = np.array([b.count(pkg.native.OUT_SHARP, k) + b.count(pkg.native.OUT_FLAT, k) for k in range(1, S)])
    sp = np.zeros(4, np.uint64)
    buf = np.zeros((T, 16), np.uint64)
    assert lib.lislam_debug_engine_prof_read(buf.ctypes.data, T) == 0
    lib.lislam_debug_engine_prof(0)
    p = buf.reshape(2 * R, I + 1, 16).astype(np.int64)
    us = 0.01
    items, lm = p[:, :I], p[:, I]
    valid = items[:, :, 3] > 0  # items that ran (all live ones)
    a_start = np.where(valid, items[:, :, 1], np.iinfo(np.int64).max).min(1)
    a_end = np.where(valid, items[:, :, 3], 0).max(1)
    a_med = np.array([np.median(items[i, valid[i], 3] - items[i, valid[i], 1]) for i in range(2 * R)])
    lm_ready, lm_loaded, lm_done = lm[:, 1], lm[:, 2], lm[:, 3]
    ev, st, npass = lm[:, 4], lm[:, 5], lm[:, 6]
    span = (lm_done[-1] - a_start[0]) * us
    print(f"chain of {R} pairs: {span / 1e3:.2f} ms on the device clock, {span / (2 * R):.1f} us per outer pass")
    rows = {
        "association span (first ready -> last done)": (a_end - a_start) * us,
        "association item median (ready -> done)": a_med * us,
        "hand-off assoc -> solve (last item done -> solve ready)": (lm_ready - a_end) * us,
        "solve record load": (lm_loaded - lm_ready) * us,
        "last item done -> solve has every share (gather tail)": (lm_loaded - a_end) * us,
        "solve evaluations (sum)": ev * us,
        "solve steps (sum)": st * us,
        "solve: step 0 beside the blocks' load (to the first barrier)": lm[:, 7] * us,
        "solve: step 0 alone (wave 0)": lm[:, 0] * us,
        "solve: step 0, the 32 share rows' sum": lm[:, 11] * us,
        "solve: step 0, the LM step (lm_start + propose)": (lm[:, 0] - lm[:, 11]) * us,
        "solve total (ready -> done)": (lm_done - lm_ready) * us,
        "hand-off solve -> assoc (solve done -> next first item ready)": (a_start[1:] - lm_done[:-1]) * us,
    }
    w0 = items[:, :, 5] > 0
    med = lambda col: np.array([np.median(items[i, w0[i], col]) for i in range(2 * R)]) * us
    rows["association wave 0: query load + transform + seeds"] = med(4)
    rows["association wave 0: 1-NN (nn_wave / nn16)"] = med(5)
    rows["association wave 0: line searches + record"] = med(6)
    rows["association item: first-evaluation share (wave 0)"] = med(7)
    rows["association wave 0: 1-NN, outer 1 (seeded)"] = med(5)[1::2]
    rows["association wave 0: line searches, outer 1 (seeded)"] = med(6)[1::2]
    rows["association span, outer pass 0"] = ((a_end - a_start) * us)[0::2]
    rows["association span, outer pass 1 (seeded)"] = ((a_end - a_start) * us)[1::2]
    rows["association item median, outer 0"] = (a_med * us)[0::2]
    rows["association item median, outer 1"] = (a_med * us)[1::2]
    late = np.array([np.sum(valid[i] & (items[i, :, 1] - a_start[i] > 300)) for i in range(2 * R)])  # > 3 us after
    spread = np.array([np.percentile(items[i, valid[i], 1] - a_start[i], 90) for i in range(2 * R)]) * us
    done_last = np.array([np.max(items[i, valid[i], 3] - items[i, valid[i], 1]) for i in range(2 * R)]) * us
    rows["association items ready > 3 us after the first (count)"] = late
    rows["association ready-time spread p90 (us)"] = spread
    rows["association slowest item (ready -> done)"] = done_last
    claim_ready = np.array([np.median(items[i, valid[i], 1] - items[i, valid[i], 0]) for i in range(2 * R)]) * us
    rows["association item claim -> ready median"] = claim_ready
    # items ready > 3 us after their pass's first: when they were claimed and began waiting
    late = []
    for i in range(1, 2 * R):
        v = valid[i]
        rd = items[i, :, 1] - a_start[i]
        for j in np.nonzero(v & (rd > 300))[0]:
            late.append(((items[i, j, 0] - a_start[i]) * us, (items[i, j, 2] - a_start[i]) * us, rd[j] * us,
                         (items[i, j, 3] - items[i, j, 1]) * us, int(j)))
    if late:
        la = np.array(late)
        print(f"  late items: {len(la)} over {2 * R} passes; relative to the pass's first ready (us): "
              f"claim p50 {np.median(la[:, 0]):.1f}, wait start p50 {np.median(la[:, 1]):.1f}, "
              f"ready p50 {np.median(la[:, 2]):.1f}, run p50 {np.median(la[:, 3]):.1f}; item index p50 {np.median(la[:, 4]):.0f}")
        for row in la[np.argsort(-la[:, 2])][:8]:
            print("   late item: claim %.1f wait %.1f ready %.1f run %.1f item %d" % tuple(row))
    # the end of each item's last query (slot 10), after the pass's first ready item
    ok10 = valid & (items[:, :, 10] > 0)
    if ok10.any():
        rows["all items: last query end (after first ready)"] = np.concatenate(
            [(items[i, ok10[i], 10] - a_start[i]) for i in range(2 * R)]) * us
    for k, v in rows.items():
        print(f"  {k:62s} mean {np.mean(v):7.2f} us  p50 {np.median(v):7.2f}  p90 {np.percentile(v, 90):7.2f}")
    print(f"  evaluations per solve: mean {np.mean(npass):.2f}")
    nrun = valid.sum(1)
    print(f"  items run per pass: mean {nrun.mean():.1f} min {nrun.min()} max {nrun.max()} (of {I} per pass); "
          f"queries per pass (n_sharp + n_flat): mean {np.mean(nq):.0f} max {np.max(nq)}")

    b.close()
