"""Developer tool (GPU box): launch the chain engine on a short continuous chain with the device
trace on and print every workgroup's {ticket, stage, LM pass, time} while it runs (10 s watchdog;
a stuck kernel leaves the process through os._exit after printing)."""
import ctypes
import os
import sys
import time

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
import __graft_entry__ as g  # noqa: E402

pkg = g.package()
if os.environ.get("LISLAM_ALT_LIB"):
    pkg.native.load(os.environ["LISLAM_ALT_LIB"])  # a developer variant of the library
S = int(sys.argv[1]) if len(sys.argv) > 1 else 3
WGS = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if WGS:
    os.environ["LISLAM_ENGINE_WGS"] = str(WGS)
scans = pkg.synth.make_sequence(S, start=100)
with pkg.Context() as ctx:
    lib = ctx.lib
    lib.lislam_debug_engine_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))]
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    ctx.synchronize()
    print("extracted", flush=True)
    NW = 256
    hp = ctypes.POINTER(ctypes.c_uint32)()
    assert lib.lislam_debug_engine_trace(NW, ctypes.byref(hp)) == 0
    tr = np.ctypeslib.as_array(hp, shape=(NW, 16, 16))[:, :, 0]
    b.odometry(S, S - 1)
    t0 = time.time()
    done = False
    while time.time() - t0 < 10:
        time.sleep(0.5)
        snap = tr.copy()
        act = snap[snap[:, 0] != 0xffffffff]
        print(f"t={time.time() - t0:.1f}s active={len(act)} max_ticket={act[:, 0].max() if len(act) else -1}", flush=True)
        q = lib.hipStreamQuery if hasattr(lib, "hipStreamQuery") else None
        if os.environ.get("TRACE_DONE_CHECK") is None and len(act) and (time.time() - t0) > 2:
            pass
    snap = tr.copy()
    for i, row in enumerate(snap):
        if row[0] != 0xffffffff:
            print(i, [int(v) for v in row], flush=True)
    print("status", b.odometry_status() if False else "n/a", flush=True)
    sys.stdout.flush()
    os._exit(0)
