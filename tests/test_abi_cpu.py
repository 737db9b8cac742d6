"""CPU checks of the drop-in boundary: liblislam.so loads and exports every symbol that
include/lislam.h declares; the ctypes structs match the header; no compute call without a GPU."""
import ctypes
import os
import re

import numpy as np

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lislam.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|void)\s+\*?(lislam_\w+)\s*\(", text, re.M)))


def test_header_declares_api():
    fns = declared_functions()
    assert "lislam_scan_registration" in fns and "lislam_odom_step" in fns and "lislam_eval_factors" in fns
    assert len(fns) >= 20


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.native.load()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(pkg.native.EXPORTED_SYMBOLS) == declared_functions()


def test_library_is_gfx950_code(pkg):
    data = open(pkg.native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_struct_layouts_match_header(pkg):
    n = pkg.native
    assert ctypes.sizeof(n.Config) == 20
    assert ctypes.sizeof(n.PointLayout) == 20
    assert ctypes.sizeof(n.Frame) == 4 * 16
    # lislam_scan_out: 5 x (ptr, int, int) + 3 ptrs
    assert ctypes.sizeof(n.ScanOut) == 5 * 16 + 3 * 8


def test_invalid_arguments_fail_cleanly(pkg):
    lib = pkg.native.load()
    h = ctypes.c_void_p()
    bad = pkg.native.Config(48, 1024, 0.3, 4, 1)  # 48 lines: not a supported N_SCANS
    assert lib.lislam_ctx_create(ctypes.byref(bad), 0, ctypes.byref(h)) == pkg.native.ERR_ARG
    assert lib.lislam_ctx_create(None, 0, ctypes.byref(h)) == pkg.native.ERR_ARG
    assert lib.lislam_batch_extract(None, 1) == pkg.native.ERR_ARG
    assert lib.lislam_odom_step(None, None, None, None, None) == pkg.native.ERR_ARG


def test_no_cpu_fallback_when_library_missing(pkg, tmp_path):
    with pytest.raises(RuntimeError):
        pkg.native.load.__wrapped__(str(tmp_path / "missing.so")) if hasattr(pkg.native.load, "__wrapped__") \
            else _load_missing(pkg, str(tmp_path / "missing.so"))


def _load_missing(pkg, path):
    saved = pkg.native._LIB
    pkg.native._LIB = None
    try:
        pkg.native.load(path)
    finally:
        pkg.native._LIB = saved


def test_mapopt_high_frequency_pose(pkg):
    """MapOptimization.laser_odometry_handler (mapOptimization.cpp:19-49): host glue, no GPU."""
    from scipy.spatial.transform import Rotation as R

    m = pkg.mapping.MapOptimization.__new__(pkg.mapping.MapOptimization)
    q = np.array([0.1, 0.2, 0.3, 0.9])
    q /= np.linalg.norm(q)
    m.state = np.concatenate([q, [1.0, 2.0, 3.0]])
    od = np.array([0, 0, np.sin(0.2), np.cos(0.2), 4.0, 5.0, 6.0])
    p = m.laser_odometry_handler(od)
    assert np.allclose(p[4:], R.from_quat(q).apply(od[4:]) + [1, 2, 3])
    assert np.allclose(R.from_quat(p[:4]).as_matrix(), (R.from_quat(q) * R.from_quat(od[:4])).as_matrix())
