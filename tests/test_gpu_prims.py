"""The map path's hand-written device primitives (csrc/lislam_prims.hpp: the ikd-Tree rebuild's and
cube map's stable radix sort, the ordered compaction of Add_Points / ICP, the exclusive scan of the
VoxelGrid runs) against numpy: the stable order of equal keys, every size class of the tile scan
(one workgroup, tiles of tiles), empty inputs."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


@pytest.fixture(scope="module")
def lib(pkg):
    with pkg.Context(n_scans=16, width=256) as ctx:  # loads the library and initialises the device
        L = ctx.lib
        L.lislam_debug_sort_pairs.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                              _i32p]
        L.lislam_debug_select_scan.argtypes = [_u8p, _i32p, ctypes.c_int32, _i32p, ctypes.POINTER(ctypes.c_int32), _i32p]
        yield L


@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("n", [0, 1, 1000, 4097, 300_000, 2_000_000])
def test_radix_sort_pairs_stable(lib, bits, n):
    rng = np.random.default_rng(n + bits)
    dt = np.uint64 if bits == 64 else np.uint32
    # few distinct keys (long runs of equal keys: the order inside a run is the input order) and
    # keys spread over every byte
    keys = (rng.integers(0, 50, n).astype(dt) << dt(bits - 8)) | rng.integers(0, 3, n).astype(dt)
    keys[::7] = rng.integers(0, np.iinfo(dt).max, (n + 6) // 7, dtype=dt)
    vals = np.arange(n, dtype=np.int32)[::-1].copy()
    ko = np.zeros(n, dt)
    vo = np.zeros(n, np.int32)
    assert lib.lislam_debug_sort_pairs(keys.ctypes.data, vals, n, bits, ko.ctypes.data, vo) == 0
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(ko, keys[order])
    assert np.array_equal(vo, vals[order])


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 100_000, 40_000_000])
def test_select_flagged_and_exclusive_sum(lib, n):
    rng = np.random.default_rng(n)
    flags = (rng.random(n) < 0.37).astype(np.uint8)
    vals = rng.integers(-5, 20, n).astype(np.int32)
    sel = np.zeros(n, np.int32)
    ex = np.zeros(n, np.int32)
    cnt = ctypes.c_int32(-1)
    assert lib.lislam_debug_select_scan(flags, vals, n, sel, ctypes.byref(cnt), ex) == 0
    ref = vals[flags != 0]
    assert cnt.value == ref.size
    assert np.array_equal(sel[:cnt.value], ref)
    refx = np.zeros(n, np.int64)
    if n:
        refx[1:] = np.cumsum(vals.astype(np.int64))[:-1]
    assert np.array_equal(ex.astype(np.int64), refx)
