"""GPU parity of laserMapping's device-resident cube map (lislam_lmap, SURVEY.md §8(f) row 1,
laserMapping.cpp:319-1002) against the oracle restatement (oracle_lmap_step).

Per frame: the stats (local-map and stack sizes, association counts), the pose (tolerance 1e-4,
measured ~1e-15) and the map itself — points per cube and every point (VoxelGrid centroids,
bit-exact) — must agree.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4


@pytest.fixture(scope="module")
def frames(oracle, synth):
    scans = synth.make_sequence(8, start=40)
    feats = [oracle.scan_registration(s) for s in scans]
    _, pose, _ = oracle.odometry_chain(feats)
    return feats, pose


def _run(pkg, oracle, ctx, feats, odoms):
    gm = pkg.mapping.LaserMapping(ctx)
    om = oracle.LaserMap()
    for k, (f, od) in enumerate(zip(feats, odoms)):
        gp, gs = gm.process(f.less_sharp, f.less_flat, od)
        op, os_ = om.step(f.less_sharp, f.less_flat, od)
        assert np.array_equal(gs, os_), (k, gs, os_)
        assert np.max(np.abs(gp - op)) < POSE_TOL, (k, gp, op)
        assert np.max(np.abs(gm.state - om.state)) < POSE_TOL
        gcc, gsc = gm.counts()
        occ, osc = om.counts()
        assert np.array_equal(gcc, occ) and np.array_equal(gsc, osc), k
        for w in (0, 1):
            assert np.array_equal(gm.points(w), om.points(w)), (k, w)
    gm.close()
    return om


def test_cube_map_sequence(pkg, oracle, frames):
    feats, pose = frames
    ctx = pkg.Context(n_scans=64, width=1024)
    om = _run(pkg, oracle, ctx, feats, pose)
    cc, sc = om.counts()
    assert cc.sum() > 1000 and sc.sum() > 300  # the map grew
    ctx.close()


def test_cube_map_recentring(pkg, oracle, frames):
    """Odometry jumps of 120 m per frame push the centre cube towards the edge: the cube array is
    re-centred (cubes shift, the wrapped ones are cleared) on the device exactly as on the host."""
    feats, pose = frames
    odoms = pose[:5].copy()
    for k in range(5):
        odoms[k, 4] += 120.0 * k  # x
        odoms[k, 5] -= 120.0 * k  # y
    ctx = pkg.Context(n_scans=64, width=1024)
    _run(pkg, oracle, ctx, feats[:5], odoms)
    ctx.close()
