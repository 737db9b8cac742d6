"""The reference's continuous odometry chain (laserOdometry.cpp:130-135,716-717: para_q / para_t
carried from scan to scan, one node over the whole stream) on the GPU, against the oracle's chain
over the same scans.  Two schedules compute it (include/lislam.h, lislam_set_odometry_schedule):
per-round launches and the persistent engine (k_odom_chain); both must equal the oracle."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4  # BASELINE.json north_star: <= 1e-4 m / <= 1e-4 rad


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(n_scans=64, width=1024)
    yield c
    c.close()


@pytest.fixture(scope="module")
def stream61(pkg, oracle, synth):
    scans = synth.make_sequence(61, start=100)
    feats = [oracle.scan_registration(s) for s in scans]
    return scans, feats


def check_chain(pkg, b, feats, pose, rel, st, k0=0):
    assert b.odometry_status() == 0  # no engine launch gave up (the sticky abort word)
    worst = 0.0
    for j in range(1, len(feats)):
        k = k0 + j
        para = b.download(pkg.native.OUT_PARA, k)
        pw = b.download(pkg.native.OUT_POSE, k)
        d = max(np.max(np.abs(para - rel[j])), np.max(np.abs(pw - pose[j])))
        worst = max(worst, d)
        assert d < POSE_TOL, (k, para, rel[j], pw, pose[j])
        gst = b.download(pkg.native.OUT_STATS, k)
        assert np.array_equal(gst[:6], st[j][:6]), (k, gst, st[j])  # correspondences + LM iterations
    return worst


def test_continuous_chain_60_pairs_engine(pkg, oracle, ctx, stream61):
    """One continuous chain over 61 scans (60 pairs) through the persistent engine."""
    scans, feats = stream61
    S = len(scans)
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, S - 1)
    pose, rel, st = oracle.odometry_chain(feats)
    worst = check_chain(pkg, b, feats, pose, rel, st)
    print(f"continuous chain of {S - 1} pairs: max |pose - oracle| = {worst:.3g}")
    b.close()
    ctx.set_odometry_schedule(ctx.ENGINE_AUTO)


def test_continuous_chain_60_pairs_single_launch_engine(pkg, oracle, ctx, stream61):
    """The same chain through the single-launch engine (k_odom_chain: roles and items in one grid),
    the fallback where CU-masked streams are unavailable (LISLAM_ENGINE_SINGLE=1 forces it)."""
    scans, feats = stream61
    S = len(scans)
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    os.environ["LISLAM_ENGINE_SINGLE"] = "1"
    try:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, S - 1)  # the batch's first engine launch reads the variable
        ctx.synchronize()
    finally:
        del os.environ["LISLAM_ENGINE_SINGLE"]
        ctx.set_odometry_schedule(ctx.ENGINE_AUTO)
    pose, rel, st = oracle.odometry_chain(feats)
    check_chain(pkg, b, feats, pose, rel, st)
    b.close()


def test_continuous_chain_60_pairs_round_launches(pkg, oracle, ctx, stream61):
    """The same chain through the per-round launches (k_odom_assoc16 + k_odom_lm2)."""
    scans, feats = stream61
    S = len(scans)
    ctx.set_odometry_schedule(ctx.ENGINE_OFF)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, S - 1)
    pose, rel, st = oracle.odometry_chain(feats)
    check_chain(pkg, b, feats, pose, rel, st)
    b.close()
    ctx.set_odometry_schedule(ctx.ENGINE_AUTO)


@pytest.mark.parametrize("chain_len", [1, 3, 7])
def test_schedules_agree(pkg, synth, ctx, chain_len):
    """Engine and per-round launches: the same correspondences and poses (to fp64 rounding of the
    two evaluation forms) for several chains per batch."""
    S = 8
    scans = synth.make_sequence(S, start=20)
    out = {}
    for mode in (ctx.ENGINE_OFF, ctx.ENGINE_ON):
        ctx.set_odometry_schedule(mode)
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, chain_len)
        out[mode] = [(b.download(pkg.native.OUT_PARA, k), b.download(pkg.native.OUT_POSE, k),
                      b.download(pkg.native.OUT_STATS, k)) for k in range(S)]
        b.close()
    ctx.set_odometry_schedule(ctx.ENGINE_AUTO)
    for k in range(S):
        (p0, w0, s0), (p1, w1, s1) = out[ctx.ENGINE_OFF][k], out[ctx.ENGINE_ON][k]
        assert np.max(np.abs(p0 - p1)) < 1e-9, k
        assert np.max(np.abs(w0 - w1)) < 1e-9, k
        assert np.array_equal(s0, s1), (k, s0, s1)


@pytest.mark.parametrize("wgs", [1, 2, 5])
def test_engine_drains_with_few_workgroups(pkg, oracle, synth, ctx, wgs):
    """The ticket queue needs no co-residency beyond the chain's solve role and one item worker: a
    grid capped at 1 (raised to that minimum of 2 by the launcher), 2 or 5 workgroups computes the
    same chain."""
    S = 5
    scans = synth.make_sequence(S, start=40)
    feats = [oracle.scan_registration(s) for s in scans]
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    os.environ["LISLAM_ENGINE_WGS"] = str(wgs)
    try:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, S - 1)
        ctx.synchronize()
    finally:
        del os.environ["LISLAM_ENGINE_WGS"]
        ctx.set_odometry_schedule(ctx.ENGINE_AUTO)
    pose, rel, st = oracle.odometry_chain(feats)
    check_chain(pkg, b, feats, pose, rel, st)
    b.close()


def test_engine_gated_chain(pkg, oracle, synth, ctx):
    """The reference's default gating inside the engine: unflagged scans skip association and solve
    and accumulate the carried estimate (laserOdometry.cpp:403-417,716-717)."""
    S = 8
    scans = synth.make_sequence(S, start=50)
    feats = [oracle.scan_registration(s) for s in scans]
    use = np.array([0, 1, 0, 0, 1, 1, 0, 1], np.int32)
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    b = pkg.Batch(ctx, S)
    b.upload(scans)
    b.extract(S)
    b.odometry(S, S - 1, use_aloam=use)
    ctx.set_odometry_schedule(ctx.ENGINE_AUTO)
    pose, rel, st = oracle.odometry_chain(feats, use_aloam=use)
    for k in range(1, S):
        assert np.max(np.abs(b.download(pkg.native.OUT_PARA, k) - rel[k])) < POSE_TOL, k
        assert np.max(np.abs(b.download(pkg.native.OUT_POSE, k) - pose[k])) < POSE_TOL, k
        assert np.array_equal(b.download(pkg.native.OUT_STATS, k)[:4], st[k][:4]), k
    b.close()


@pytest.mark.parametrize("budget", [1, 37])
def test_engine_item_budget(pkg, oracle, synth, ctx, budget):
    """More queries than the engine keeps items in flight: the items' waves take second (and later)
    queries (EngCtl::budget), with the same correspondences and poses."""
    S = 5
    scans = synth.make_sequence(S, start=60)
    feats = [oracle.scan_registration(s) for s in scans]
    ctx.set_odometry_schedule(ctx.ENGINE_ON)
    os.environ["LISLAM_ENGINE_BUDGET"] = str(budget)
    try:
        b = pkg.Batch(ctx, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, S - 1)
        ctx.synchronize()
    finally:
        del os.environ["LISLAM_ENGINE_BUDGET"]
        ctx.set_odometry_schedule(ctx.ENGINE_AUTO)
    pose, rel, st = oracle.odometry_chain(feats)
    check_chain(pkg, b, feats, pose, rel, st)
    b.close()


def test_continuous_chain_config3_high_res_engine(pkg, oracle, synth):
    """Config 3 (128 x 2048, the N_SCANS == 128 branch of scanRegistration.cpp:317-325) as one
    continuous chain of 30 pairs through the persistent engine: every pair's pose and para within
    1e-4 and its correspondence counts and LM iterations equal to the oracle's chain."""
    S = 31
    scans = synth.make_sequence(S, 128, 2048, start=200)
    feats = [oracle.scan_registration(s) for s in scans]
    c = pkg.Context(n_scans=128, width=2048)
    try:
        c.set_odometry_schedule(c.ENGINE_ON)
        b = pkg.Batch(c, S)
        b.upload(scans)
        b.extract(S)
        b.odometry(S, S - 1)
        pose, rel, st = oracle.odometry_chain(feats)
        worst = check_chain(pkg, b, feats, pose, rel, st)
        print(f"128x2048 continuous chain of {S - 1} pairs: max |pose - oracle| = {worst:.3g}")
        b.close()
    finally:
        c.close()


def test_engine_abort_is_recovered_on_the_round_schedule(pkg, oracle, synth, ctx):
    """A launch whose bounded device wait expires (forced: a 1 us bound) is recovered, not refused:
    the next call on the batch re-runs its chains on the per-round schedule, so the outputs equal the
    per-round schedule's and the oracle's, and lislam_batch_odometry_status counts the fallback
    (reading clears it).  Both engines: the split launches and the single launch."""
    S = 6
    scans = synth.make_sequence(S, start=70)
    feats = [oracle.scan_registration(s) for s in scans]
    pose, rel, st = oracle.odometry_chain(feats)
    nat = pkg.native
    b = pkg.Batch(ctx, S)
    try:
        b.upload(scans)
        b.extract(S)
        ctx.set_odometry_schedule(ctx.ENGINE_OFF)
        b.odometry(S, S - 1)
        ref = [(b.download(nat.OUT_PARA, k), b.download(nat.OUT_POSE, k), b.download(nat.OUT_STATS, k))
               for k in range(S)]
        ctx.set_odometry_schedule(ctx.ENGINE_ON)
        for single in ("0", "1"):
            b2 = b if single == "0" else pkg.Batch(ctx, S)  # the engine kind is fixed per batch
            if b2 is not b:
                b2.upload(scans)
                b2.extract(S)
            os.environ["LISLAM_ENGINE_SINGLE"] = single
            os.environ["LISLAM_ENGINE_WAIT_US"] = "1"
            try:
                b2.odometry(S, S - 1)
            finally:
                del os.environ["LISLAM_ENGINE_WAIT_US"]
                del os.environ["LISLAM_ENGINE_SINGLE"]
            got = [(b2.download(nat.OUT_PARA, k), b2.download(nat.OUT_POSE, k), b2.download(nat.OUT_STATS, k))
                   for k in range(S)]
            assert b2.odometry_status() == 1, single  # one launch gave up and was re-run
            assert b2.odometry_status() == 0, single  # read and cleared
            for k in range(S):
                assert np.array_equal(got[k][0], ref[k][0]) and np.array_equal(got[k][1], ref[k][1]), (single, k)
                assert np.array_equal(got[k][2], ref[k][2]), (single, k)
            check_chain(pkg, b2, feats, pose, rel, st)
            b2.odometry(S, S - 1)  # a clean engine launch afterwards
            check_chain(pkg, b2, feats, pose, rel, st)
            if b2 is not b:
                b2.close()
    finally:
        b.close()
        ctx.set_odometry_schedule(ctx.ENGINE_AUTO)


def test_odom_step_recovers_from_an_engine_abort(pkg, oracle, synth):
    """lislam_odom_step (the laserOdometry node's per-scan call) runs its pair through the engine;
    an aborted launch is re-run within the same step, so that step and every later one succeed and
    equal the oracle's chain (the abort used to lock the node: every later step was refused)."""
    S = 5
    scans = synth.make_sequence(S, start=90)
    feats = [oracle.scan_registration(s) for s in scans]
    pose, rel, _ = oracle.odometry_chain(feats)
    c = pkg.Context(n_scans=64, width=1024)
    odo = pkg.LaserOdometry(c)
    try:
        for k in range(S):
            if k == 2:
                os.environ["LISLAM_ENGINE_WAIT_US"] = "1"
            try:
                para, pw, _ = odo.step(feats[k])
            finally:
                os.environ.pop("LISLAM_ENGINE_WAIT_US", None)
            if k:
                assert np.max(np.abs(para - rel[k])) < POSE_TOL, k
                assert np.max(np.abs(pw - pose[k])) < POSE_TOL, k
    finally:
        odo.close()
        c.close()


@pytest.mark.parametrize("qpw", ["1", "4"])
def test_engine_over_poisoned_buffers(pkg, oracle, synth, qpw):
    """Every batch buffer filled with 0xFF bytes (NaN doubles, -1 words) before first use
    (LISLAM_POISON, the library's read-before-write probe): the engine's records are written whole
    for every query, with or without a correspondence, so a stale non-finite word from an earlier
    use of the memory never enters an evaluation (weighted by 0 it would still be NaN).  Before the
    fix the first pair's second solve diverged (para off by 4.8e-3) whenever such words were left."""
    os.environ["LISLAM_POISON"] = "255"
    os.environ["LISLAM_ENGINE_QPW"] = qpw
    try:
        c = pkg.Context(n_scans=64, width=1024)
        scans = synth.make_sequence(5, start=40)
        b = pkg.Batch(c, 5)
        b.upload(scans)
        b.extract(5)
        b.odometry(5, 4)
        c.synchronize()
        feats = [oracle.scan_registration(s) for s in scans]
        pose, rel, st = oracle.odometry_chain(feats)
        assert b.odometry_engine() != 0
        check_chain(pkg, b, feats, pose, rel, st)
        b.close()
        c.close()
    finally:
        del os.environ["LISLAM_POISON"]
        del os.environ["LISLAM_ENGINE_QPW"]
