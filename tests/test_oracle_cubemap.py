"""CPU pin of the oracle's laserMapping cube map (oracle_lmap_step, laserMapping.cpp:319-1002)
against an independent Python transcription of its bookkeeping: re-centring shifts (pointer
rotation, wrapped cubes cleared), the valid-cube loop order of the local map, insertion at the
optimized pose (Eigen q * v + t in double, stored as float) and the per-cube VoxelGrid of the
valid cubes.  The optimization itself is taken from the oracle's returned pose (it is pinned by
tests/test_oracle_map.py).  No GPU."""
import numpy as np

W, H, D = 21, 21, 11


def _qrot(q, v):
    u = np.array([q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]])
    u = u + u
    c = np.array([q[1] * u[2] - q[2] * u[1], q[2] * u[0] - q[0] * u[2], q[0] * u[1] - q[1] * u[0]])
    return (v + q[3] * u) + c


def _cube(v, cen):
    c = int((v + 25.0) / 50.0) + cen
    return c - 1 if v + 25.0 < 0 else c


class PyCubeMap:
    def __init__(self, oracle):
        self.O = oracle
        self.cen = [10, 10, 5]
        self.arr = [[np.zeros((0, 4), np.float32) for _ in range(W * H * D)] for _ in range(2)]

    def at(self, i, j, k):
        return i + W * j + W * H * k

    def frame(self, stacks, x, t_curr):
        """stacks: voxelized corner / surf (sensor frame); x: the optimized pose; t_curr: the
        pose's translation before the optimization (decides the centre cube)."""
        cc = [_cube(t_curr[a], self.cen[a]) for a in range(3)]
        dims = (W, H, D)
        for a in range(3):
            while cc[a] < 3:
                self._shift(a, +1)
                cc[a] += 1
                self.cen[a] += 1
            while cc[a] >= dims[a] - 3:
                self._shift(a, -1)
                cc[a] -= 1
                self.cen[a] -= 1
        valid = [self.at(i, j, k) for i in range(cc[0] - 2, cc[0] + 3) for j in range(cc[1] - 2, cc[1] + 3)
                 for k in range(cc[2] - 1, cc[2] + 2) if 0 <= i < W and 0 <= j < H and 0 <= k < D]
        local = [np.concatenate([self.arr[w][v] for v in valid]) if valid else np.zeros((0, 4), np.float32)
                 for w in (0, 1)]
        for w in (0, 1):
            for p in stacks[w]:
                pw = (_qrot(x[:4], p[:3].astype(np.float64)) + x[4:]).astype(np.float32)
                ci = [_cube(float(pw[a]), self.cen[a]) for a in range(3)]
                if all(0 <= ci[a] < dims[a] for a in range(3)):
                    c = self.at(*ci)
                    self.arr[w][c] = np.concatenate([self.arr[w][c], np.array([[pw[0], pw[1], pw[2], p[3]]], np.float32)])
        for v in valid:
            for w, leaf in ((0, 0.4), (1, 0.8)):
                self.arr[w][v] = self.O.voxel_grid(self.arr[w][v], leaf)
        return local

    def _shift(self, a, s):
        for w in (0, 1):
            g = np.array(self.arr[w], dtype=object).reshape(D, H, W)  # [k][j][i]
            ax = 2 - a
            g = np.roll(g, s, axis=ax)
            idx = [slice(None)] * 3
            idx[ax] = 0 if s > 0 else -1  # the wrapped-around slab is cleared
            cleared = g[tuple(idx)]
            for e in np.ndindex(cleared.shape):
                cleared[e] = np.zeros((0, 4), np.float32)
            g[tuple(idx)] = cleared
            self.arr[w] = list(g.reshape(-1))


def _check(oracle, synth, odom_shift):
    scans = synth.make_sequence(5, 32, 512, start=3)
    feats = [oracle.scan_registration(s) for s in scans]
    _, pose, _ = oracle.odometry_chain(feats)
    pose = pose.copy()
    for k in range(len(pose)):
        pose[k, 4:6] += odom_shift * k
    om = oracle.LaserMap()
    pm = PyCubeMap(oracle)
    for k, f in enumerate(feats):
        state0 = om.state.copy()
        x, stats = om.step(f.less_sharp, f.less_flat, pose[k])
        # the centre cube follows t_w_curr = q_wmap_wodom t_wodom + t_wmap_wodom before the optimization
        t_curr = _qrot(state0[:4], pose[k, 4:].astype(np.float64)) + state0[4:]
        stacks = [oracle.voxel_grid(f.less_sharp, 0.4), oracle.voxel_grid(f.less_flat, 0.8)]
        local = pm.frame(stacks, x, t_curr)
        assert stats[0] == local[0].shape[0] and stats[1] == local[1].shape[0]  # local maps before insertion
        cc, sc = om.counts()
        for w, cnt in ((0, cc), (1, sc)):
            py = np.array([a.shape[0] for a in pm.arr[w]])
            assert np.array_equal(cnt, py), (k, w)
            assert np.array_equal(om.points(w), np.concatenate(pm.arr[w]))
    return pm


def test_cube_bookkeeping_matches_python(oracle, synth):
    _check(oracle, synth, 0.0)


def test_cube_recentring_matches_python(oracle, synth):
    pm = _check(oracle, synth, np.array([130.0, -140.0]))
    assert pm.cen[0] < 10 and pm.cen[1] > 10  # the cube array was re-centred on both axes
