"""The GPU's exact k-NN (k_knn behind lislam_map_nearest_search, the ikd-Tree's Nearest_Search
drop-in) against the reference's OWN vendored kd-tree: the neighbour sets nanoflann v1.3.2
(/root/reference/include/nanoflann.hpp:62) returned on the same inputs, committed in
tests/golden/knn_nanoflann.npz (tests/golden/make_nanoflann_golden.py).  Squared distances must be
bit-identical and ids identical wherever the k-th distance is not shared (ties counted apart, as in
tests/test_oracle_nanoflann.py)."""
import numpy as np
import pytest

from test_oracle_nanoflann import compare, golden  # noqa: F401  (the fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["corridor5", "lessflat1", "lesssharp1"])
@pytest.mark.parametrize("cell", [0.0, 0.3])
def test_gpu_knn_matches_reference_nanoflann(pkg, golden, name, cell):  # noqa: F811
    g, cs = golden
    t, q, k = cs[name]
    with pkg.Context(n_scans=64, width=1024) as ctx:
        m = pkg.mapping.IkdMap(ctx, 0.4, cell)
        m.build(t)
        pts, d2, found = m.nearest_search(q, k)
        m.close()
    ids = pts[:, :, 3].copy().view(np.int32)
    exact, ties = compare(ids, d2, found, g, name, t, q)
    print(f"{name} (cell {cell}): {exact} queries id-exact, {ties} with tied distances")
    assert ties <= max(1, q.shape[0] // 100)
