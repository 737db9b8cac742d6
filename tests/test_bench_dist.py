"""The multi-rank bench path on CPU (gloo, world_size 2): stream sharding and the
max-over-ranks timing reduction used by bench.py (no GPU involved)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, n = bench.shard(rank, world, 300)
    m = bench.max_over_ranks(1.0 + rank, dist)
    dist.barrier()
    q.put((rank, start, n, m))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_sharding_and_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert res[0][1:3] == (0, 300) and res[1][1:3] == (300, 300)   # disjoint contiguous stream segments
    assert res[0][3] == res[1][3] == 2.0                            # max over ranks


def _bench(*argv, timeout=180):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *argv], capture_output=True, text=True,
                         timeout=timeout, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout  # one JSON line on stdout, from rank 0 only
    return json.loads(lines[0])


@pytest.mark.timeout(200)
def test_bench_gpus_flag_starts_the_ranks():
    """`bench.py --gpus 2` without a launcher starts both ranks itself (gloo rendezvous on
    127.0.0.1): weak scaling gives each rank its own 300-scan segment."""
    d = _bench("--gpus", "2", "--dry-run")
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["shards"] == [[0, 300], [300, 300]]
    assert d["max_elapsed"] == 0.002  # max over ranks (rank r reports 0.001 (r + 1))


@pytest.mark.timeout(200)
def test_bench_config4_total_scans_shards():
    """Config 4: 1000 scans split into contiguous shards of ceil(1000 / N); the chain restarts at
    every shard boundary: one continuous chain per shard, or chains of --chain."""
    d = _bench("--gpus", "3", "--dry-run", "--total-scans", "1000")
    assert d["scaling"] == "strong"
    assert d["shards"] == [[0, 334], [334, 334], [668, 332]]
    assert d["chains_per_shard"] == [1, 1, 1]  # one continuous chain per shard (the default)
    d10 = _bench("--gpus", "3", "--dry-run", "--total-scans", "1000", "--chain", "10")
    assert d10["chains_per_shard"] == [34, 34, 34]  # ceil((334 - 1) / 10), ceil(331 / 10)
    d1 = _bench("--dry-run", "--total-scans", "1000")
    assert d1["n_gpus"] == 1 and d1["shards"] == [[0, 1000]]


def test_bench_world_size_mismatch_fails_loudly():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--dry-run"],
                         capture_output=True, text=True, timeout=60, env=env, cwd=root)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
