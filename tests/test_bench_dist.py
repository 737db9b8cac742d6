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
