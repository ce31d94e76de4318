"""The N>1 benchmark path on CPU: world_size 2 over gloo (127.0.0.1).

bench.py shards pages by rank with no data-path collective; the process group
only provides the barrier and the max/sum reductions of the timing.  This
checks that those pieces behave across real processes.
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, pages, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    d = bench.Dist()
    first, n = bench.shard(d.rank, pages)
    d.barrier()
    mx = d.max(float(rank + 1))
    tot = d.sum(float(n))
    d.barrier()
    d.close()
    q.put((rank, first, n, mx, tot))


@pytest.mark.parametrize("world", [2])
def test_gloo_sharding_and_reductions(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    pages = 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, pages, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards are disjoint, consecutive and cover world * pages pages
    spans = [(first, first + n) for _, first, n, _, _ in res]
    assert spans[0][0] == 0
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0
    assert spans[-1][1] == world * pages
    # max over ranks and the whole-job page count are the same on every rank
    assert all(mx == float(world) for _, _, _, mx, _ in res)
    assert all(tot == float(world * pages) for _, _, _, _, tot in res)
