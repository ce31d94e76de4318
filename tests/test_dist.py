"""The N>1 benchmark path on CPU: world_size 2 over gloo (127.0.0.1).

bench.py shards pages by rank with no data-path collective; the process group
only provides the barrier and the max/sum reductions of the timing.  This
checks that those pieces behave across real processes, and the single-process
`--gpus N` plan (one runner thread per device, lib/batch_worker.c peer).
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
    devices, firsts, n_gpus = bench.shard_plan(d.world, d.rank, d.local_rank, 1, 8, pages)
    assert devices == [rank] and n_gpus == world
    first, n = firsts[0], pages
    d.barrier()
    mx = d.max(float(rank + 1))
    tot = d.sum(float(n))
    bad = d.sum(0.0)
    d.barrier()
    d.close()
    q.put((rank, first, n, mx, tot + bad))


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


def test_single_process_device_fanout_plan():
    sys.path.insert(0, ROOT)
    import bench
    devices, firsts, n = bench.shard_plan(1, 0, 0, 4, 8, 1000)
    assert devices == [0, 1, 2, 3] and firsts == [0, 1000, 2000, 3000] and n == 4
    with pytest.raises(Exception, match="only 2 HIP devices"):
        bench.shard_plan(1, 0, 0, 4, 2, 1000)


def test_diag_guard():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.diag_guard("unpaper-hip 0.2 (gfx950)", {}, False) is True
    with pytest.raises(SystemExit):
        bench.diag_guard("unpaper-hip 0.2 (gfx950, diag)", {}, False)
    with pytest.raises(SystemExit):
        bench.diag_guard("unpaper-hip 0.2 (gfx950)", {"UPHIP_DIAG_SKIP": "1"}, False)
    assert bench.diag_guard("unpaper-hip 0.2 (gfx950, diag)", {}, True) is False


def test_product_library_has_no_diagnostics():
    """`make lib` builds without UPHIP_DIAG: the version string says so, and
    the library reads no diagnostics or debug variable at all (UPHIP_DIAG_*,
    UPHIP_DEBUG_*): no hidden sync or host print in the product path."""
    sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))
    from unpaper_hip.device import LIB_PATH, load_library
    L = load_library()
    assert "diag" not in L.uphip_version().decode()
    with open(LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"UPHIP_DIAG" not in blob
    assert b"UPHIP_DEBUG" not in blob
