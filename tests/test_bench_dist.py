"""bench.py's multi-rank plumbing on CPU: world_size 2 over gloo (127.0.0.1), as the driver launches it.

Every rank runs an independent stream; only the timing max and the update sum cross ranks
(bench.combine_ranks).  The GPU part of the bench is exercised by the driver's N=1..8 runs.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    el, up = bench.combine_ranks(dist, elapsed=1.0 + rank, updates=100 * (rank + 1))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, el, up))


@pytest.mark.timeout(120)
def test_combine_ranks_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for _, el, up in res:
        assert el == 2.0 and up == 300.0  # max time, summed updates


def test_combine_ranks_single():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.combine_ranks(None, 0.5, 7) == (0.5, 7.0)
