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


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_run_real_engines(tmp_path):
    """bench.py --gpus 2 as the driver launches it (torch.distributed.run, gloo barrier / max / sum), both
    ranks pinned to the one GPU of the box (PFMPE_BENCH_DEVICE=0): each rank runs its own camera stream
    through a real engine, and each rank's records and final particle set equal a single-rank run of the
    same stream (no data crosses ranks)."""
    import json
    import subprocess
    env = dict(os.environ, PFMPE_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    common = ["--steps", "6", "--warmup", "2", "--config", "C5", "--particles", "20000", "--cpu-frames", "0",
              "--worst-frames", "0", "--no-timing"]
    dump2 = str(tmp_path / "two")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--dump-records", dump2] + common, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["N_particles"] == 20000
    for rank in (0, 1):
        dump1 = str(tmp_path / f"one{rank}")
        r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--stream-id", str(rank),
                             "--dump-records", dump1] + common, cwd=ROOT, env=env, capture_output=True, text=True,
                            timeout=300)
        assert r1.returncode == 0, r1.stderr[-3000:]
        with open(f"{dump2}.{rank}.json") as f:
            a = json.load(f)
        with open(f"{dump1}.0.json") as f:
            b = json.load(f)
        assert a["stream"] == b["stream"] == rank
        assert a["records"] == b["records"]
        assert a["post_sha1"] == b["post_sha1"]
    # the two streams differ (independent seeds)
    with open(f"{dump2}.0.json") as f0, open(f"{dump2}.1.json") as f1:
        assert json.load(f0)["post_sha1"] != json.load(f1)["post_sha1"]
