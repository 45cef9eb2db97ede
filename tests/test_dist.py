"""CPU, world_size 2 over gloo: bench.py's multi-rank harness (barriers around exactly K steps,
max-over-ranks timing, whole-job Mpx/s).  The data path itself has no collectives (replicas:
one frame per GPU), so the only distributed logic to prove is the timing/aggregation."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import time

    import torch.distributed as dist

    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.01 * (rank + 1))  # rank 1 is the slow one

    dt = bench.timed_steps(step, 5, dist.barrier, lambda: None)
    dtm = bench.reduce_max(dt)
    q.put((rank, len(calls), dt, dtm))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_timing_and_max_reduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, dt0, m0), (r1, n1, dt1, m1) = res
    assert n0 == n1 == 5                       # exactly K steps on every rank
    assert m0 == pytest.approx(m1)             # every rank sees the same max
    assert m0 == pytest.approx(max(dt0, dt1))
    assert m0 >= 0.05                          # bounded below by the slow rank's 5 x 10 ms


def test_whole_job_value_is_sum_over_ranks():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.whole_job_mpx(world=4, npx=4096 * 4096, steps=10, dt_max=2.0) == pytest.approx(
        4 * 4096 * 4096 * 10 / 2.0 / 1e6)
