"""CPU, world_size 2 over gloo: bench.py's multi-rank harness (barriers around exactly K steps,
max-over-ranks timing, whole-job Mpx/s, the per-rank config-5 frame blocks and the summed digest
parity).  The data path itself has no collectives (replicas: 8 frames per GPU), so the only
distributed logic to prove is the frame assignment, the timing and the aggregation."""
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


def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` with no launcher starts 2 ranks itself (torch.distributed.run
    children, before any GPU call) and rank 0 reports n_gpus = 2.  The harness-test step (a sleep,
    gloo) stands in for the GPU step so the launch path runs on CPU."""
    import json
    import subprocess

    env = dict(os.environ, MSEG_BENCH_HARNESS_TEST="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                          "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                     # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 3
    assert d["value"] == pytest.approx(2 * 3 / (d["ms_per_step"] * 3 / 1000.0), rel=1e-3)


def _replica_worker(rank, world, port, q):
    """One rank of bench.py's N > 1 layout on CPU: the frames bench.default_frames / frame_seed give
    this rank (config 5's 100 + 8r .. 100 + 8r + 7), flooded by the C oracle as the stand-in for the
    GPU batch step, checked against the committed digests with bench.digest_parity and summed over
    the ranks with bench.reduce_sum_ints -- the parity count bench.py prints; the data path itself
    has no exchange."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]
    import json
    from concurrent.futures import ThreadPoolExecutor

    import torch.distributed as dist

    import bench
    from msegment import synth
    from oracle import ws_oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    K = bench.default_frames(None, world)
    seed = bench.frame_seed(None, rank, world, K)
    seeds = list(range(seed, seed + K))

    def flood(s):  # the oracle runs without the GIL inside ctypes
        img, m, _ = synth.frame("mosaic", 4096, 4096, s)
        return ws_oracle.watershed(img, m)

    with ThreadPoolExecutor(4) as ex:
        labs = list(ex.map(flood, seeds))
    dgs = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    mine = bench.digest_parity(labs, ["mosaic_4096x4096_s%d" % s for s in seeds], dgs)
    total = bench.reduce_sum_ints(mine)
    q.put((rank, seeds, mine, total))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_replicas_segment_their_own_config5_frames():
    """world size 2: rank r floods config 5's frames 100 + 8r .. 100 + 8r + 7 (bench.py's default
    N > 1 step), every label map equals the committed oracle digest of its frame, the two ranks did
    different frames, and the summed parity count is 16/16."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (r0, s0, m0, t0), (r1, s1, m1, t1) = res
    assert s0 == list(range(100, 108)) and s1 == list(range(108, 116))
    assert tuple(m0) == tuple(m1) == (8, 0)
    assert t0 == t1 == [16, 0]


def test_bench_rejects_gpus_world_mismatch():
    import subprocess

    env = dict(os.environ, MSEG_BENCH_HARNESS_TEST="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


@pytest.mark.gpu
def test_bench_two_ranks_config5_on_one_gpu():
    """bench.py's N = 2 path end to end on the GPU box's one GPU (MSEG_BENCH_SHARED_GPU: both ranks on
    GPU 0, gloo for the timing and parity collectives): each rank floods its 8 config-5 frames as one
    batch call, checks them against the oracle digests, and rank 0 prints the summed count."""
    import json
    import subprocess

    env = dict(os.environ, MSEG_BENCH_SHARED_GPU="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--no-profile-pass"], env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["frames_per_rank_per_step"] == 8
    assert d["parity"].startswith("16/16 frames bit-exact"), d["parity"]
    assert "rehearsal" in d["config"]
