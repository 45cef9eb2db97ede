#!/usr/bin/env python3
"""Headline benchmark: Mpixels/sec segmented at 4096x4096 RGB (BASELINE.json metric, config 3).

One step = PictureService.watershed (PictureService.java:908-911) on one 4096x4096 synthetic
mosaic frame already resident in HBM: the exact cv::watershed flood (labels written to a separate
int32 buffer, the input markers stay pristine) + colorByIndexes(colored=false) into a BGR frame,
through libmsegment's device entry point msg_watershed_colorize_dev.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python bench.py --pipeline nc [--kind mosaic_noise]   # notConnectedMarkers'
      marker stage (gray + histogram -> levels -> markers) + watershed + colorByIndexes per step
  python bench.py --pipeline color                      # colorAutoMarkerWatershed's
      marker stage (sharpen, Otsu, chamfer distance, contours) + the flood of the sharpened frame

N > 1 (launched by torch.distributed.run, one rank per GPU): BASELINE config 5 -- rank r floods
config 5's frames 100 + 8r .. 100 + 8r + 7 as ONE batch call per step, 4 floods in flight (weak
scaling: 8 frames per GPU; at N = 8 the 64 frames of config 5).  Every rank checks its 8 label maps
against the committed oracle digests and the counts are summed over ranks ("64/64 frames bit-exact"
at N = 8).  The data path has no collectives; the only ones are the timing barriers, the
max-over-ranks of the elapsed time and that parity sum.

Rank 0 prints ONE JSON line.  Extra objects: "roofline" (dominant kernel, HIP-event timed on the
launch stream), "cpu_baseline" (the C oracle = same algorithm, timed on this host, rank 0, N=1),
and side lines that are parity cases, not the headline: "batch" (BASELINE config 5 per GPU: 8
frames per call, digest-checked), "stress" / "stress_random" (config 3's mosaic+noise and uniform
random variants, digest-checked, 1-core oracle beside them), "many_floods" (1024
notConnectedMarkers floods of 1024^2 per call in the many-floods mode, every frame checked
against the oracle, 16-thread oracle beside it; --many-frames), "correlation" (the reference's own
flood pattern: CorrelationTestService's 92 floods of ONE image per call -- 90 notConnectedMarkers
marker maps, the shape and the colour method's -- on a 1024^2 synthetic frame and on album.jpg,
every flood checked against the oracle, 16-thread oracle beside it; --correlation),
"colour_distance" (the stand-alone L-inf stencil against the HBM roofline).
"""
import argparse
import hashlib
import json
import os
import sys
import time

# Batch mode (--frames / the "batch" object) keeps several floods in flight on their own streams;
# the HIP runtime maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4, as the GPU boxes
# export).  Round 2 raised it to 8 here (4 in flight: 7250 Mpx/s at 8 queues against 5160 at 4);
# on the round-3 library the default 4 queues give the same rate (batch.hwq4 8781 against 8653 Mpx/s
# at 8, profiles/r03i_bench.json), so the bench now runs at whatever the environment sets, as a
# library user would.  The batch_hwq4 child pins exactly MSEG_BENCH_HWQ.
if os.environ.get("MSEG_BENCH_HWQ"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["MSEG_BENCH_HWQ"]

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "opencv-msegment_amd"))

METRIC = "Mpixels/sec segmented at {S}x{S} RGB; achieved HBM GB/s vs peak"  # BASELINE.json at S = 4096
METRIC_NC = "Mpixels/sec segmented by notConnectedMarkers (marker stage + watershed + colorByIndexes)"
METRIC_SHAPE = "Mpixels/sec segmented by shapeAutoMarkerWatershed (marker stage + watershed + colorByIndexes)"
METRIC_COLOR = "Mpixels/sec segmented by colorAutoMarkerWatershed (marker stage + watershed + colorByIndexes)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# Algorithmic bytes (DESIGN.md "Kernels"): what each kernel must move at minimum per unit.
BYTES_PER_PIXEL = {"k_prep": 15.0, "k_untile": 11.0, "k_colorize": 7.0, "k_edge_weights": 5.0,
                   "k_gray_hist": 4.0, "k_nc_markers": 5.0,
                   # shape marker stage: 1 B in + 1 B out per pixel for the 8-bit stencils
                   "k_gray": 4.0, "k_median": 2.0, "k_canny_nms": 2.0, "k_ring_median3": 2.0}
# Per-unit algorithmic bytes of the flood kernels whose unit is not a pixel, each over the units
# that kernel itself processed (msg_stats counts them where the work happens, so no kernel is
# priced on another's units -- round 4's stress lines priced k_resolve on every committed virtual
# item of the speculative engine and printed frac 1.19):
# k_resolve per item of the batches it decided (msg_stats.resolve_items): queue entry 4 + own
# weights 4 + 4 neighbour states 16 in, out ipx 4 + granule 8 + desc 8 (push-competitor reads are
# data dependent and not counted).
# k_spec_round per pop it ran pop by pop (msg_stats.spec_exec_pops: top pops and cascade pops of
# the executions that were not replayed, every round): queue entry 4 + own weights 4 + 4 neighbour
# states 16 in, claim 8 + label 4 + record 8 out (replayed executions' log reads are not counted).
BYTES_PER_UNIT = {"k_resolve": (44.0, "resolve_items"), "k_spec_round": (44.0, "spec_exec_pops")}
# k_scatter and k_commit_fast: per committed item 24 B (descriptor 8 + pixel 4 + granule 8 in,
# state 4 out), per appended push 8 B (queue slot 4 + state 4 out); each over the items that path
# committed (msg_stats fast_* / scatter_*)
BYTES_SCATTER = (24.0, 8.0)                 # per committed item, per appended push
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")  # scripts/pmc_summary.py output
E2E_BYTES_PER_PIXEL = 14.0                  # 3 B BGR + 4 B markers in, 4 B labels + 3 B BGR out


def frame_seed(seed, rank, world, frames=1, size=4096):
    """The first frame a rank segments: --seed, else on one GPU SURVEY 8d's seed of the config that
    size is (config 2's 1024^2 seed 1, config 3's 4096^2 seed 2, config 4's 16384^2 seed 3), else
    config 5's frame 100 + frames * rank (config 5's frames are 100 + k, k = 0..63; with 8 frames
    per rank, rank r takes 100 + 8r .. 100 + 8r + 7; replicas, no collectives)."""
    if seed is not None:
        return seed
    return {1024: 1, 16384: 3}.get(size, 2) if world == 1 else 100 + frames * rank


def default_frames(frames, world):
    """Frames per rank per step: --frames, else 1 on one GPU (the headline config 3 step) and
    BASELINE config 5's 8 per GPU (64 frames over 8 GPUs) when N > 1."""
    if frames is not None:
        return max(1, frames)
    return 1 if world == 1 else 8


def digest_parity(labels, keys, dgs):
    """(checked, bad): label maps (numpy int32) against the committed oracle digests of `keys`;
    frames without a digest are not counted."""
    checked = bad = 0
    for lab, key in zip(labels, keys):
        if key in dgs:
            checked += 1
            bad += hashlib.sha256(lab.tobytes()).hexdigest() != dgs[key]["labels_sha256"]
    return checked, bad


def reduce_sum_ints(vals, device=None):
    """Element-wise sum of a small int list over the ranks (identity on one rank)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(vals)
    t = torch.tensor(list(vals), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spawn_ranks(n, argv):
    """`--gpus N` without a launcher: start N rank processes through torch.distributed.run (one
    per GPU, rendezvous on 127.0.0.1) as children of this process, before anything here touches
    the GPU, and return their exit code.  The ranks see WORLD_SIZE and do not spawn again."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def timed_steps(step, steps, barrier, sync):
    """Barrier + sync on both sides of exactly `steps` steps; returns this rank's seconds.  Python's
    cyclic garbage collector is run before and paused inside the timed region: harness time, not the
    library's.  (Round 6: this file's timed steps took 3.7-4.9 ms per headline frame on boxes where a
    bare loop of the same call took 3.15-3.20 and the kernel trace showed every flood at ~3.2 ms --
    a one-off stall of ~15 ms inside the timed region; profiles/r06e_headline_spread.txt.)"""
    import gc

    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        barrier()
        return time.perf_counter() - t0
    finally:
        if was:
            gc.enable()


def reduce_max(x, device=None):
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def whole_job_mpx(world, npx, steps, dt_max):
    """Whole-job throughput: every rank segments `steps` frames of `npx` pixels; the job takes
    the slowest rank's time."""
    return world * npx * steps / dt_max / 1e6


def kernel_roofline(prof, stats_per_step, npx, steps):
    """Pick the kernel with the largest total time; achieved = algorithmic bytes per launch /
    average launch duration (both from the same HIP-event-timed steps)."""
    rows = []
    for name, (launches, total_ms) in prof.items():
        if launches == 0:
            continue
        if name in BYTES_PER_PIXEL:
            alg = BYTES_PER_PIXEL[name] * npx * steps
        elif name in BYTES_PER_UNIT:
            per, unit = BYTES_PER_UNIT[name]
            alg = per * stats_per_step[unit] * steps or None
        elif name == "k_scatter":
            alg = (BYTES_SCATTER[0] * stats_per_step["scatter_pops"]
                   + BYTES_SCATTER[1] * stats_per_step["scatter_pushes"]) * steps or None
        elif name == "k_commit_fast":
            alg = (BYTES_SCATTER[0] * stats_per_step["fast_pops"]
                   + BYTES_SCATTER[1] * stats_per_step["fast_pushes"]) * steps or None
        else:
            alg = None
        avg_us = 1000.0 * total_ms / launches
        gbs = (alg / launches) / (avg_us * 1e-6) / 1e9 if alg else None
        rows.append({"kernel": name, "launches_per_step": launches / steps, "avg_us": round(avg_us, 3),
                     "total_ms_per_step": round(total_ms / steps, 4),
                     "alg_bytes_per_launch": (alg / launches) if alg else None,
                     "achieved_gbs": round(gbs, 2) if gbs else None,
                     "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None})
    rows.sort(key=lambda r: -r["total_ms_per_step"])
    return rows


def cpu_baseline(img, m, depth, budget_s=12.0, max_reps=10):
    """The C oracle (same algorithm and complexity as cv::watershed + colorByIndexes), serial,
    on the SAME frame, repeated until ~budget_s of CPU work."""
    from oracle import ws_oracle

    H, W = m.shape
    reps, t_tot = 0, 0.0
    while reps < max_reps and t_tot < budget_s:
        t0 = time.perf_counter()
        lab = ws_oracle.watershed(img, m)
        ws_oracle.colorize(lab, depth, None)
        t_tot += time.perf_counter() - t0
        reps += 1
    return {"value": round(H * W * reps / t_tot / 1e6, 3), "unit": "Mpx/s", "cores": 1, "kind": "port",
            "sample": "%d full %dx%d frame(s): oracle/ws_oracle.c watershed + colorize, 1 thread, %.1f s"
                      % (reps, H, W, t_tot)}, lab


def cpu_baseline_nc(img, depth_opt, options, budget_s=12.0, max_reps=10):
    """The oracles of the NC pipeline (numpy marker stage + the C flood), serial, same frame."""
    from oracle import nc_oracle, ws_oracle

    H, W = img.shape[:2]
    reps, t_tot = 0, 0.0
    while reps < max_reps and t_tot < budget_s:
        t0 = time.perf_counter()
        _, _, lv, mk = nc_oracle.marker_stage(img, depth_opt, gisto_diap="GISTO_DIAP" in options)
        lab = ws_oracle.watershed(img, mk)
        ws_oracle.colorize(lab, len(lv), None)
        t_tot += time.perf_counter() - t0
        reps += 1
    return {"value": round(H * W * reps / t_tot / 1e6, 3), "unit": "Mpx/s", "cores": 1, "kind": "port",
            "comparable": False,
            "note": "numpy restatement of the marker stage, not an OpenCV-class C implementation: "
                    "not comparable, no ratio quoted (the flood leg is the C oracle)",
            "sample": "%d full %dx%d frame(s): oracle/nc_oracle.py marker stage (numpy) + ws_oracle.c "
                      "watershed + colorize, 1 thread, %.1f s" % (reps, H, W, t_tot)}, lab


def cpu_baseline_shape(img, budget_s=12.0, max_reps=10, rows=512):
    """The oracles of the shape pipeline (numpy/scipy marker stage + the C flood) on a band of the
    frame (the first `rows` rows, the full frame's median size), bounded to ~budget_s."""
    import numpy as np

    from oracle import shape_oracle, ws_oracle

    k = shape_oracle.blur_mask_size(*img.shape[:2])
    img = np.ascontiguousarray(img[:rows])
    H, W = img.shape[:2]
    reps, t_tot = 0, 0.0
    while reps < max_reps and t_tot < budget_s:
        t0 = time.perf_counter()
        mk, depth = shape_oracle.shape_markers(img, k)
        lab = ws_oracle.watershed(img, mk)
        ws_oracle.colorize(lab, depth, None)
        t_tot += time.perf_counter() - t0
        reps += 1
    return {"value": round(H * W * reps / t_tot / 1e6, 3), "unit": "Mpx/s", "cores": 1, "kind": "port",
            "comparable": False,
            "note": "numpy/scipy restatement of the marker stage, not an OpenCV-class C implementation "
                    "(OpenCV's O(1) median and SIMD Canny are far faster): not comparable, no ratio quoted",
            "sample": "%d band(s) of %dx%d (median %d as for the full frame): oracle/shape_oracle.py "
                      "marker stage (numpy/scipy) + ws_oracle.c watershed + colorize, 1 thread, %.1f s"
                      % (reps, H, W, k, t_tot)}, None


def cpu_baseline_color(img, budget_s=12.0, max_reps=10, rows=512):
    """The oracles of the colour pipeline (numpy + C chamfer marker stage, the C flood) on a band of
    the frame (its first `rows` rows), bounded to ~budget_s."""
    import numpy as np

    from oracle import color_oracle, ws_oracle

    img = np.ascontiguousarray(img[:rows])
    H, W = img.shape[:2]
    reps, t_tot = 0, 0.0
    while reps < max_reps and t_tot < budget_s:
        t0 = time.perf_counter()
        sharp, mk, depth = color_oracle.color_markers(img)
        lab = ws_oracle.watershed(sharp, mk)
        ws_oracle.colorize(lab, depth, None)
        t_tot += time.perf_counter() - t0
        reps += 1
    return {"value": round(H * W * reps / t_tot / 1e6, 3), "unit": "Mpx/s", "cores": 1, "kind": "port",
            "comparable": False,
            "note": "numpy/scipy restatement of the marker stage, not an OpenCV-class C implementation: "
                    "not comparable, no ratio quoted",
            "sample": "%d band(s) of %dx%d: oracle/color_oracle.py marker stage (numpy/scipy, C chamfer) + "
                      "ws_oracle.c watershed + colorize, 1 thread, %.1f s" % (reps, H, W, t_tot)}, None


def batch_throughput(seg, args, S, seed, sync, steps=5, warmup=2):
    """BASELINE config 5 on this GPU: --batch-frames frames of the same workload per call, up to
    --inflight floods in flight (msg_watershed_colorize_batch_dev); whole-batch Mpx/s.  `seed` is
    the first frame's seed: SURVEY 8(d) numbers config 5's 64 frames 100+k, k = 0..63, so rank r
    of 8 takes frames 100 + 8r .. 100 + 8r + 7."""
    import torch

    from msegment import synth

    K = args.batch_frames
    dev = torch.device("cuda", torch.cuda.current_device())
    fr = [synth.frame(args.kind, S, S, seed + k) for k in range(K)]
    depth = max(f[2] for f in fr)
    imgs = [torch.from_numpy(f[0]).to(dev) for f in fr]
    mks = [torch.from_numpy(f[1]).to(dev) for f in fr]
    labs = [torch.empty_like(m) for m in mks]
    dsts = [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in fr]
    seg.set_batch_inflight(args.inflight)
    for _ in range(warmup):
        seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
    sync()
    dt = time.perf_counter() - t0
    # every frame of the timed batch against its committed oracle digest, where there is one
    dgs = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    checked = bad = 0
    for k in range(K):
        key = "%s_%dx%d_s%d" % (args.kind, S, S, seed + k)
        if key in dgs:
            checked += 1
            bad += hashlib.sha256(labs[k].cpu().numpy().tobytes()).hexdigest() != dgs[key]["labels_sha256"]
    parity = ("%d/%d frames bit-exact vs oracle digests" % (checked - bad, checked)) if checked else None
    del imgs, mks, labs, dsts
    return {"value": round(K * S * S * steps / dt / 1e6, 3), "unit": "Mpx/s", "frames": K,
            "inflight": min(K, args.inflight), "steps": steps, "parity": parity,
            "note": "BASELINE config 5 per GPU: %d frames (seeds %d..%d) per call, floods overlapped"
                    % (K, seed, seed + K - 1)}


def batch_hwq4(args, S, seed):
    """The batch line pinned to GPU_MAX_HW_QUEUES=4 (the boxes' default; this process runs at
    whatever the environment sets): a child process with exactly 4 queues runs the same batch at
    2, 3 and 4 floods in flight."""
    import subprocess

    env = dict(os.environ, MSEG_BENCH_HWQ="4")
    cmd = [sys.executable, os.path.abspath(__file__), "--batch-only", "--size", str(S), "--kind", args.kind,
           "--seed", str(seed), "--batch-frames", str(args.batch_frames)]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        return json.loads(line)
    except Exception as e:  # noqa: BLE001 -- reported, not fatal to the headline line
        return {"error": "batch_hwq4 child failed: %s" % e}


def batch_only(args):
    """--batch-only (the batch_hwq4 child): batch throughput at 2, 3, 4 floods in flight."""
    import torch

    import msegment

    torch.cuda.set_device(0)
    seg = msegment.Segmenter(0)
    sync = torch.cuda.synchronize
    rows = {}
    for k in (2, 3, 4):
        args.inflight = k
        rows[str(k)] = batch_throughput(seg, args, args.size, args.seed, sync)["value"]
    seg.close()
    best = max(rows, key=lambda k: rows[k])
    print(json.dumps({"value": rows[best], "unit": "Mpx/s", "inflight": int(best), "by_inflight": rows,
                      "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "note": "the batch line at the boxes' default GPU_MAX_HW_QUEUES=4 (child process)"}),
          flush=True)
    return 0


def batch_cpu_threads(K):
    """Threads for the batch CPU baseline: OMP_NUM_THREADS (16 on the GPU boxes), at most 16, at
    most one per frame."""
    n = int(os.environ.get("OMP_NUM_THREADS", "8") or 8)
    return max(1, min(n, 16, K))


def cpu_baseline_batch(kind, S, seed, K):
    """SURVEY 8(d) batch baseline: the K frames on the host's cores (the same thread count as the
    many-floods baseline: every thread gets a frame, the K frames repeated as needed), one frame per
    thread (the C oracle runs without the GIL inside ctypes), aggregate Mpx/s over one pass."""
    from concurrent.futures import ThreadPoolExecutor

    from msegment import synth
    from oracle import ws_oracle

    nt = batch_cpu_threads(16)
    fr = [synth.frame(kind, S, S, seed + k) for k in range(K)]
    work = [fr[i % K] for i in range(max(K, nt))]

    def one(f):
        ws_oracle.colorize(ws_oracle.watershed(f[0], f[1]), f[2], None)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(nt) as ex:
        list(ex.map(one, work))
    dt = time.perf_counter() - t0
    return {"value": round(len(work) * S * S / dt / 1e6, 3), "unit": "Mpx/s", "cores": nt, "kind": "port",
            "sample": "%d floods of the %d %s %dx%d frames (seeds %d..%d), one flood per thread: "
                      "oracle/ws_oracle.c watershed + colorize, %.1f s" % (len(work), K, kind, S, S, seed,
                                                                            seed + K - 1, dt)}


def many_floods_line(seg, sync, dev, K, S=1024, steps=2, cpu=True, nc_depth=4):
    """The reference's real call pattern for the flood: many floods whose seeds put cv::watershed's
    exact order in its serial regime -- notConnectedMarkers' scattered seeds (PictureService.java:852,
    90 times per image from CorrelationTestService.java:84-86, 141).  K frames (mosaic+noise SxS,
    seeds 100..100+K-1), their NC markers from the GPU marker stage (GISTO_DIAP, depth nc_depth;
    outside the timed region), then per step ONE batch call of all K floods + colorByIndexes in the
    many-floods mode (msg_set_batch_floods 1: one k_serial_multi launch, one wave per flood).
    Beside it: the default batch path (the full engine per flood, 4 in flight) on the first 8
    frames, and the C oracle on 8 threads over all K frames, whose labels are the parity check."""
    import numpy as np
    import torch

    from msegment import synth

    from concurrent.futures import ThreadPoolExecutor

    # ~0.1 s of numpy hashing per 1024^2 frame: synthesised on the host threads (numpy drops the GIL)
    with ThreadPoolExecutor(batch_cpu_threads(K)) as ex:
        fr = list(ex.map(lambda k: synth.frame("mosaic_noise", S, S, 100 + k)[0], range(K)))
    imgs = [torch.from_numpy(f).to(dev) for f in fr]
    mks = [torch.empty((S, S), dtype=torch.int32, device=dev) for _ in fr]
    depth = 1
    for t_img, t_m in zip(imgs, mks):
        depth = max(depth, len(seg.nc_marker_stage_dev(t_img, nc_depth, t_m, 1)))  # GISTO_DIAP
    sync()
    labs = [torch.empty_like(m) for m in mks]
    dsts = [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in fr]
    seg.set_batch_floods(1)
    try:
        seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)  # warm-up (workspaces)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
        sync()
        dt = time.perf_counter() - t0
    finally:
        seg.set_batch_floods(0)  # releases the mode's workspaces; then back to the default (automatic)
        seg.set_batch_floods(3)
    st = seg.stats()
    out = {"workload": "%d notConnectedMarkers floods (mosaic_noise %dx%d seeds 100..%d, GISTO_DIAP depth %d "
                       "markers) + colorByIndexes per batch call, device-resident, many-floods mode"
                       % (K, S, S, 99 + K, nc_depth),
           "value": round(K * S * S * steps / dt / 1e6, 3), "unit": "Mpx/s", "steps": steps,
           "ms_per_step": round(1000.0 * dt / steps, 3), "pops_per_step": st["pops"]}
    # the full engine per flood (mode 0, 4 streams in flight) on the first 8 frames
    k8 = min(8, K)
    seg.set_batch_inflight(4)
    seg.set_batch_floods(0)
    try:
        t0 = time.perf_counter()
        seg.watershed_colorize_batch_dev(imgs[:k8], mks[:k8], labs[:k8], depth, None, dsts[:k8])
        sync()
        out["mode0_batch_path"] = {"value": round(k8 * S * S / (time.perf_counter() - t0) / 1e6, 3),
                                   "unit": "Mpx/s", "frames": k8, "inflight": 4,
                                   "note": "msg_set_batch_floods 0: the full engine per flood"}
    finally:
        seg.set_batch_floods(3)
    if cpu:
        from oracle import ws_oracle

        nt = batch_cpu_threads(K)
        m_host = [m.cpu().numpy() for m in mks]

        def one(k):
            lab = ws_oracle.watershed(fr[k], m_host[k])
            ws_oracle.colorize(lab, depth, None)
            return lab

        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            want = list(ex.map(one, range(K)))
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(K * S * S / cdt / 1e6, 3), "unit": "Mpx/s", "cores": nt,
                               "kind": "port", "sample": "the same %d floods (the GPU's markers), one frame "
                               "per thread: oracle/ws_oracle.c watershed + colorize, %.1f s" % (K, cdt)}
        bad = sum(not np.array_equal(labs[k].cpu().numpy(), want[k]) for k in range(K))
        out["parity"] = "%d/%d frames bit-exact vs the C oracle" % (K - bad, K)
    del imgs, mks, labs, dsts
    return out


# CorrelationTestService.test (CorrelationTestService.java:28-40, 84-99): per image, the colour and
# shape methods once and notConnectedMarkers for every depth x mask size x option set -- 92 floods
# of ONE image per test, each through PictureService.watershed (PictureService.java:378, 455, 852)
CORR_DEPTHS = (2, 3, 4, 5, 6)
CORR_MASKS = (3, 5, 7)
CORR_OPTS = (("MEDIAN_BLUR",), ("MEDIAN_BLUR", "GISTO_DIAP"), ("BILATERIAL",), ("BILATERIAL", "GISTO_DIAP"),
             (), ("GISTO_DIAP",))
NC_FLAG = {"GISTO_DIAP": 0x1, "MULTI_OTSU": 0x2, "MEDIAN_BLUR": 0x4, "BILATERIAL": 0x8}


def correlation_image(name):
    """The image of the correlation line: 'album' = the reference's own album.jpg (1500^2, decoded
    pixels in tests/golden/album_1500x1500.png), else a synthetic 1024^2 frame of that kind."""
    import numpy as np

    from msegment import synth

    if name == "album":
        from PIL import Image

        rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
        return np.ascontiguousarray(rgb[:, :, ::-1]), "album.jpg 1500x1500 (tests/golden)"
    return synth.frame(name, 1024, 1024, 100)[0], "%s 1024x1024 seed 100" % name


def correlation_markers(seg, dev, t_img):
    """CorrelationTestService.test's 92 marker maps of one image (device tensor t_img) from the GPU
    marker stages: (flood sources, markers, depths, names, the colour method's sharpened image)."""
    import torch

    H, W = t_img.shape[:2]
    srcs, mks, depths, names = [], [], [], []
    for depth in CORR_DEPTHS:
        for mask in CORR_MASKS:
            for opts in CORR_OPTS:
                m = torch.empty((H, W), dtype=torch.int32, device=dev)
                flags = sum(NC_FLAG[o] for o in opts) | ((mask & 0xff) << 8)
                lv = seg.nc_marker_stage_dev(t_img, depth, m, flags)
                srcs.append(t_img)
                mks.append(m)
                depths.append(len(lv))
                names.append("NC,%d,%d,%s" % (depth, mask, "-".join(opts)))
    m = torch.empty((H, W), dtype=torch.int32, device=dev)
    d, _ = seg.shape_markers_dev(t_img, m)
    srcs.append(t_img)
    mks.append(m)
    depths.append(d)
    names.append("SHAPE")
    t_sharp = torch.empty_like(t_img)
    m = torch.empty((H, W), dtype=torch.int32, device=dev)
    depths.append(seg.color_markers_dev(t_img, t_sharp, m))
    srcs.append(t_sharp)
    mks.append(m)
    names.append("COLOR")
    return srcs, mks, depths, names, t_sharp


def correlation_mass_line(seg, sync, dev, images=8, S=1024, cpu=True, steps=2):
    """CorrelationTestService.massTest (CorrelationTestService.java:49-53) runs test() over a map of
    images: batched at that level, the 92 floods of each of `images` images (1024^2 noisy mosaics,
    seeds 100..) go to ONE call -- the many-floods kernel then has 92 x images floods in flight.
    Every flood checked against the C oracle; the 16-thread oracle over the same floods beside it."""
    import numpy as np
    import torch

    from msegment import synth

    srcs, mks, depths, keep = [], [], [], []
    for k in range(images):
        t_img = torch.from_numpy(synth.frame("mosaic_noise", S, S, 100 + k)[0]).to(dev)
        s_k, m_k, d_k, _, t_sharp = correlation_markers(seg, dev, t_img)
        srcs += s_k
        mks += m_k
        depths += d_k
        keep += [t_img, t_sharp]
    sync()
    n = len(mks)
    depth = max(depths)
    labs = [torch.empty_like(x) for x in mks]
    dsts = [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in mks]
    seg.set_batch_floods(1)
    try:
        seg.watershed_colorize_batch_dev(srcs, mks, labs, depth, None, dsts)  # warm-up (workspaces)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            seg.watershed_colorize_batch_dev(srcs, mks, labs, depth, None, dsts)
        sync()
        dt = time.perf_counter() - t0
    finally:
        seg.set_batch_floods(0)
        seg.set_batch_floods(3)
    out = {"workload": "CorrelationTestService.massTest batched: %d images (mosaic_noise %dx%d seeds 100..%d) x 92 "
                       "floods (90 notConnectedMarkers marker maps, the shape and the colour method's) = %d floods "
                       "+ colorByIndexes in ONE batch call, device-resident, many-floods mode"
                       % (images, S, S, 99 + images, n),
           "value": round(n * S * S * steps / dt / 1e6, 3), "unit": "Mpx/s", "floods": n, "steps": steps,
           "ms_per_step": round(1000.0 * dt / steps, 3)}
    if cpu:
        from concurrent.futures import ThreadPoolExecutor

        from oracle import ws_oracle

        nt = batch_cpu_threads(n)
        src_host = {id(x): x.cpu().numpy() for x in keep}
        m_host = [x.cpu().numpy() for x in mks]

        def one(k):
            lab = ws_oracle.watershed(src_host[id(srcs[k])], m_host[k])
            ws_oracle.colorize(lab, depth, None)
            return lab

        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            want = list(ex.map(one, range(n)))
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n * S * S / cdt / 1e6, 3), "unit": "Mpx/s", "cores": nt, "kind": "port",
                               "sample": "the same %d floods (the GPU's marker maps), one flood per thread: "
                                         "oracle/ws_oracle.c watershed + colorize, %.2f s" % (n, cdt)}
        bad = sum(not np.array_equal(labs[k].cpu().numpy(), want[k]) for k in range(n))
        out["parity"] = "%d/%d floods bit-exact vs the C oracle" % (n - bad, n)
        del want, m_host
    del srcs, mks, labs, dsts, keep
    torch.cuda.empty_cache()
    return out


def correlation_line(seg, sync, dev, name, cpu=True, steps=2):
    """The reference's real call pattern for the flood: CorrelationTestService floods ONE image 92
    times per test -- 90 notConnectedMarkers marker maps (5 depths x 3 mask sizes x 6 option sets),
    the shape method's and the colour method's (whose flood source is the sharpened image).  The
    marker maps come from the GPU marker stages (outside the timed region); each step is ONE batch
    call of the 92 floods + colorByIndexes in the many-floods mode (msg_set_batch_floods 1), the
    default batch path (full engine per flood, 4 in flight) timed once beside it, and the C oracle
    over the same 92 floods on the host's threads, whose labels are the parity check."""
    import numpy as np
    import torch

    img, desc = correlation_image(name)
    H, W = img.shape[:2]
    t_img = torch.from_numpy(img).to(dev)
    srcs, mks, depths, names, t_sharp = correlation_markers(seg, dev, t_img)
    sync()
    n = len(mks)
    depth = max(depths)
    labs = [torch.empty_like(x) for x in mks]
    dsts = [torch.empty((H, W, 3), dtype=torch.uint8, device=dev) for _ in mks]
    seg.set_batch_floods(1)
    try:
        seg.watershed_colorize_batch_dev(srcs, mks, labs, depth, None, dsts)  # warm-up (workspaces)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            seg.watershed_colorize_batch_dev(srcs, mks, labs, depth, None, dsts)
        sync()
        dt = time.perf_counter() - t0
    finally:
        seg.set_batch_floods(0)
        seg.set_batch_floods(3)
    st = seg.stats()
    out = {"workload": "CorrelationTestService.test's %d floods of ONE image (%s): 90 notConnectedMarkers "
                       "marker maps (depths 2-6 x masks 3,5,7 x 6 option sets), the shape and the colour "
                       "method's, + colorByIndexes, one batch call, device-resident, many-floods mode"
                       % (n, desc),
           "value": round(n * H * W * steps / dt / 1e6, 3), "unit": "Mpx/s", "floods": n, "steps": steps,
           "ms_per_step": round(1000.0 * dt / steps, 3), "pops_per_step": st["pops"]}
    # the library's default (msg_set_batch_floods 3, automatic): the first call of a frame size
    # floods frame 0 alone as a probe and picks the path for the rest; the second call reuses it
    seg.set_batch_inflight(4)
    auto = []
    for _ in range(2):
        t0 = time.perf_counter()
        seg.watershed_colorize_batch_dev(srcs, mks, labs, depth, None, dsts)
        sync()
        sa = seg.stats()
        auto.append({"value": round(n * H * W / (time.perf_counter() - t0) / 1e6, 3), "unit": "Mpx/s",
                     "batch_mode": sa["batch_mode"], "probe": bool(sa["batch_probe"])})
    out["default_path"] = {"first_call": auto[0], "second_call": auto[1],
                           "note": "msg_set_batch_floods 3 (the default): frame 0 probed alone on the first call"}
    # the full engine per flood (mode 0, 4 in flight) on the first 8 floods
    seg.set_batch_floods(0)
    try:
        t0 = time.perf_counter()
        seg.watershed_colorize_batch_dev(srcs[:8], mks[:8], labs[:8], depth, None, dsts[:8])
        sync()
        out["mode0_batch_path"] = {"value": round(8 * H * W / (time.perf_counter() - t0) / 1e6, 3), "unit": "Mpx/s",
                                   "floods": 8, "inflight": 4, "note": "msg_set_batch_floods 0, the first 8 floods"}
    finally:
        seg.set_batch_floods(3)
    if cpu:
        from concurrent.futures import ThreadPoolExecutor

        from oracle import ws_oracle

        nt = batch_cpu_threads(n)
        src_host = {id(x): x.cpu().numpy() for x in (t_img, t_sharp)}
        m_host = [x.cpu().numpy() for x in mks]

        def one(k):
            lab = ws_oracle.watershed(src_host[id(srcs[k])], m_host[k])
            ws_oracle.colorize(lab, depth, None)
            return lab

        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            want = list(ex.map(one, range(n)))
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n * H * W / cdt / 1e6, 3), "unit": "Mpx/s", "cores": nt, "kind": "port",
                               "sample": "the same %d floods (the GPU's marker maps), one flood per thread: "
                                         "oracle/ws_oracle.c watershed + colorize, %.2f s" % (n, cdt)}
        bad = [names[k] for k in range(n) if not np.array_equal(labs[k].cpu().numpy(), want[k])]
        out["parity"] = "%d/%d floods bit-exact vs the C oracle%s" % (n - len(bad), n,
                                                                    (" (differ: %s)" % bad[:4]) if bad else "")
    del srcs, mks, labs, dsts, t_img, t_sharp
    return out


def stress_line(seg, S, sync, dev, steps, cpu=True, kind="mosaic_noise", seed=2):
    """BASELINE config 3's stress variant beside the headline: mosaic+noise SxS seed 2 (the
    interrupt-dense regime: per-channel noise makes pushes below the popped level every few pops),
    the same device-resident step, its parity against the committed oracle digest, and the C
    oracle timed on the same frame (1 thread)."""
    import numpy as np
    import torch

    from msegment import synth

    import msegment

    img, m, depth = synth.frame(kind, S, S, seed)
    t_img = torch.from_numpy(img).to(dev)
    t_m = torch.from_numpy(m).to(dev)
    t_lab = torch.empty_like(t_m)
    t_dst = torch.empty((S, S, 3), dtype=torch.uint8, device=dev)
    # the first flood of a fresh context (workspace allocation included), timed on its own: the
    # timed steps below reuse the bench context, so a first-flood cliff would not show in them
    sync()
    t0 = time.perf_counter()
    fresh = msegment.Segmenter(dev.index)
    fresh.watershed_colorize_dev(t_img, t_m, t_lab, depth, None, t_dst)
    sync()
    first_ms = 1000.0 * (time.perf_counter() - t0)
    fresh.close()
    seg.watershed_colorize_dev(t_img, t_m, t_lab, depth, None, t_dst)
    sync()
    st = seg.stats()
    dkey = "%s_%dx%d_s%d" % (kind, S, S, seed)
    dgs = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    lab = t_lab.cpu().numpy()
    parity = None
    if dkey in dgs:
        parity = ("bit-exact vs oracle digest " if hashlib.sha256(lab.tobytes()).hexdigest()
                  == dgs[dkey]["labels_sha256"] else "MISMATCH vs oracle digest ") + dkey
    t0 = time.perf_counter()
    for _ in range(steps):
        seg.watershed_colorize_dev(t_img, t_m, t_lab, depth, None, t_dst)
    sync()
    dt = time.perf_counter() - t0
    value = S * S * steps / dt / 1e6
    out = {"workload": "%s %dx%d seed %d, watershed + colorByIndexes(colored=false), device-resident "
                       "(BASELINE config 3 stress variant)" % (kind, S, S, seed),
           "value": round(value, 3), "unit": "Mpx/s", "steps": steps,
           "ms_per_step": round(1000.0 * dt / steps, 3), "parity": parity,
           "first_flood_ms": round(first_ms, 3),
           "first_flood_note": "one step on a freshly created context (its workspace allocation included)"}
    # the dominant kernel of the same step, HIP-event timed (one profiled step); the flood's
    # counters from that step (the first flood of a context may run part of the way without the
    # speculative engine, which is allocated on first use)
    seg.set_profiling(True)
    seg.kernel_profile(reset=True)
    seg.watershed_colorize_dev(t_img, t_m, t_lab, depth, None, t_dst)
    sync()
    prof = seg.kernel_profile(reset=True)
    seg.set_profiling(False)
    st = seg.stats()
    out["flood"] = {"batches": st["batches"], "pops": st["pops"], "items": st["items"],
                    "spec_generations": st["spec_generations"], "spec_rounds": st["spec_rounds"],
                    "spec_executions": st["spec_executions"], "spec_replays": st["spec_replays"],
                    "spec_fallbacks": st["spec_fallbacks"],
                    "executions_per_pop": round(st["spec_executions"] / max(1, st["pops"]), 3),
                    # executions that ran their cascade pop by pop (the rest replayed the last round's)
                    "full_executions_per_pop": round((st["spec_executions"] - st["spec_replays"]) / max(1, st["pops"]), 3)}
    kern = kernel_roofline(prof, st, S * S, 1)
    out["kernels"] = kern
    top = kern[0] if kern else None
    e2e = value * 1e6 * E2E_BYTES_PER_PIXEL / 1e9
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "e2e_achieved": round(e2e, 3), "e2e_frac": round(e2e / HBM_PEAK_GBS, 6)}
    if top:
        traffic, tsrc = pmc_traffic(top["kernel"], {"pipeline": "watershed", "kind": kind, "size": S, "seed": seed,
                                                    "frames": 1})
        roof.update({"kernel": top["kernel"], "achieved": top["achieved_gbs"],
                     "frac": round(top["achieved_gbs"] / HBM_PEAK_GBS, 6) if top["achieved_gbs"] else None,
                     "alg_bytes_per_launch": top["alg_bytes_per_launch"], "avg_launch_us": top["avg_us"],
                     "launches": round(top["launches_per_step"], 1), "traffic": traffic, "traffic_source": tsrc})
    out["roofline"] = roof
    if cpu:
        c, cl = cpu_baseline(img, m, depth, budget_s=8.0, max_reps=5)
        out["cpu_baseline"] = c
        if parity is None:
            out["parity"] = "bit-exact vs oracle" if np.array_equal(cl, lab) else "MISMATCH vs oracle"
    del t_img, t_m, t_lab, t_dst
    return out


def pmc_build_id(pm):
    """The libmsegment build a PMC summary's counters came from (its "build_id", or the id its note
    names: scripts/gpu_check.sh writes "libmsegment build <id>")."""
    import re

    if pm.get("build_id"):
        return pm["build_id"]
    m = re.search(r"build ([0-9a-f]{16})", pm.get("note", ""))
    return m.group(1) if m else None


def pmc_traffic(kernel, cfg):
    """HBM bytes per launch of `kernel` from the committed PMC passes (profiles/pmc_*.json,
    scripts/pmc_summary.py), only from a file collected on this same workload `cfg` AND on the
    library build this process loaded: counters of another build are not quoted (traffic None, the
    source says which build they came from)."""
    import glob

    import msegment

    here = msegment._lib.load().msg_build_id().decode()
    stale = None
    for path in [PMC_SUMMARY] + sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        if not os.path.exists(path):
            continue
        pm = json.load(open(path))
        kk = pm.get("kernels", {}).get(kernel)
        if kk and pm.get("config") == cfg:
            bid = pmc_build_id(pm)
            if bid != here:
                stale = stale or "not quoted: %s holds counters of build %s, this library is build %s" % (
                    os.path.relpath(path, ROOT), bid, here)
                continue
            return round(kk["hbm_bytes_per_launch"]), "%s (%s; %s)" % (
                os.path.relpath(path, ROOT), pm.get("correction"), pm.get("note", ""))
    return None, stale


def colour_distance(seg, t_img, img, S, sync, pmc_cfg, reps=20, check=True):
    """The stand-alone colour-distance stencil (msg_edge_weights_dev) on the bench
    frame: HIP-event-timed launches, 5 algorithmic bytes per pixel (3 in, 2 out); its output is
    checked against numpy on the same frame."""
    import numpy as np
    import torch

    wr = torch.empty((S, S), dtype=torch.uint8, device=t_img.device)
    wd = torch.empty_like(wr)
    seg.edge_weights_dev(t_img, wr, wd)
    sync()
    ok = None
    if check:
        x = img.astype(np.int16)
        er = np.zeros((S, S), np.uint8)
        ed = np.zeros((S, S), np.uint8)
        er[:, :-1] = np.abs(x[:, 1:] - x[:, :-1]).max(axis=2)
        ed[:-1] = np.abs(x[1:] - x[:-1]).max(axis=2)
        ok = bool(np.array_equal(wr.cpu().numpy(), er) and np.array_equal(wd.cpu().numpy(), ed))
    seg.set_profiling(True)
    seg.kernel_profile(reset=True)
    for _ in range(reps):
        seg.edge_weights_dev(t_img, wr, wd)
    sync()
    prof = seg.kernel_profile(reset=True)
    seg.set_profiling(False)
    launches, total_ms = prof.get("k_edge_weights", (0, 0.0))
    if not launches:
        return None
    avg_us = 1000.0 * total_ms / launches
    # the same launches back to back on one stream between two events (no event pair around
    # each launch: that pair adds a few us of its own to a 13-us kernel); the span still holds
    # the kernel boundaries, so it is an upper bound on the kernel's own duration
    s = torch.cuda.Stream(device=t_img.device)
    s.wait_stream(torch.cuda.current_stream(t_img.device))
    with torch.cuda.stream(s):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        seg.edge_weights_dev(t_img, wr, wd)
        e0.record(s)
        for _ in range(reps):
            seg.edge_weights_dev(t_img, wr, wd)
        e1.record(s)
    s.synchronize()
    span_us = 1000.0 * e0.elapsed_time(e1) / reps
    gbs = BYTES_PER_PIXEL["k_edge_weights"] * S * S / (span_us * 1e-6) / 1e9
    traffic, _ = pmc_traffic("k_edge_weights16", pmc_cfg)
    return {"bound": "hbm", "kernel": "k_edge_weights16", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5), "avg_launch_us": round(span_us, 3),
            "timing": "%d back-to-back launches between two HIP events on the launch stream" % reps,
            "avg_launch_us_event_pairs": round(avg_us, 3),
            "alg_bytes_per_launch": BYTES_PER_PIXEL["k_edge_weights"] * S * S, "traffic": traffic,
            "launches": launches, "parity": None if ok is None else ("bit-exact vs numpy" if ok else "MISMATCH")}


def harness_test(args, rank, world):
    """Test-only (tests/test_dist.py, CPU): the launch / barrier / max-over-ranks / JSON path of
    this file over gloo with a 5 ms sleep as the step.  Measures nothing about the GPU path and
    says so in its line; never selected unless MSEG_BENCH_HARNESS_TEST is set."""
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    for _ in range(args.warmup):
        time.sleep(0.005)
    dt = timed_steps(lambda: time.sleep(0.005), args.steps, barrier, lambda: None)
    dt_max = reduce_max(dt)
    if rank == 0:
        print(json.dumps({"metric": "bench.py harness test (no GPU)", "value": round(world * args.steps / dt_max, 3),
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(1000.0 * dt_max / args.steps, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": None,
                          "data": "harness test: each rank's step is a 5 ms sleep",
                          "config": {"workload": "harness test", "parallelism": "replicas%d" % world}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher N > 1 spawns them (torch.distributed.run)")
    ap.add_argument("--steps", type=int, default=None, help="default 10 (nc: 2)")
    ap.add_argument("--warmup", type=int, default=None, help="default 3 (nc: 1)")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--kind", default="mosaic", choices=["mosaic", "mosaic_noise", "random"])
    ap.add_argument("--seed", type=int, default=None, help="default: 2 (N=1), 100+frames*rank (N>1)")
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per rank per step; default 1 on one GPU (the headline single-frame "
                         "step, config 3) and 8 when N > 1 (BASELINE config 5: 64 frames over 8 GPUs)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="floods kept in flight together when --frames > 1")
    ap.add_argument("--batch-frames", type=int, default=8,
                    help="frames of the extra 'batch' measurement (config 5 per GPU); 0/1 = skip")
    ap.add_argument("--pipeline", default="watershed", choices=["watershed", "nc", "shape", "color"],
                    help="nc: notConnectedMarkers' marker stage builds the seeds each step; "
                         "shape: shapeAutoMarkerWatershed's (median, Canny, rings, components)")
    ap.add_argument("--nc-depth", type=int, default=4, help="user depth of the nc pipeline")
    ap.add_argument("--nc-options", default="GISTO_DIAP", help="comma list: GISTO_DIAP,MULTI_OTSU")
    ap.add_argument("--stress-steps", type=int, default=5,
                    help="steps of the config-3 stress line (mosaic+noise at --size); 0 = skip")
    ap.add_argument("--many-frames", type=int, default=1024,
                    help="frames of the many-floods line (0: skip it)")
    ap.add_argument("--correlation", default="mosaic_noise,album",
                    help="images of the correlation line (CorrelationTestService's 92 floods of one image "
                         "per call): comma list of mosaic_noise / random / mosaic (1024^2) / album; '' = skip")
    ap.add_argument("--correlation-images", type=int, default=8,
                    help="images of the correlation line's massTest object (92 floods each, one call); 0 = skip")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile-pass", action="store_true")
    ap.add_argument("--batch-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-hwq4", action="store_true", help="skip the batch_hwq4 child process")
    args = ap.parse_args(argv)
    if args.batch_only:
        if args.seed is None:
            args.seed = 100
        return batch_only(args)
    # the nc pipeline's scattered seeds put the flood in its slowest regime
    if args.steps is None:
        args.steps = 2 if args.pipeline in ("nc", "color") else 10
    if args.warmup is None:
        args.warmup = 1 if args.pipeline in ("nc", "color") else 3

    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:] if argv is None else argv))
    rank, world, local = dist_env()
    if args.gpus is not None and world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks" % (args.gpus, world))
    if os.environ.get("MSEG_BENCH_HARNESS_TEST"):
        return harness_test(args, rank, world)
    import numpy as np
    import torch
    import torch.distributed as dist

    import msegment
    from msegment import synth

    # MSEG_BENCH_SHARED_GPU=1 (rehearsal of the N > 1 path on a one-GPU box): every rank on GPU 0
    # and gloo for the timing / parity collectives (RCCL refuses two ranks on one GPU); the line says
    # so.  Never set by the driver's runs.
    shared = bool(os.environ.get("MSEG_BENCH_SHARED_GPU")) and world > 1
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = None if shared else dev  # where the collectives' tensors live
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    sync = torch.cuda.synchronize

    S = args.size
    K = default_frames(args.frames, world)
    seed = frame_seed(args.seed, rank, world, K, S)
    # the workload the PMC passes must have been collected on for their traffic to be quoted
    pmc_cfg = {"pipeline": args.pipeline, "kind": args.kind, "size": S, "seed": seed, "frames": K}
    t0 = time.perf_counter()
    img, m, depth = synth.frame(args.kind, S, S, seed)
    log("[rank %d] generated %s %dx%d seed %d in %.1fs" % (rank, args.kind, S, S, seed, time.perf_counter() - t0))
    t_img = torch.from_numpy(img).to(dev)
    t_m = torch.from_numpy(m).to(dev)
    t_lab = torch.empty_like(t_m)
    t_dst = torch.empty((S, S, 3), dtype=torch.uint8, device=dev)
    seg = msegment.Segmenter(local)
    if K > 1:  # K frames (seeds seed..seed+K-1) per step, up to --inflight floods in flight
        extra = [synth.frame(args.kind, S, S, seed + k) for k in range(1, K)]
        b_img = [t_img] + [torch.from_numpy(f[0]).to(dev) for f in extra]
        b_m = [t_m] + [torch.from_numpy(f[1]).to(dev) for f in extra]
        b_lab = [t_lab] + [torch.empty_like(x) for x in b_m[1:]]
        b_dst = [t_dst] + [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in extra]
        depth = max([depth] + [f[2] for f in extra])
        seg.set_batch_inflight(args.inflight)

    def step1():
        seg.watershed_colorize_dev(t_img, t_m, t_lab, depth, None, t_dst)

    def stepk():
        seg.watershed_colorize_batch_dev(b_img, b_m, b_lab, depth, None, b_dst)

    step = step1 if K == 1 else stepk
    NC = args.pipeline == "nc"
    if NC:
        if K > 1:
            raise SystemExit("--pipeline nc runs one frame per step")
        nc_opts = [o for o in args.nc_options.split(",") if o]
        nc_flags = sum({"GISTO_DIAP": 1, "MULTI_OTSU": 2}[o] for o in nc_opts)
        t_gray = torch.empty((S, S), dtype=torch.uint8, device=dev)
        nc_levels = []

        def step1():  # noqa: F811
            lv = seg.nc_marker_stage_dev(t_img, args.nc_depth, t_lab, nc_flags, gray=t_gray)
            nc_levels[:] = lv
            seg.watershed_colorize_dev(t_img, t_lab, t_lab, len(lv), None, t_dst)

        step = step1
    SHAPE = args.pipeline == "shape"
    if SHAPE:
        if K > 1:
            raise SystemExit("--pipeline shape runs one frame per step")
        shape_depth = []

        def step1():  # noqa: F811
            d, _ = seg.shape_markers_dev(t_img, t_lab)
            shape_depth[:] = [d]
            seg.watershed_colorize_dev(t_img, t_lab, t_lab, d, None, t_dst)

        step = step1
    COLOR = args.pipeline == "color"
    if COLOR:
        if K > 1:
            raise SystemExit("--pipeline color runs one frame per step")
        color_depth = []
        t_sharp = torch.empty_like(t_img)

        def step1():  # noqa: F811
            d = seg.color_markers_dev(t_img, t_sharp, t_lab)
            color_depth[:] = [d]
            seg.watershed_colorize_dev(t_sharp, t_lab, t_lab, d, None, t_dst)

        step = step1
    MARKERS = NC or SHAPE or COLOR  # a marker stage before the flood: the pipeline's digest, no side lines
    pipe_key = None
    if NC:
        pipe_key = "nc_%s_%dx%d_s%d_d%d_%s" % (args.kind, S, S, seed, args.nc_depth, "+".join(nc_opts) or "none")
    elif SHAPE or COLOR:
        pipe_key = "%s_%s_%dx%d_s%d" % (args.pipeline, args.kind, S, S, seed)

    # one step for the parity check, then the warm-up steps right before the timed ones (the check's
    # host work -- a 64 MB read-back and its hash -- used to sit between warm-up and timing, leaving
    # the GPU idle for ~80 ms just before the first timed step)
    step()
    sync()
    parity = None
    dgs = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    dkey = "%s_%dx%d_s%d" % (args.kind, S, S, seed)
    if MARKERS and dgs.get(pipe_key):
        # the marker-stage pipeline's frame against the oracle digest of the whole pipeline
        # (tests/golden/make_golden.py --pipelines: numpy marker stage + the C flood)
        got = hashlib.sha256(t_lab.cpu().numpy().tobytes()).hexdigest()
        parity = ("bit-exact vs oracle digest" if got == dgs[pipe_key]["labels_sha256"]
                  else "MISMATCH vs oracle digest") + " " + pipe_key
    if not MARKERS:
        # every rank: each of its K label maps against its committed oracle digest, summed over ranks
        keys = ["%s_%dx%d_s%d" % (args.kind, S, S, seed + k) for k in range(K)]
        labs_now = [t_lab.cpu().numpy()] if K == 1 else [x.cpu().numpy() for x in b_lab]
        checked, bad = reduce_sum_ints(digest_parity(labs_now, keys, dgs), cdev)
        del labs_now
        if K == 1 and world == 1:
            if checked:
                parity = ("bit-exact vs oracle digest" if not bad else "MISMATCH vs oracle digest") + " " + dkey
        elif checked:
            parity = "%d/%d frames bit-exact vs oracle digests (%s frames %d..%d over %d rank%s)" % (
                checked - bad, checked, args.kind, frame_seed(args.seed, 0, world, K, S),
                frame_seed(args.seed, world - 1, world, K, S) + K - 1, world, "s" if world > 1 else "")
        if rank == 0:
            log("[rank 0] parity:", parity)

    for _ in range(args.warmup):
        step()
    sync()
    st = seg.stats()
    dt = timed_steps(step, args.steps, barrier, sync)
    dt_max = reduce_max(dt, cdev)
    value = whole_job_mpx(world, K * S * S, args.steps, dt_max)
    ms_per_step = 1000.0 * dt_max / args.steps
    log("[rank %d] %.3f ms/step (max over ranks %.3f)" % (rank, 1000 * dt / args.steps, ms_per_step))

    kern = None
    if not args.no_profile_pass:
        seg.set_profiling(True)
        seg.kernel_profile(reset=True)
        for _ in range(args.steps):
            step1()  # the kernels of one flood (batch sub-contexts are not instrumented)
        sync()
        prof = seg.kernel_profile(reset=True)
        seg.set_profiling(False)
        kern = kernel_roofline(prof, st if K == 1 else seg.stats(), S * S, args.steps)

    stencil = None
    if not MARKERS and K == 1:
        stencil = colour_distance(seg, t_img, img, S, sync, pmc_cfg, check=(rank == 0))

    batch = None
    if K == 1 and not MARKERS and args.batch_frames > 1:
        bseed = 100 + rank * args.batch_frames
        batch = batch_throughput(seg, args, S, bseed, sync)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            batch["cpu_baseline"] = cpu_baseline_batch(args.kind, S, bseed, args.batch_frames)
        if rank == 0 and world == 1 and not args.no_hwq4:
            batch["hwq4"] = batch_hwq4(args, S, bseed)

    many = None
    if rank == 0 and world == 1 and K == 1 and not MARKERS and args.kind == "mosaic" and args.many_frames > 0:
        many = many_floods_line(seg, sync, dev, args.many_frames, cpu=not args.no_cpu_baseline)

    corr = None
    if rank == 0 and world == 1 and K == 1 and not MARKERS and args.kind == "mosaic" and args.correlation:
        corr = {}
        for name in args.correlation.split(","):
            corr[name] = correlation_line(seg, sync, dev, name, cpu=not args.no_cpu_baseline)
        if args.correlation_images > 0:
            corr["mass"] = correlation_mass_line(seg, sync, dev, images=args.correlation_images,
                                                 cpu=not args.no_cpu_baseline)

    stress = stress_random = None
    if rank == 0 and world == 1 and K == 1 and not MARKERS and args.kind == "mosaic" and args.stress_steps > 0:
        stress = stress_line(seg, S, sync, dev, args.stress_steps, cpu=not args.no_cpu_baseline)
        # the uniform-random variant (config 3's worst case), fewer steps
        stress_random = stress_line(seg, S, sync, dev, max(1, args.stress_steps // 2),
                                    cpu=not args.no_cpu_baseline, kind="random")

    pcie = None
    if rank == 0 and world == 1 and not MARKERS:
        # host-buffer entry point (what the JNI shim calls): H2D + flood + colourise + D2H
        reps, t_host = 3, 0.0
        for _ in range(reps):
            work = m.copy()
            t1 = time.perf_counter()
            seg.watershed_colorize(img, work, depth, None)
            t_host += time.perf_counter() - t1
        pcie = {"value": round(S * S * reps / t_host / 1e6, 3), "unit": "Mpx/s",
                "note": "msg_watershed_colorize on pageable host buffers, %d frames" % reps}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if SHAPE:
            cpu, cpu_lab = cpu_baseline_shape(img)
        elif COLOR:
            cpu, cpu_lab = cpu_baseline_color(img)
        elif NC:
            cpu, cpu_lab = cpu_baseline_nc(img, args.nc_depth, nc_opts)
        else:
            cpu, cpu_lab = cpu_baseline(img, m, depth)
        if parity is None and cpu_lab is not None:
            parity = "bit-exact vs oracle" if np.array_equal(cpu_lab, t_lab.cpu().numpy()) else "MISMATCH vs oracle"

    if world > 1:
        barrier()
    seg_blur_k = msegment._lib.load().msg_blur_mask_size(S, S) if SHAPE else None
    if rank == 0:
        roof = None
        if kern:
            top = kern[0]
            traffic, tsrc = pmc_traffic(top["kernel"], pmc_cfg)
            roof = {"bound": "hbm", "kernel": top["kernel"], "achieved": top["achieved_gbs"],
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(top["achieved_gbs"] / HBM_PEAK_GBS, 5) if top["achieved_gbs"] else None,
                    "traffic": traffic, "traffic_source": tsrc,
                    "alg_bytes_per_launch": top["alg_bytes_per_launch"], "avg_launch_us": top["avg_us"]}
        e2e_gbs = value * 1e6 * E2E_BYTES_PER_PIXEL / 1e9
        out = {
            "metric": (METRIC_SHAPE if SHAPE else METRIC_NC if NC else METRIC_COLOR if COLOR
                       else METRIC.format(S=S)), "value": round(value, 3), "unit": "Mpx/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (msegment.synth %s, splitmix64; regenerated on the box)" % args.kind,
            "config": {"workload": "%s %dx%d seed %s%s, %s + colorByIndexes(colored=false), "
                                   "device-resident (BASELINE config %s)"
                                   % (args.kind, S, S, seed if (world == 1 or args.seed is not None)
                                      else "100+%d*rank" % K,
                                      "" if K == 1 else "..+%d, %d floods in flight" % (K - 1, min(K, args.inflight)),
                                      ("notConnectedMarkers marker stage (depth %d, %s; %d levels) + watershed"
                                       % (args.nc_depth, "+".join(nc_opts) or "no options", len(nc_levels)))
                                      if NC else ("shapeAutoMarkerWatershed marker stage (median %d, depth %d) "
                                                  "+ watershed" % (seg_blur_k, shape_depth[0])) if SHAPE
                                      else ("colorAutoMarkerWatershed marker stage (depth %d) + watershed of "
                                            "the sharpened frame" % color_depth[0]) if COLOR
                                      else "watershed",
                                      ({1024: "2", 4096: "3", 16384: "4 frame on one GPU"}.get(
                                          S, "-: a %d-pixel frame" % (S * S)) if K == 1
                                       else "5 batching") if world == 1 else "5"),
                       "frames_per_rank_per_step": K, "parallelism": "replicas%d (no collectives)" % world,
                       **({"rehearsal": "MSEG_BENCH_SHARED_GPU: all %d ranks on GPU 0, gloo collectives "
                                        "(not a multi-GPU measurement)" % world} if shared else {})},
            "roofline": roof,
            "colour_distance": stencil,
            "batch": batch,
            "stress": stress,
            "stress_random": stress_random,
            "many_floods": many,
            "correlation": corr,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "e2e_hbm": {"achieved": round(e2e_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(e2e_gbs / HBM_PEAK_GBS, 5), "bytes_per_pixel": E2E_BYTES_PER_PIXEL},
            "flood": {"batches": st["batches"], "pops": st["pops"], "items": st["items"],
                      "pushes": st["pushes"], "host_syncs": st["host_syncs"]},
            "kernels": kern,
            "parity": parity,
            "build_id": msegment._lib.load().msg_build_id().decode(),
        }
        print(json.dumps(out), flush=True)
    seg.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
