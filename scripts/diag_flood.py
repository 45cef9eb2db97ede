#!/usr/bin/env python3
"""Flood diagnostics on the GPU: per-kernel HIP-event profile + in-kernel cycle counters
(msg_set_diag) for one synthetic frame.  Not a benchmark (diagnostics add atomics)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opencv-msegment_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mosaic")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=2)
    args = ap.parse_args()
    import torch

    import msegment
    from msegment import synth

    img, m, depth = synth.frame(args.kind, args.size, args.size, args.seed)
    dev = torch.device("cuda", 0)
    t_img = torch.from_numpy(img).to(dev)
    t_m = torch.from_numpy(m).to(dev)
    t_lab = torch.empty_like(t_m)
    seg = msegment.Segmenter(0)
    seg.watershed_dev(t_img, t_m, t_lab)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seg.watershed_dev(t_img, t_m, t_lab)
    torch.cuda.synchronize()
    plain_ms = 1000 * (time.perf_counter() - t0)
    seg.set_diag(True)
    seg.set_profiling(True)
    seg.kernel_profile(reset=True)
    seg.watershed_dev(t_img, t_m, t_lab)
    torch.cuda.synchronize()
    prof = seg.kernel_profile(reset=True)
    st = seg.stats()
    d = st["diag"]
    out = {"kind": args.kind, "size": args.size, "plain_ms": round(plain_ms, 3), "stats": st,
           "profile": {k: (n, round(ms, 4)) for k, (n, ms) in prof.items() if n},
           "resolve": {"gather_cycles_per_wave_round": d[0] / max(d[4], 1),
                       "loop_cycles_per_wave_round": d[1] / max(d[4], 1),
                       "loop_rounds_per_wave_round": d[2] / max(d[4], 1),
                       "max_loop_cycles": d[3], "wave_rounds": d[4]},
           "small": {"loop_rounds": d[5], "launches_worked": d[6]}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
