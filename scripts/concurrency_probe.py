#!/usr/bin/env python3
"""Do independent floods overlap on one GPU?  K contexts, each on its own stream, each flooding
its own 4096^2 mosaic; reports aggregate Mpx/s for K = 1, 2, 4 (tuning aid, not a benchmark)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opencv-msegment_amd"))


def main():
    import torch

    import msegment
    from msegment import synth

    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda", 0)
    frames = []
    for k in range(4):
        img, m, depth = synth.frame("mosaic", S, S, 100 + k)
        frames.append((torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev), depth))
    segs = [msegment.Segmenter(0) for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in range(4)]
    labs = [torch.empty_like(f[1]) for f in frames]
    dsts = [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in frames]
    import threading

    def run(k, reps):
        with torch.cuda.stream(streams[k]):
            for _ in range(reps):
                segs[k].watershed_colorize_dev(frames[k][0], frames[k][1], labs[k], frames[k][2], None, dsts[k],
                                               stream=streams[k].cuda_stream)

    for K in (1, 2, 4):  # one host thread per context (the API's model), each on its own stream
        for k in range(K):
            run(k, 1)
        torch.cuda.synchronize()
        reps = 10
        th = [threading.Thread(target=run, args=(k, reps)) for k in range(K)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print("K=%d aggregate %.1f Mpx/s" % (K, K * S * S * reps / dt / 1e6), flush=True)


if __name__ == "__main__":
    main()
