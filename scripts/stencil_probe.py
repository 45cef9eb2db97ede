"""Colour-distance stencil (msg_edge_weights_dev) at several frame sizes: HIP-event-timed
launches -> algorithmic GB/s (5 B/px).  Run under `rocprofv3 --kernel-trace --stats` to compare
with the profiler's kernel durations.  usage: python scripts/stencil_probe.py [sizes...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opencv-msegment_amd"))

import torch  # noqa: E402

import msegment  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [4096, 8192, 16384]
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    for S in sizes:
        img = torch.randint(0, 256, (S, S, 3), dtype=torch.uint8, device=dev)
        wr = torch.empty((S, S), dtype=torch.uint8, device=dev)
        wd = torch.empty_like(wr)
        for _ in range(3):
            seg.edge_weights_dev(img, wr, wd)
        torch.cuda.synchronize()
        seg.set_profiling(True)
        seg.kernel_profile(reset=True)
        reps = 20
        for _ in range(reps):
            seg.edge_weights_dev(img, wr, wd)
        torch.cuda.synchronize()
        n, ms = seg.kernel_profile(reset=True)["k_edge_weights"]
        seg.set_profiling(False)
        us = 1000.0 * ms / n
        print("%5d^2: %8.2f us/launch  %7.1f GB/s algorithmic (5 B/px)" % (S, us, 5.0 * S * S / us / 1e3), flush=True)
        del img, wr, wd
    seg.close()


if __name__ == "__main__":
    main()
