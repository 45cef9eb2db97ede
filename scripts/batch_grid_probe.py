"""Config 5 per GPU (8 mosaic 4096^2 frames per call) against the k_resolve grid size and the number
of floods in flight: does a smaller per-flood grid let concurrent floods share the chip?
(Round 4 also swept the commit grid's share through an environment knob, since removed.)
usage: python scripts/batch_grid_probe.py [grids (0 = default) [floods in flight]], e.g. "0,384,256" "4,8"."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def main():
    S, K = 4096, 8
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    frames = [synth.frame("mosaic", S, S, 100 + k) for k in range(K)]
    imgs = [torch.from_numpy(f[0]).to(dev) for f in frames]
    mks = [torch.from_numpy(f[1]).to(dev) for f in frames]
    labs = [torch.empty_like(m) for m in mks]
    dsts = [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in frames]
    depth = max(f[2] for f in frames)
    grids = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 384, 256, 128]
    flights = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4, 8]
    for grid in grids:
        for inflight in flights:
            seg.set_resolve_grid(grid)
            seg.set_batch_inflight(inflight)
            seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            print("resolve grid %4s  in flight %d: %7.0f Mpx/s" % (grid or "dflt", inflight, K * S * S / dt / 1e6),
                  flush=True)


if __name__ == "__main__":
    main()
