"""The headline step (4096^2 mosaic, device-resident watershed + colorise) against the k_resolve
grid size (msg_set_resolve_grid; 0 = the default, one wave of the device's occupancy), interleaved
passes.  usage: python scripts/resolve_grid_probe.py [grid ...]  (default 0 640 512 384 256)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def main():
    S = 4096
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    img, m, depth = synth.frame("mosaic", S, S, 2)
    ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
    tl = torch.empty_like(tm)
    dst = torch.empty((S, S, 3), dtype=torch.uint8, device=dev)
    grids = [int(a) for a in sys.argv[1:]] or [0, 640, 512, 384, 256]
    for rep in range(2):
        for g in grids:
            seg.set_resolve_grid(g)
            for _ in range(3):
                seg.watershed_colorize_dev(ti, tm, tl, depth, None, dst)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                seg.watershed_colorize_dev(ti, tm, tl, depth, None, dst)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
            st = seg.stats()
            print("rep %d grid %4s: %.3f ms  %.0f Mpx/s  resolve items %d" % (rep, g or "dflt", dt * 1e3, S * S / dt / 1e6,
                                                                            st["resolve_items"]), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
