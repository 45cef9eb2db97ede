"""Config 5 per GPU (8 mosaic 4096^2 frames per call) against the k_resolve grid size, the commit
grid's share (MSEG_BATCH_COMMIT_SUBS; default: 1/k of the chip) and the number of floods in flight:
does a smaller per-flood grid let concurrent floods share the chip?
usage: python scripts/batch_grid_probe.py [commit_subs,...]   (0 = the default share)"""
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
    csubs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0]
    for cs in csubs:
        if cs:
            os.environ["MSEG_BATCH_COMMIT_SUBS"] = str(cs)
        else:
            os.environ.pop("MSEG_BATCH_COMMIT_SUBS", None)
        for grid in (0, 384, 256, 128):
            for inflight in (4, 8):
                seg.set_resolve_grid(grid)
                seg.set_batch_inflight(inflight)
                seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(3):
                    seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / 3
                print("commit subs %4s  resolve grid %4s  in flight %d: %7.0f Mpx/s"
                      % (cs or "dflt", grid or "dflt", inflight, K * S * S / dt / 1e6), flush=True)


if __name__ == "__main__":
    main()
