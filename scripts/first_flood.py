"""First flood of a fresh context against the next ones (the speculative engine's workspace is
allocated on the first entry into the serial regime).  usage: python scripts/first_flood.py NAME..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for nm in sys.argv[1:]:
        kind, S, seed = nm.rsplit("_", 2)
        img, m, _ = synth.frame(kind, int(S), int(S), int(seed[1:]))
        ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        tl = torch.empty_like(tm)
        seg = msegment.Segmenter(0)
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            seg.watershed_dev(ti, tm, tl)
            torch.cuda.synchronize()
            st = seg.stats()
            print("%-22s flood %d: %8.1f ms  batches %d  gens %d  cools %d" % (
                nm, rep, 1e3 * (time.perf_counter() - t0), st["batches"], st["spec_generations"],
                st["spec_cooldowns"]), flush=True)
        seg.close()


if __name__ == "__main__":
    main()
