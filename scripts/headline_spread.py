"""Run-to-run spread of the headline step (config 3: mosaic 4096^2 seed 2, watershed + colorize,
device-resident): BLOCKS blocks of STEPS timed steps in ONE process, a context per block or one for
all, printing ms per frame per block -- to tell a per-process state (workspace placement) from a
per-period one (clocks).  usage: python scripts/headline_spread.py [blocks] [steps] [fresh]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402

blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 4
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
fresh = len(sys.argv) > 3 and sys.argv[3] == "fresh"
dev = torch.device("cuda", 0)
img, m, depth = synth.frame("mosaic", 4096, 4096, 2)
ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
tl = torch.empty_like(tm)
td = torch.empty((4096, 4096, 3), dtype=torch.uint8, device=dev)
seg = msegment.Segmenter(0)
out = []
for b in range(blocks):
    if fresh and b:
        seg.close()
        seg = msegment.Segmenter(0)
    for _ in range(3):
        seg.watershed_colorize_dev(ti, tm, tl, depth, None, td)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        seg.watershed_colorize_dev(ti, tm, tl, depth, None, td)
    torch.cuda.synchronize()
    out.append(1e3 * (time.perf_counter() - t0) / steps)
    time.sleep(0.2)
print("pid %d %s: %s ms per frame" % (os.getpid(), "fresh contexts" if fresh else "one context",
                                     " ".join("%.3f" % x for x in out)), flush=True)
seg.close()
