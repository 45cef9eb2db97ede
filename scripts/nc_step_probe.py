"""Time the NC pipeline step by step on cuda:0 (diagnostic): marker stage, then the flood."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]
import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
kind = sys.argv[2] if len(sys.argv) > 2 else "mosaic_noise"
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 1
img, m, depth = synth.frame(kind, S, S, 2)
seg = msegment.Segmenter(0)
t_img = torch.from_numpy(img).cuda()
lab = torch.empty((S, S), dtype=torch.int32, device="cuda")
dst = torch.empty((S, S, 3), dtype=torch.uint8, device="cuda")
g = torch.empty((S, S), dtype=torch.uint8, device="cuda")
for it in range(4):
    t0 = time.perf_counter()
    lv = seg.nc_marker_stage_dev(t_img, 4, lab, flags, gray=g)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    nseed = int((lab > 0).sum().item())
    print("it %d stage %.1f us, %d levels, %d seed px" % (it, (t1 - t0) * 1e6, len(lv), nseed), flush=True)
    t1 = time.perf_counter()
    seg.watershed_colorize_dev(t_img, lab, lab, len(lv), None, dst)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    st = seg.stats()
    print("   flood %.1f ms  batches %d pops %d items %d pushes %d syncs %d" % (
        (t2 - t1) * 1e3, st["batches"], st["pops"], st["items"], st["pushes"], st["host_syncs"]), flush=True)
