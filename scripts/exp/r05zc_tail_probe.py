import os, sys
ROOT = "/root/repo" if os.path.isdir("/root/repo") else os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]
import torch, msegment
from msegment import synth
img, m, d = synth.frame("mosaic", 4096, 4096, 2)
dev = torch.device("cuda", 0)
ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
tl = torch.empty_like(tm)
seg = msegment.Segmenter(0)
seg.watershed_dev(ti, tm, tl); torch.cuda.synchronize()
seg.set_diag(3)
seg.watershed_dev(ti, tm, tl); torch.cuda.synchronize()
st = seg.stats()
print("diag bank 3 (tiny batches, their pops, their time 10ns, serial pops, serial time, -, -, small-batch pops):", st["diag"])
print({k: st[k] for k in ("batches", "pops", "items", "pushes", "host_syncs", "fast_pops", "scatter_pops", "resolve_items")})
seg.close()
