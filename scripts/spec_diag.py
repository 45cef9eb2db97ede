import os, sys, time
sys.path[:0] = ["/root/repo", "/root/repo/opencv-msegment_amd"]
import numpy as np, torch, msegment
from msegment import synth
seg = msegment.Segmenter(0); dev = torch.device("cuda", 0)
for nm in sys.argv[1:]:
    kind, S, seed = nm.rsplit("_", 2); S = int(S)
    img, m, _ = synth.frame(kind, S, S, int(seed[1:]))
    ti = torch.from_numpy(img).to(dev); tm = torch.from_numpy(m).to(dev); tl = torch.empty_like(tm)
    seg.watershed_dev(ti, tm, tl); torch.cuda.synchronize()
    seg.set_diag(True)
    seg.watershed_dev(ti, tm, tl); torch.cuda.synchronize()
    st = seg.stats(); d = st["diag"]; seg.set_diag(False)
    r = max(1, st["spec_rounds"])
    o = d[5] - d[4] - d[6] - d[0] - d[1]
    print(nm, "rounds", r, "waves", d[7], "kern/wave us %.2f | max wave us %.1f | sum of the rounds' longest waves ms %.1f:"
          " cooperative cascades %.1f, top-pop gather %.1f, top-pop waits %.1f, top-pop writes + cascades %.1f,"
          " log copy + change marks %.1f" % (
        d[2]/1e2/max(1,d[7]), d[3]/1e2, d[5]/1e5, d[0]/1e5, o/1e5, d[4]/1e5, d[6]/1e5, d[1]/1e5), flush=True)
