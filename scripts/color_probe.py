import sys, time
sys.path[:0] = ["/root/repo", "/root/repo/opencv-msegment_amd"]
import numpy as np, torch, msegment
from msegment import synth
from oracle import color_oracle as C
seg = msegment.Segmenter(0); dev = torch.device("cuda", 0)
for kind, S in (("mosaic", 1024), ("mosaic", 4096), ("mosaic_noise", 4096)):
    img = synth.frame(kind, S, S, 2)[0]
    ti = torch.from_numpy(img).to(dev); sh = torch.empty_like(ti); mk = torch.empty((S, S), dtype=torch.int32, device=dev)
    lab = torch.empty_like(mk); dst = torch.empty_like(ti)
    d = seg.color_markers_dev(ti, sh, mk); torch.cuda.synchronize()
    t0 = time.perf_counter(); reps = 3
    for _ in range(reps): d = seg.color_markers_dev(ti, sh, mk)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    for _ in range(reps): seg.watershed_colorize_dev(sh, mk, lab, d, None, dst)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    ok = ""
    if S <= 1024:
        w = C.stages(img); ok = "exact" if np.array_equal(mk.cpu().numpy(), w["markers"]) else "MISMATCH"
    print("%s %d: marker stage %.2f ms, flood+colour %.2f ms, depth %d %s" % (kind, S, (t1-t0)/reps*1e3, (t2-t1)/reps*1e3, d, ok), flush=True)
