"""Flood time in the interrupt-dense regimes, device-resident, one frame
each: the reference's album.jpg (1500^2) with the shape method's seeds (built by the library's
own marker stage), mosaic+noise 1024^2, uniform-random 512^2.  Labels are checked against the C
oracle.  MSEGMENT_LIB selects an alternative library build (A/B).
usage: python scripts/regime_probe.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402
from oracle import ws_oracle  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
    album = np.ascontiguousarray(rgb[..., ::-1])
    album_mk = np.ascontiguousarray(seg.shape_markers(album)[0])
    cases = [("album_shape_seeds", album, album_mk)]
    for kind, S, seed in (("mosaic_noise", 1024, 1), ("random", 512, 3)):
        img, m, _ = synth.frame(kind, S, S, seed)
        cases.append(("%s_%d" % (kind, S), img, m))
    for name, img, m in cases:
        t_img = torch.from_numpy(img).to(dev)
        t_m = torch.from_numpy(m).to(dev)
        t_lab = torch.empty_like(t_m)
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        want = ws_oracle.watershed(img, m)
        cpu_ms = 1e3 * (time.perf_counter() - c0)
        ok = np.array_equal(t_lab.cpu().numpy(), want)
        t0 = time.perf_counter()
        for _ in range(reps):
            seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / reps
        st = seg.stats()
        print("%-20s %8.1f ms  %7.2f Mpx/s  batches %d  %s  (C oracle, 1 core: %.1f ms)"
              % (name, ms, img.shape[0] * img.shape[1] / ms / 1e3, st["batches"],
                 "bit-exact" if ok else "MISMATCH", cpu_ms), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
