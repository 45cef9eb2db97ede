"""Where a single flood's time goes by regime (msg_set_diag 3, bank 2): tiny batches (count, pops,
time), serial pops (count, time: k_scan's loop and k_serial_one), small-batch pops, speculative
generations.  Frames as in scripts/spec_probe.py, plus color_KIND_S_sSEED (the colour method's
sharpened frame and markers of a synthetic frame, the colour pipeline's flood).
usage: python scripts/regime_split.py [frame names]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd"), os.path.join(ROOT, "scripts")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msegment  # noqa: E402
import spec_probe  # noqa: E402
from msegment import synth  # noqa: E402


def load(seg, nm):
    if nm.startswith("color_"):
        kind, S, seed = nm[6:].rsplit("_", 2)
        img = synth.frame(kind, int(S), int(S), int(seed[1:]))[0]
        sharp, mk, _ = seg.color_markers(img)
        return np.ascontiguousarray(sharp), np.ascontiguousarray(mk)
    return spec_probe.load(seg, nm)


def main():
    names = sys.argv[1:] or ["album_shape", "nc_mosaic_noise_1024_s100"]
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    for nm in names:
        img, m = load(seg, nm)
        ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        tl = torch.empty_like(tm)
        seg.set_diag(0)
        ms = spec_probe.flood_ms(seg, ti, tm, tl)
        seg.set_diag(3)
        seg.watershed_dev(ti, tm, tl)
        torch.cuda.synchronize()
        st = seg.stats()
        d = st["diag"]
        seg.set_diag(0)
        print("%-26s %.1f ms (diag off) | tiny batches %d (%d pops, %.1f ms) | serial pops %d (%.1f ms) | "
              "small-batch pops %d | generation pops %d (%.1f ms) | total pops %d"
              % (nm, ms, d[0], d[1], d[2] / 1e5, d[3], d[4] / 1e5, d[7], st["spec_gen_pops"],
                 st["spec_gen_us"] / 1e3, st["pops"]), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
