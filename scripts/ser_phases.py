"""Where a serial pop's cycles go (the -DMSEG_SER_PROF diagnostic build, msg_set_diag 4): s_memtime
stamps around serial_loop_lanes' load (address + neighbour states + weights), fold, push (slots,
LDS tails, stores) and the loop between pops, summed over wave 0's pops in k_scan.  The stamps
themselves cost cycles (each waits for its scalar counter read), so the split is a proportion.
usage: MSEGMENT_LIB=.../libmsegment_serprof.so python scripts/ser_phases.py [frame names]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import msegment  # noqa: E402
from spec_probe import load  # noqa: E402


def main():
    names = sys.argv[1:] or ["nc_mosaic_noise_1024_s100", "album_shape"]
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    for nm in names:
        img, m = load(seg, nm)
        ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        tl = torch.empty_like(tm)
        seg.watershed_dev(ti, tm, tl)
        seg.set_diag(4)
        seg.watershed_dev(ti, tm, tl)
        torch.cuda.synchronize()
        d = seg.stats()["diag"]
        seg.set_diag(False)
        pops = max(1, d[5])
        print("%-26s serial pops %d | cycles per pop: load %.0f fold %.0f push %.0f between %.0f | pushes/pop %.2f"
              " | of 'between': ring refills %.0f, empty-bucket scans %.0f"
              % (nm, d[5], d[0] / pops, d[1] / pops, d[2] / pops, d[3] / pops, d[4] / pops, d[6] / pops,
                 d[7] / pops), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
