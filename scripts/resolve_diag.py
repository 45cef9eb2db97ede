"""k_resolve's own split on the headline frame (msg_set_diag 1, csrc/ws_kernels.hip): per wave
of a block-round, the gather (queue slot, neighbour states, competitors: dependent round trips)
and the decision loop (waits on lower ranks' granules), in s_memtime shader cycles.
usage: python scripts/resolve_diag.py [size]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    img, m, _ = synth.frame("mosaic", S, S, 2)
    t_img, t_m = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
    t_lab = torch.empty_like(t_m)
    seg.watershed_dev(t_img, t_m, t_lab)
    seg.set_diag(1)
    for rep in range(2):
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        d = seg.stats()["diag"]
        w = max(1, d[4])
        print("rep %d: %d wave-chunks; per wave: gather %.0f cycles, decision loop %.0f cycles (%.2f passes), "
              "longest loop %d cycles" % (rep, d[4], d[0] / w, d[1] / w, d[2] / w, d[3]), flush=True)


if __name__ == "__main__":
    main()
