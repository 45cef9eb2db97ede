"""Phase split of k_commit_fast (the two-launch iterations' commit, csrc/ws_kernels.hip) on the
headline frame.  Needs the diagnostic build (make -C opencv-msegment_amd/csrc cfprof):
MSEGMENT_LIB=.../libmsegment_cfprof.so python scripts/cf_phases.py
The finalizer block's thread 0 stamps s_memrealtime (100 MHz) after the batch header, the queue
state, the histogram rows, the segments + next batch, the wait for every sub-round block's
arrival and the queue-state writes; sub-round block 0 stamps its arrival.  Averages per committed
launch, in microseconds from each block's own first instruction."""
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
    img, m, depth = synth.frame("mosaic", S, S, 2)
    t_img, t_m = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
    t_lab = torch.empty_like(t_m)
    seg.watershed_dev(t_img, t_m, t_lab)  # warm-up (workspace, code objects)
    seg.set_diag(1)
    for rep in range(3):
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        d = seg.stats()["diag"]
        n = max(1, d[7])
        us = [x / n / 100.0 for x in d]
        print("rep %d: %d committed launches; finalizer: header %.2f, queue state %.2f, rows %.2f, "
              "segments + next batch %.2f, arrivals %.2f, writes %.2f (sum %.2f us); sub-round block 0 "
              "arrives at %.2f us" % (rep, d[7], us[0], us[1], us[2], us[3], us[4], us[5], sum(us[:6]), us[6]),
              flush=True)


if __name__ == "__main__":
    main()
