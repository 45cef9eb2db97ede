"""Config-5-style stress: K device frames per step (msg_watershed_colorize_batch_dev) with up to
`inflight` floods in flight; counts steps that raise and frames whose labels differ from the
same frames flooded one at a time (inflight 1); exit 1 if any.  usage: python scripts/stress_inflight_dev.py [steps] [K] [inflight] [size] [speculative 0/1]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("STRESS_PKG") or os.path.join(ROOT, "opencv-msegment_amd")]
import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    inflight = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    dev = torch.device("cuda", 0)
    fr = [synth.frame("mosaic", S, S, 2 + k) for k in range(K)]
    depth = max(f[2] for f in fr)
    imgs = [torch.from_numpy(f[0]).to(dev) for f in fr]
    mks = [torch.from_numpy(f[1]).to(dev) for f in fr]
    labs = [torch.empty_like(m) for m in mks]
    dsts = [torch.empty((S, S, 3), dtype=torch.uint8, device=dev) for _ in fr]
    seg = msegment.Segmenter(0)
    if len(sys.argv) > 5:
        seg.set_speculative(bool(int(sys.argv[5])))
    if os.environ.get("STRESS_DIAG"):
        seg.set_diag(True)
    seg.set_batch_inflight(1)  # reference labels: one flood at a time on the context itself
    seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
    torch.cuda.synchronize()
    ref = [x.clone() for x in labs]
    seg.set_batch_inflight(inflight)
    errs = bad = 0
    for s in range(steps):
        try:
            seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            errs += 1
            print("step %d: %s" % (s, e), flush=True)
            continue
        for k in range(K):
            if not torch.equal(ref[k], labs[k]):
                bad += 1
                d = (ref[k] != labs[k]).nonzero()
                info = ", ".join("(%d,%d) ref %d got %d" % (int(y), int(x), int(ref[k][y, x]), int(labs[k][y, x]))
                                 for y, x in d[:4].tolist())
                print("step %d frame %d differs in %d px: %s" % (s, k, d.shape[0], info), flush=True)
    print("K %d inflight %d size %d: %d error steps, %d bad frames in %d steps" % (K, inflight, S, errs, bad, steps),
          flush=True)
    seg.close()
    return 1 if errs or bad else 0


if __name__ == "__main__":
    sys.exit(main())
