"""Repeat the concurrent host-buffer batch (several floods in flight, one host thread each) and
count frames that differ from the oracle.  usage: python scripts/stress_batch.py [reps] [inflight]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402

if os.environ.get("STRESS_TORCH"):  # the pytest session's state: torch's HIP runtime, a busy stream
    import torch  # noqa: F401

import msegment  # noqa: E402
from msegment import synth  # noqa: E402
from oracle import ws_oracle  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    inflight = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rng = np.random.default_rng(1)
    sets = []
    for v in range(6):  # frame sets of different sizes: sub-context buffers get reallocated
        fr = [synth.frame(("mosaic", "mosaic_noise", "random")[(k + v) % 3], 40 + int(rng.integers(0, 200)),
                          40 + int(rng.integers(0, 200)), 300 + 10 * v + k)[:2] for k in range(7)]
        sets.append((fr, [ws_oracle.watershed(img, m) for img, m in fr]))
    seg = msegment.Segmenter(0)
    if os.environ.get("STRESS_TORCH"):
        x = torch.randn(4096, 4096, device="cuda:0")
        for _ in range(3):
            x = x @ x
        torch.cuda.synchronize()
    exact = os.environ.get("STRESS_EXACT")
    if exact:  # tests/test_gpu_parity.py::test_batch_api_inflight's frames
        fr = [synth.frame(("mosaic", "mosaic_noise")[k % 2], 60 + 17 * k, 90 + 5 * k, 200 + k)[:2] for k in range(7)]
        sets = [(fr, [ws_oracle.watershed(img, m) for img, m in fr])]
    bad = 0
    t0 = time.time()
    for r in range(reps):
        frames, want = sets[r % len(sets)]
        seg.set_batch_inflight(inflight if inflight > 0 else int(rng.integers(1, 9)))
        work = [(img, m.copy()) for img, m in frames]
        try:
            seg.watershed_batch(work)
        except Exception as e:  # noqa: BLE001
            print("rep %d: error %s" % (r, e), flush=True)
            bad += 1
            continue
        for k, (w, (_, out)) in enumerate(zip(want, work)):
            if not np.array_equal(out, w):
                bad += 1
                print("rep %d frame %d: %d px differ, out min/max %d/%d" % (r, k, int((out != w).sum()),
                                                                          out.min(), out.max()), flush=True)
    print("inflight %d: %d bad frames in %d reps (%.1f s)" % (inflight, bad, reps, time.time() - t0), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
