"""A/B flood timing of library builds on one box: each build in its own process (MSEGMENT_LIB),
alternating, the same frame, event-timed floods after a warm-up.
usage: python scripts/ab_flood.py <frame e.g. mosaic_noise_4096_s2> <reps> <lib.so> [<lib.so> ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, statistics
sys.path[:0] = [%r, %r]
import torch, msegment
from msegment import synth
kind, S, seed = %r.rsplit("_", 2)
S = int(S)
img, m, _ = synth.frame(kind, S, S, int(seed[1:]))
dev = torch.device("cuda", 0)
ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
tl = torch.empty_like(tm)
seg = msegment.Segmenter(0)
seg.watershed_dev(ti, tm, tl); torch.cuda.synchronize()
ts = []
for _ in range(3):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(); seg.watershed_dev(ti, tm, tl); b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
st = seg.stats()
print("%%.1f ms (min %%.1f) rounds %%d execs %%d" %% (statistics.median(ts), min(ts), st["spec_rounds"], st["spec_executions"]), flush=True)
seg.close()
'''


def main():
    frame, reps, libs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    code = CHILD % (ROOT, os.path.join(ROOT, "opencv-msegment_amd"), frame)
    for r in range(reps):
        for lib in libs:
            env = dict(os.environ, MSEGMENT_LIB=os.path.abspath(lib))
            out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
            line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else "FAILED rc=%d %s" % (out.returncode, out.stderr[-300:])
            print("rep %d %s: %s" % (r, os.path.basename(lib), line), flush=True)
            if out.returncode != 0:
                sys.exit(out.returncode)


if __name__ == "__main__":
    main()
