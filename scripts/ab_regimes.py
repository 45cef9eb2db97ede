"""A/B of library builds (MSEGMENT_LIB, one child process per build) on the interrupt-dense
frames: uniform-random 512^2..4096^2 (BASELINE config 3's random stress variant at 4096^2),
mosaic+noise, album.jpg with the shape method's seeds, the notConnectedMarkers seeds of a 1024^2
noisy mosaic.  Each frame: one warm-up flood, then the median of 2 event-timed floods, the labels
checked against the C oracle (or the committed digest at 4096^2).
usage: python scripts/ab_regimes.py <lib.so> [<lib.so> ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, os, json, hashlib, statistics
sys.path[:0] = [%r, %r]
import numpy as np, torch, msegment
from PIL import Image
from msegment import synth
from oracle import ws_oracle
ROOT = %r
dig = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
seg = msegment.Segmenter(0)
dev = torch.device("cuda", 0)
cases = []
for kind, S, seed in (("random", 512, 3), ("random", 1024, 3), ("random", 2048, 3), ("random", 4096, 2),
                      ("mosaic_noise", 1024, 1), ("mosaic_noise", 4096, 2)):
    cases.append(("%%s_%%d" %% (kind, S), kind, S, seed))
cases.append(("album_shape_seeds", None, 0, 0))
cases.append(("nc_seeds_1024", None, 0, 0))
only = os.environ.get("AB_ONLY")
for name, kind, S, seed in cases:
    if only and name not in only.split(","):
        continue
    if kind:
        img, m, _ = synth.frame(kind, S, S, seed)
    elif name.startswith("album"):
        rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
        img = np.ascontiguousarray(rgb[..., ::-1]); m = np.ascontiguousarray(seg.shape_markers(img)[0])
    else:
        img = synth.frame("mosaic_noise", 1024, 1024, 2)[0]; m = np.ascontiguousarray(seg.nc_marker_stage(img, 4)[0])
    ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
    tl = torch.empty_like(tm)
    seg.watershed_dev(ti, tm, tl); torch.cuda.synchronize()
    ts = []
    for _ in range(2):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(); seg.watershed_dev(ti, tm, tl); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    st = seg.stats()
    lab = tl.cpu().numpy()
    key = "%%s_%%dx%%d_s%%d" %% (kind, S, S, seed) if kind else None
    if key in dig:
        ok = hashlib.sha256(np.ascontiguousarray(lab).tobytes()).hexdigest() == dig[key]["labels_sha256"]
    else:
        ok = np.array_equal(lab, ws_oracle.watershed(img, m))
    print("%%-18s %%9.1f ms  %%s  gens %%d rounds %%d execs %%d fallbacks %%d pops %%d batches %%d | cooldowns %%d "
          "gen pops %%d in %%.1f ms (%%.3f us/pop)" %% (
        name, statistics.median(ts), "exact" if ok else "MISMATCH", st["spec_generations"], st["spec_rounds"],
        st["spec_executions"], st["spec_fallbacks"], st["pops"], st["batches"], st["spec_cooldowns"],
        st["spec_gen_pops"], st["spec_gen_us"] / 1e3, st["spec_gen_us"] / max(1, st["spec_gen_pops"])), flush=True)
seg.close()
'''


def main():
    libs = sys.argv[1:]
    code = CHILD % (ROOT, os.path.join(ROOT, "opencv-msegment_amd"), ROOT)
    for lib in libs:
        print("== %s" % os.path.basename(lib), flush=True)
        env = dict(os.environ, MSEGMENT_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
        print(out.stdout, end="", flush=True)
        if out.returncode != 0:
            print("FAILED rc=%d %s" % (out.returncode, out.stderr[-500:]), flush=True)
            sys.exit(out.returncode)


if __name__ == "__main__":
    main()
