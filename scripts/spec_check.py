"""Speculative generations (csrc/spec_kernels.hip) against the C oracle on interrupt-dense frames,
with the engine's counters and the flood time with the engine on and off.
usage: python scripts/spec_check.py [quick]"""
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


def frames(quick):
    out = []
    for kind, S, seed in (("mosaic_noise", 64, 1), ("random", 64, 2), ("mosaic_noise", 256, 1),
                          ("random", 128, 3), ("mosaic_noise", 1024, 1), ("random", 512, 3)):
        img, m, _ = synth.frame(kind, S, S, seed)
        out.append(("%s_%d_s%d" % (kind, S, seed), img, m))
    if not quick:
        rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
        album = np.ascontiguousarray(rgb[..., ::-1])
        out.append(("album_crop_400", np.ascontiguousarray(album[300:700, 500:900]), None))
        out.append(("album_shape_seeds", album, None))
    return out


def named(names):
    """kind_S_sSEED frames; an "nc_" prefix replaces the seeds by the NC pipeline's marker map
    (depth 4, GISTO_DIAP: every pixel whose gray is a level's mean band is a seed)."""
    out = []
    for nm in names:
        nc = nm.startswith("nc_")
        kind, S, seed = (nm[3:] if nc else nm).rsplit("_", 2)
        img, m, _ = synth.frame(kind, int(S), int(S), int(seed[1:]))
        if nc:
            from oracle import nc_oracle
            m = np.ascontiguousarray(nc_oracle.marker_stage(img, 4, gisto_diap=True)[3])
        out.append((nm, img, m))
    return out


def main():
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    prof = "prof" in sys.argv
    sel = [a for a in sys.argv[1:] if a not in ("quick", "prof", "album")]
    if "album" in sys.argv:
        sel = None
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    bad = 0
    todo = named(sel) if sel else frames(quick)
    if sel is None:
        todo = [f for f in frames(False) if f[0].startswith("album")]
    for name, img, m in todo:
        if m is None:
            m = np.ascontiguousarray(seg.shape_markers(img)[0])
        want = ws_oracle.watershed(img, m)
        t_img = torch.from_numpy(img).to(dev)
        t_m = torch.from_numpy(m).to(dev)
        t_lab = torch.empty_like(t_m)
        line = "%-22s" % name
        for on in (True, False):
            seg.set_speculative(on)
            seg.watershed_dev(t_img, t_m, t_lab)
            torch.cuda.synchronize()
            ok = np.array_equal(t_lab.cpu().numpy(), want)
            bad += not ok
            if prof:
                seg.set_profiling(True)
                seg.kernel_profile(reset=True)
            t0 = time.perf_counter()
            seg.watershed_dev(t_img, t_m, t_lab)
            torch.cuda.synchronize()
            ms = 1e3 * (time.perf_counter() - t0)
            st = seg.stats()
            if prof:
                kp = seg.kernel_profile(reset=True)
                seg.set_profiling(False)
                print("   spec=%d kernels: %s" % (on, ", ".join("%s %d/%.1fms" % (k, v[0], v[1]) for k, v in kp.items() if v[0])), flush=True)
                print("   spec=%d stats: batches %d pops %d items %d host_syncs %d diag %s" % (
                    on, st["batches"], st["pops"], st["items"], st["host_syncs"], st["diag"]), flush=True)
            line += " | spec=%d %9.1f ms %8.2f Mpx/s %s" % (on, ms, img.shape[0] * img.shape[1] / ms / 1e3,
                                                             "exact" if ok else "MISMATCH")
            if on:
                line += " gens %d rounds %d execs %d cpops %d fb %d batches %d" % (
                    st["spec_generations"], st["spec_rounds"], st["spec_executions"],
                    st["spec_cascade_pops"], st["spec_fallbacks"], st["batches"])
        print(line, flush=True)
    seg.close()
    print("ALL EXACT" if bad == 0 else "%d MISMATCHES" % bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
