"""Where the interrupt-dense regime's time goes, per input: the one-workgroup
loop's split (msg_set_diag 3: tiny batches / serial pops / small batches, counts and s_memtime
cycles) next to the flood's wall time without diagnostics and the C oracle's time on the same
frame.  Inputs: album.jpg with the shape method's seeds, the same with the colour method's seeds,
the notConnectedMarkers seeds of a 1024^2 noisy mosaic, mosaic+noise 1024^2, random 512^2.
usage: python scripts/regime_split.py [reps]"""
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


def cases(seg):
    rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
    album = np.ascontiguousarray(rgb[..., ::-1])
    out = [("album_shape_seeds", album, np.ascontiguousarray(seg.shape_markers(album)[0]))]
    sharp, mk, _ = seg.color_markers(album)
    out.append(("album_color_seeds", np.ascontiguousarray(sharp), np.ascontiguousarray(mk)))
    img = synth.frame("mosaic_noise", 1024, 1024, 2)[0]
    out.append(("nc_seeds_1024", img, np.ascontiguousarray(seg.nc_marker_stage(img, 4)[0])))
    for kind, S, seed in (("mosaic_noise", 1024, 1), ("random", 512, 3)):
        img, m, _ = synth.frame(kind, S, S, seed)
        out.append(("%s_%d" % (kind, S), img, m))
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    for name, img, m in cases(seg):
        t_img = torch.from_numpy(img).to(dev)
        t_m = torch.from_numpy(m).to(dev)
        t_lab = torch.empty_like(t_m)
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        want = ws_oracle.watershed(img, m)
        cpu_ms = 1e3 * (time.perf_counter() - c0)
        ok = np.array_equal(t_lab.cpu().numpy(), want)
        seg.set_serial_kernel(False)  # A/B: serial pops inside k_scan's loop (round 2's path)
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        ms_inloop = 1e3 * (time.perf_counter() - t0) / reps
        seg.set_serial_kernel(True)
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / reps
        st = seg.stats()
        seg.set_diag(3)
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        d = seg.stats()["diag"]
        seg.set_diag(False)
        tk = lambda c: c / 1e5  # noqa: E731  s_memrealtime: 100 MHz ticks -> ms
        print("%-18s %8.1f ms (serial pops in k_scan: %.1f ms) %s (C oracle 1 core %.1f ms) pops %d batches %d "
              "spec_gens %d" % (name, ms, ms_inloop, "bit-exact" if ok else "MISMATCH", cpu_ms, st["pops"],
                                st["batches"], st["spec_generations"]))
        print("    tiny batches %d (%d pops, %.1f ms)  serial pops %d (%.1f ms, %.3f us/pop; k_serial entries %d, "
              "line fills %.2f/pop)  small-batch pops %d" % (
                  d[0], d[1], tk(d[2]), d[3], tk(d[4]), 1e3 * tk(d[4]) / max(d[3], 1), d[5], d[6] / max(d[3], 1),
                  d[7]), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
