"""Per-pop time split of the serial-pop regime (k_serial, csrc/ws_kernels.hip) on the inputs that
live in it: album.jpg with the shape method's seeds, the notConnectedMarkers seeds of a 1024^2
noisy mosaic, uniform-random 512^2.  Needs the diagnostic build (make -C opencv-msegment_amd/csrc
serprof): MSEGMENT_LIB=.../libmsegment_serprof.so python scripts/serial_phases.py
Phases (s_memtime shader cycles, summed over the pops): select = lowest bucket + queue slot,
load = the four neighbour states + weights and the label fold (one dependent round trip),
push = the label store and the pushes.  'wall' is the k_serial launches' s_memrealtime total."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402
from oracle import ws_oracle  # noqa: E402


def main():
    seg = msegment.Segmenter(0)
    seg.set_serial_kernel(True)
    rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
    album = np.ascontiguousarray(rgb[..., ::-1])
    cases = [("album_shape_seeds", album, np.ascontiguousarray(seg.shape_markers(album)[0]))]
    img = synth.frame("mosaic_noise", 1024, 1024, 2)[0]
    cases.append(("nc_seeds_1024", img, np.ascontiguousarray(seg.nc_marker_stage(img, 4)[0])))
    img, m, _ = synth.frame("random", 512, 512, 3)
    cases.append(("random_512", img, m))
    dev = torch.device("cuda", 0)
    for name, img, m in cases:
        t_img, t_m = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        t_lab = torch.empty_like(t_m)
        seg.set_diag(3)
        seg.watershed_dev(t_img, t_m, t_lab)
        torch.cuda.synchronize()
        d = seg.stats()["diag"]
        seg.set_diag(False)
        ok = np.array_equal(t_lab.cpu().numpy(), ws_oracle.watershed(img, m))
        n = max(d[3], 1)
        print("%-18s %s  serial pops %d in %d launches, wall %.1f ms = %.3f us/pop; per pop (cycles): select %.0f, "
              "load+fold %.0f, push %.0f, loop total %.0f" % (
                  name, "bit-exact" if ok else "MISMATCH", d[3], d[5], d[4] / 1e5, d[4] / 1e2 / n, d[0] / n, d[1] / n,
                  d[2] / n, d[6] / n), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
