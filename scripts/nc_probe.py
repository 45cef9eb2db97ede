"""Time the NOT_CONNECTED_MARKERS marker stage kernels (k_gray_hist, k_nc_markers) on cuda:0
with the library's HIP-event profiling: per-kernel average and algorithmic GB/s
(k_gray_hist 3 B in + 1 B out per pixel, k_nc_markers 1 B in + 4 B out)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402

BYTES = {"k_gray_hist": 4, "k_nc_markers": 5}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = 30
    seg = msegment.Segmenter(0)
    frames = {
        "mosaic_noise": synth.mosaic_image(n, n, 2, noise=3),
        "uniform": np.full((n, n, 3), 77, np.uint8),
        "random": np.random.default_rng(0).integers(0, 256, (n, n, 3), dtype=np.uint8),
    }
    for name, img in frames.items():
        d = torch.from_numpy(img).cuda()
        m = torch.empty((n, n), dtype=torch.int32, device="cuda")
        g = torch.empty((n, n), dtype=torch.uint8, device="cuda")
        for _ in range(3):
            lv = seg.nc_marker_stage_dev(d, 4, m, msegment._lib.MSG_NC_GISTO_DIAP, gray=g)
        torch.cuda.synchronize()
        seg.set_profiling(True)
        seg.kernel_profile(reset=True)
        t0 = time.perf_counter()
        for _ in range(reps):
            seg.nc_marker_stage_dev(d, 4, m, msegment._lib.MSG_NC_GISTO_DIAP, gray=g)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        prof = seg.kernel_profile(reset=True)
        seg.set_profiling(False)
        line = ["%-13s levels=%3d stage=%7.1f us" % (name, len(lv), wall * 1e6)]
        for k, (launches, ms) in prof.items():
            if k in BYTES and launches:
                us = ms * 1e3 / launches
                line.append("%s %.1f us %.0f GB/s" % (k, us, BYTES[k] * n * n / (us * 1e-6) / 1e9))
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
