"""k_bilateral (the NC BILATERAL pre-filter, PictureService.java:488-495) at 4096^2: per-launch
time from the library's HIP events for several mask sizes d, and the gathered bytes per launch
(one byte per tap per pixel, mostly L1/L2 hits) against the streamed 2 B/px; the 1024^2 output is
checked against oracle/nc_oracle.bilateral."""
import sys

sys.path[:0] = ["/root/repo", "/root/repo/opencv-msegment_amd"]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import _lib, synth  # noqa: E402
from oracle import nc_oracle as O  # noqa: E402

seg = msegment.Segmenter(0)
dev = torch.device("cuda", 0)
for S, ds in ((1024, (5,)), (4096, (3, 5, 9, 15))):
    img = synth.mosaic_image(S, S, 2, noise=3)
    ti = torch.from_numpy(img).to(dev)
    mk = torch.empty((S, S), dtype=torch.int32, device=dev)
    g = torch.empty((S, S), dtype=torch.uint8, device=dev)
    for d in ds:
        flags = _lib.MSG_NC_BILATERAL | _lib.MSG_NC_MASK(d)
        seg.nc_marker_stage_dev(ti, 4, mk, flags, gray=g)
        torch.cuda.synchronize()
        ok = ""
        if S <= 1024:
            ok = "exact" if np.array_equal(g.cpu().numpy(), O.bilateral(O.gray(img), d)) else "MISMATCH"
        seg.set_profiling(True)
        seg.kernel_profile(reset=True)
        reps = 5
        for _ in range(reps):
            seg.nc_marker_stage_dev(ti, 4, mk, flags, gray=g)
        torch.cuda.synchronize()
        prof = seg.kernel_profile(reset=True)
        seg.set_profiling(False)
        n, ms = prof["k_bilateral"]
        us = 1000.0 * ms / n
        taps = len(O.bilateral_tables(d)[2])
        print("%d^2 d=%d taps=%d: k_bilateral %.1f us (%.0f Mpx/s, %.2f TB/s of tap gathers, %.2f TB/s streamed) %s"
              % (S, d, taps, us, S * S / us, S * S * taps / us / 1e6, 2 * S * S / us / 1e6, ok), flush=True)
