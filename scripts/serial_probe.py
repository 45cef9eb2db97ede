"""The serial-pop regime per frame: flood time with the serial pops inside k_scan's loop (the
default) and in k_serial (msg_set_serial_kernel), each with the speculative engine on and off,
bit-exactness against the C oracle, and the C oracle's time.  Frames as in spec_probe.py.
usage: python scripts/serial_probe.py NAME..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd"), os.path.join(ROOT, "scripts")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import msegment  # noqa: E402
from spec_probe import flood_ms, load  # noqa: E402


def main():
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    from oracle import ws_oracle
    for nm in sys.argv[1:]:
        img, m = load(seg, nm)
        ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        tl = torch.empty_like(tm)
        c0 = time.perf_counter()
        want = ws_oracle.watershed(img, m)
        cms = 1e3 * (time.perf_counter() - c0)
        row = []
        for serk in (False, True):
            for spec in (True, False):
                seg.set_serial_kernel(serk)
                seg.set_speculative(spec)
                ms = flood_ms(seg, ti, tm, tl)
                ok = np.array_equal(tl.cpu().numpy(), want)
                row.append("%s/%s %.1f ms%s" % ("k_serial" if serk else "in-loop", "spec" if spec else "nospec", ms,
                                                "" if ok else " MISMATCH"))
        seg.set_serial_kernel(False)
        seg.set_speculative(True)
        print("%-24s C oracle %.1f ms | %s" % (nm, cms, " | ".join(row)), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
