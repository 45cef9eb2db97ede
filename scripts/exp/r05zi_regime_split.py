"""Where a serial-regime flood's time goes (msg_set_diag 3, bank 2): tiny batches (count, pops,
time), serial pops (count, time), small-batch pops; album.jpg with the shape seeds, NC 1024^2."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

import msegment  # noqa: E402
import spec_probe  # noqa: E402

seg = msegment.Segmenter(0)
dev = torch.device("cuda", 0)
for nm in ("album_shape", "nc_mosaic_noise_1024_s1"):
    img, m = spec_probe.load(seg, nm)
    ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
    tl = torch.empty_like(tm)
    seg.set_diag(0)
    ms = spec_probe.flood_ms(seg, ti, tm, tl)
    seg.set_diag(3)
    seg.watershed_dev(ti, tm, tl)
    torch.cuda.synchronize()
    d = seg.stats()["diag"]
    st = seg.stats()
    print("%-24s %.1f ms (diag off) | tiny batches %d (%d pops, %.1f ms) | serial pops %d (%.1f ms) | small-batch pops %d | "
          "generation pops %d (%.1f ms) | total pops %d" % (nm, ms, d[0], d[1], d[2] / 1e5, d[3], d[4] / 1e5, d[7],
                                                            st["spec_gen_pops"], st["spec_gen_us"] / 1e3, st["pops"]),
          flush=True)
seg.close()
