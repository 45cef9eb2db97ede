"""Real-photograph timing (the reference's album.jpg, 1500x1500, decoded pixels in
tests/golden/album_1500x1500.png): the shape-method pipeline (seed stage + flood +
colorByIndexes) on the GPU, each part timed, against the CPU oracles on the same pixels; and the
flood alone from the oracle's markers.  usage: python scripts/real_image_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

import msegment  # noqa: E402
from oracle import shape_oracle as so  # noqa: E402
from oracle import ws_oracle  # noqa: E402


def main():
    rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
    img = np.ascontiguousarray(rgb[..., ::-1])
    H, W = img.shape[:2]
    dev = torch.device("cuda", 0)
    seg = msegment.Segmenter(0)
    t_img = torch.from_numpy(img).to(dev)
    mk = torch.empty((H, W), dtype=torch.int32, device=dev)
    lab = torch.empty_like(mk)
    dst = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
    out = {"frame": "album.jpg %dx%d" % (H, W)}
    for _ in range(2):  # warm-up
        d, n = seg.shape_markers_dev(t_img, mk)
        seg.watershed_colorize_dev(t_img, mk, lab, d, None, dst)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        d, n = seg.shape_markers_dev(t_img, mk)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(reps):
        seg.watershed_colorize_dev(t_img, mk, lab, d, None, dst)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    st = seg.stats()
    gpu_stage, gpu_flood = (t1 - t0) / reps, (t2 - t1) / reps
    c0 = time.perf_counter()
    s = so.shape_stages(img)
    c1 = time.perf_counter()
    want = ws_oracle.watershed(img, s["markers"])
    c2 = time.perf_counter()
    out.update({
        "depth": d, "ncomp": n,
        "markers_bit_exact": bool(np.array_equal(mk.cpu().numpy(), s["markers"])) and d == s["depth"],
        "labels_bit_exact": bool(np.array_equal(lab.cpu().numpy(), want)),
        "gpu_stage_ms": round(1000 * gpu_stage, 3), "gpu_flood_ms": round(1000 * gpu_flood, 3),
        "gpu_mpx_s": round(H * W / (gpu_stage + gpu_flood) / 1e6, 2),
        "cpu_stage_ms": round(1000 * (c1 - c0), 1), "cpu_flood_ms": round(1000 * (c2 - c1), 1),
        "cpu_mpx_s": round(H * W / (c2 - c0) / 1e6, 2),
        "flood": {k: st[k] for k in ("batches", "pops", "items", "host_syncs")},
    })
    print(json.dumps(out), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
