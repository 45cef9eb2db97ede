"""Generate the committed golden fixtures for the watershed hot path.

Run from the repo root:  python tests/golden/make_golden.py

Parity is unpinned by the reference (it has no tests or fixtures for this path and OpenCV 3.4.2
cannot run here), so every expected output below is produced by the C oracle
(oracle/ws_oracle.c) AND checked against the independent pure-Python restatement
(oracle/ws_pyref.py) before it is written.  The one real-image case decodes the reference's own
resource src/main/resources/images/hkp.jpg with PIL (into raw BGR bytes, stored as data) when the
reference tree is present; the decoded pixels are what the fixture pins, not the JPEG decoder.

album_1500x1500.png is the reference's resource src/main/resources/images/album.jpg decoded by PIL
and re-encoded losslessly (write_album below): a real 1500x1500 photograph for the shape-method
pipeline and real-image flood timing (scripts/real_image_probe.py, tests/test_gpu_real.py).

Outputs (numpy .npz, no pickles):
  small_cases.npz  inputs + expected labels + expected colourised/gray outputs, small frames
  digests.json     SHA-256 of the oracle's label maps for larger synthetic frames, and of the
                   marker-stage pipelines' 4096^2 frames (--pipelines)
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "opencv-msegment_amd"))

from oracle import ws_oracle, ws_pyref  # noqa: E402
from msegment import synth  # noqa: E402
from msegment.jrandom import generate_bgr_palette  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_IMG = "/root/reference/src/main/resources/images/hkp.jpg"


def random_markers(rng, H, W, k, lo=-3, hi=6):
    m = np.zeros((H, W), np.int32)
    for _ in range(k):
        m[rng.integers(0, H), rng.integers(0, W)] = rng.integers(lo, hi)
    return m


def cases():
    rng = np.random.default_rng(20261015)
    out = []
    # synthetic generator frames (small sizes of BASELINE configs' kinds)
    for kind, H, W, seed in [("mosaic", 32, 32, 0), ("mosaic", 48, 64, 5), ("mosaic_noise", 64, 64, 7),
                             ("random", 40, 48, 9), ("mosaic", 256, 256, 0),
                             ("mosaic_noise", 96, 80, 11)]:
        img, m, depth = synth.frame(kind, H, W, seed)
        out.append(("%s_%dx%d_s%d" % (kind, H, W, seed), img, m, depth))
    # quantised random images with sparse random markers, negatives and frame labels included
    for t in range(8):
        H, W = int(rng.integers(3, 40)), int(rng.integers(3, 40))
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        if t % 2:
            img = (img // 85 * 85).astype(np.uint8)
        m = random_markers(rng, H, W, int(rng.integers(1, 12)))
        out.append(("rand%d_%dx%d" % (t, H, W), img, m, 5))
    # a plateau with two seeds (ties everywhere) and a ramp
    H, W = 24, 30
    img = np.full((H, W, 3), 77, np.uint8)
    m = np.zeros((H, W), np.int32)
    m[5, 5] = 1
    m[17, 22] = 2
    out.append(("plateau_24x30", img, m, 2))
    ramp = np.broadcast_to((np.arange(W, dtype=np.int32) * 7 % 256).astype(np.uint8)[None, :, None], (H, W, 3)).copy()
    out.append(("ramp_24x30", ramp, m.copy(), 2))
    # real image from the reference's resources (decoded pixels are the fixture)
    if os.path.exists(REF_IMG):
        from PIL import Image

        rgb = np.asarray(Image.open(REF_IMG).convert("RGB"))
        bgr = np.ascontiguousarray(rgb[:, :, ::-1])
        H, W, _ = bgr.shape
        m = synth.seeds(H, W, 4, cells=12)
        out.append(("hkp_%dx%d" % (H, W), bgr, m, int(m.max())))
    return out


def main():
    arrays = {}
    names = []
    for name, img, m, depth in cases():
        lab = ws_oracle.watershed(img, m)
        if img.shape[0] * img.shape[1] <= 70000:
            ref = ws_pyref.watershed(img, m)
            assert np.array_equal(lab, ref), "oracle and pyref disagree on %s" % name
        pal = generate_bgr_palette(depth, 1234)
        col = ws_oracle.colorize(lab, depth, pal)
        white = ws_oracle.colorize(lab, depth, None)
        arrays[name + "__img"] = img
        arrays[name + "__markers"] = m
        arrays[name + "__labels"] = lab
        arrays[name + "__depth"] = np.array(depth, np.int32)
        arrays[name + "__palette"] = pal
        arrays[name + "__color"] = col
        arrays[name + "__white"] = white
        arrays[name + "__gray"] = ws_oracle.bgr2gray(col)
        names.append(name)
    arrays["__names"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "small_cases.npz"), **arrays)

    write_digests()
    write_pipeline_digests()
    print("wrote", len(names), "small cases")


# (kind, H, W, seed): SURVEY.md §8d seeds -- cfg2 1024^2 s=1, cfg3 4096^2 s=2, cfg4 16384^2 s=3,
# cfg5's first frame 4096^2 s=100; plus a large frame with ragged 4x4 tiles in both directions;
# cfg3's stress variants (mosaic+noise and uniform-random at 4096^2 s=2);
# a 537 M-pixel frame (2x config 4) near the flood's 32-bit index limit
DIGEST_CASES = [("mosaic", 1024, 1024, 1), ("mosaic_noise", 1024, 1024, 1),
                ("random", 512, 512, 3), ("mosaic", 4096, 4096, 2), ("mosaic", 16384, 16384, 3),
                ("mosaic", 4096, 4096, 100), ("mosaic", 3001, 5003, 7),
                ("mosaic_noise", 4096, 4096, 2), ("random", 4096, 4096, 2),
                ("mosaic", 16387, 32749, 11)]  # above 2^28 pixels, ragged tiles: the flood's size limit
# config 5's other 63 frames (seeds 100 + k, k = 1..63: SURVEY 8d; bench.py --gpus N gives rank r
# the batch of frames 100 + 8r .. 100 + 8r + 7, so all 64 are checked at N = 8)
DIGEST_CASES += [("mosaic", 4096, 4096, 100 + k) for k in range(1, 64)]


def write_digests(only=None):
    path = os.path.join(OUT, "digests.json")
    digests = json.load(open(path)) if (only and os.path.exists(path)) else {}
    for kind, H, W, seed in DIGEST_CASES:
        key = "%s_%dx%d_s%d" % (kind, H, W, seed)
        if only and key not in only:
            continue
        img, m, depth = synth.frame(kind, H, W, seed)
        lab = ws_oracle.watershed(img, m)
        digests[key] = {
            "labels_sha256": hashlib.sha256(lab.tobytes()).hexdigest(),
            "img_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
            "markers_sha256": hashlib.sha256(m.tobytes()).hexdigest(),
            "depth": depth,
            "wshed_pixels": int((lab == -1).sum()),
            "zero_pixels": int((lab == 0).sum()),
        }
        print(key, digests[key]["labels_sha256"][:16])
        del img, m, lab
    with open(path, "w") as f:
        json.dump(digests, f, indent=1, sort_keys=True)


# The marker-stage pipelines' 4096^2 frames as bench.py --pipeline nc / shape / color time them
# (mosaic seed 2; nc: depth 4, GISTO_DIAP): the numpy restatements of the marker stages
# (oracle/nc_oracle.py, shape_oracle.py, color_oracle.py) then the C flood.  ~1 min in all.
PIPELINE_CASES = [("nc", "mosaic", 4096, 2, 4, "GISTO_DIAP"), ("shape", "mosaic", 4096, 2, None, None),
                  ("color", "mosaic", 4096, 2, None, None)]


def pipeline_key(pipe, kind, S, seed, depth=None, opts=None):
    if pipe == "nc":
        return "nc_%s_%dx%d_s%d_d%d_%s" % (kind, S, S, seed, depth, opts or "none")
    return "%s_%s_%dx%d_s%d" % (pipe, kind, S, S, seed)


def write_pipeline_digests():
    from oracle import color_oracle, nc_oracle, shape_oracle

    path = os.path.join(OUT, "digests.json")
    digests = json.load(open(path))
    for pipe, kind, S, seed, depth, opts in PIPELINE_CASES:
        img, _, _ = synth.frame(kind, S, S, seed)
        src, extra = img, {}
        if pipe == "nc":
            _, _, lv, mk = nc_oracle.marker_stage(img, depth, gisto_diap="GISTO_DIAP" in (opts or ""))
            d = len(lv)
        elif pipe == "shape":
            mk, d = shape_oracle.shape_markers(img, shape_oracle.blur_mask_size(S, S))
        else:
            src, mk, d = color_oracle.color_markers(img)
            extra["sharp_sha256"] = hashlib.sha256(src.tobytes()).hexdigest()
        lab = ws_oracle.watershed(src, mk)
        key = pipeline_key(pipe, kind, S, seed, depth, opts)
        digests[key] = dict(extra, labels_sha256=hashlib.sha256(lab.tobytes()).hexdigest(),
                            markers_sha256=hashlib.sha256(np.ascontiguousarray(mk, np.int32).tobytes()).hexdigest(),
                            depth=int(d), wshed_pixels=int((lab == -1).sum()), zero_pixels=int((lab == 0).sum()))
        print(key, digests[key]["labels_sha256"][:16], "depth", d)
    with open(path, "w") as f:
        json.dump(digests, f, indent=1, sort_keys=True)


def write_album():
    """The reference's resource images, decoded by PIL (RGB, palette expanded) and re-encoded
    losslessly: the decoded pixels are the fixture (data), not the decoder."""
    from PIL import Image

    res = "/root/reference/src/main/resources/images/"
    for src, name in (("album.jpg", "album_1500x1500.png"), ("guide.png", None), ("haha.jpg", None)):
        rgb = np.asarray(Image.open(res + src).convert("RGB"))
        if name is None:
            name = "%s_%dx%d.png" % (src.split(".")[0], rgb.shape[0], rgb.shape[1])
        Image.fromarray(rgb).save(os.path.join(OUT, name), optimize=True)
        print(name, rgb.shape, int(np.all(rgb == 255, axis=2).sum()), "white pixels")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--album":
        write_album()
    elif len(sys.argv) > 1 and sys.argv[1] == "--pipelines":
        write_pipeline_digests()
    elif len(sys.argv) > 1 and sys.argv[1] == "--digests-only":  # e.g. --digests-only mosaic_16384x16384_s3
        write_digests(set(sys.argv[2:]) or None)
    else:
        main()
