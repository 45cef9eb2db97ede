"""GPU parity of the COLOR_METHOD marker stage (PictureService.java:301-366) and of the whole
colour pipeline (marker stage -> watershed of the sharpened image -> colorByIndexes ->
BGR2GRAY) against the CPU oracle (oracle/color_oracle.py, oracle/ws_oracle.py), bit-exact on
every intermediate, through the C ABI.  Unpinned against a real OpenCV build."""
import os

import numpy as np
import pytest

import msegment
from msegment import synth
from msegment.jrandom import JavaRandom
from oracle import color_oracle as C
from oracle import ws_oracle

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch


def _rings(H, W, specs):
    img = np.zeros((H, W, 3), np.uint8)
    yy, xx = np.mgrid[0:H, 0:W]
    for cy, cx, r, colour in specs:
        d = np.hypot(yy - cy, xx - cx)
        img[(d < r) & (d > r * 0.35)] = colour
    return img


def _frames():
    out = []
    for kind, H, W, seed in (("mosaic", 256, 256, 3), ("mosaic_noise", 300, 211, 4), ("random", 128, 97, 5),
                             ("mosaic", 64, 1030, 6)):
        out.append(("%s_%dx%d" % (kind, H, W), synth.frame(kind, H, W, seed)[0]))
    out.append(("rings", _rings(160, 200, [(50, 60, 40, (200, 180, 160)), (100, 140, 45, (90, 200, 40)),
                                            (60, 150, 12, (255, 255, 255))])))
    # a ring enclosing an island enclosing a hole (nested components and holes)
    img = _rings(200, 200, [(100, 100, 90, (220, 220, 30))])
    img[70:130, 70:130] = (40, 230, 200)
    img[90:110, 90:110] = 0
    out.append(("nested", img))
    img = np.full((40, 60, 3), 255, np.uint8)  # white everywhere except a blob: white -> black
    img[10:30, 20:45] = (120, 30, 200)
    out.append(("white_bg", img))
    for H, W in ((1, 1), (2, 9), (9, 2), (5, 5), (7, 13)):
        rng = np.random.default_rng(H * 31 + W)
        out.append(("tiny_%dx%d" % (H, W), rng.integers(0, 256, (H, W, 3), dtype=np.uint8)))
    rgb = np.asarray(__import__("PIL.Image", fromlist=["Image"]).open(
        os.path.join(os.path.dirname(__file__), "golden", "album_1500x1500.png")).convert("RGB"))
    out.append(("album_crop", np.ascontiguousarray(rgb[400:800, 200:700, ::-1])))
    return out


@pytest.mark.parametrize("name,img", _frames(), ids=[f[0] for f in _frames()])
def test_color_markers_match_oracle(seg, name, img):
    torch = _torch()
    want = C.stages(img)
    H, W = img.shape[:2]
    d_img = torch.from_numpy(np.ascontiguousarray(img)).to("cuda:0")
    sharp = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    mk = torch.empty((H, W), dtype=torch.int32, device="cuda:0")
    depth = seg.color_markers_dev(d_img, sharp, mk)
    torch.cuda.synchronize()
    assert np.array_equal(sharp.cpu().numpy(), want["sharp"]), name
    got = mk.cpu().numpy()
    if not np.array_equal(got, want["markers"]):
        bad = np.argwhere(got != want["markers"])
        raise AssertionError("%s: %d marker pixels differ, first %s gpu=%d cpu=%d (depth %d/%d)" % (
            name, len(bad), bad[0].tolist(), got[tuple(bad[0])], want["markers"][tuple(bad[0])], depth,
            want["depth"]))
    assert depth == want["depth"], name


def test_color_markers_host_buffers(seg):
    img = synth.frame("mosaic_noise", 97, 131, 8)[0]
    sharp, m, depth = seg.color_markers(img)
    want = C.stages(img)
    assert np.array_equal(sharp, want["sharp"]) and np.array_equal(m, want["markers"])
    assert depth == want["depth"]


@pytest.mark.parametrize("opts", [("COLORED",), ()])
def test_color_auto_marker_watershed_pipeline(opts):
    img = synth.frame("mosaic", 192, 160, 12)[0]
    ps = msegment.PictureService(seed=77)
    r = ps.color_auto_marker_watershed(img, opts)
    sharp, mk, depth = C.color_markers(img)
    assert r.depth == depth and np.array_equal(r.sharp, sharp)
    labels = ws_oracle.watershed(sharp, mk)
    pal = None
    if "COLORED" in opts:
        rnd = JavaRandom(77)
        pal = np.array([[rnd.next_int(156) + 100 for _ in range(3)] for _ in range(depth)], np.uint8)
    dst = ws_oracle.colorize(labels, depth, pal)
    assert np.array_equal(r.labels, labels)
    assert np.array_equal(r.dst, dst)
    assert np.array_equal(r.bw, ws_oracle.bgr2gray(dst))


def _reference_image(name):
    from PIL import Image

    rgb = np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "golden", name)).convert("RGB"))
    return np.ascontiguousarray(rgb[:, :, ::-1])  # imread's BGR


@pytest.mark.parametrize("name", ["album_1500x1500.png", "guide_225x225.png", "haha_373x400.png"])
def test_color_pipeline_on_reference_images(name):
    """App.java:28's colour method end to end on the reference's own pictures (every one holds
    pure-white pixels, which the Java white -> black loop leaves white: PixelUtil.java:19)."""
    img = _reference_image(name)
    assert np.all(img == 255, axis=2).any()
    ps = msegment.PictureService(seed=5)
    r = ps.color_auto_marker_watershed(img, ())
    sharp, mk, depth = C.color_markers(img)
    assert np.array_equal(r.sharp, sharp), name
    assert r.depth == depth, name
    labels = ws_oracle.watershed(sharp, mk)
    if not np.array_equal(r.labels, labels):
        bad = np.argwhere(r.labels != labels)
        raise AssertionError("%s: %d labels differ, first %s" % (name, len(bad), bad[0].tolist()))
    dst = ws_oracle.colorize(labels, depth, None)
    assert np.array_equal(r.dst, dst) and np.array_equal(r.bw, ws_oracle.bgr2gray(dst))
