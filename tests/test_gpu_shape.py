"""GPU parity of the SHAPE_METHOD marker stage (PictureService.shapeAutoMarkerWatershed,
PictureService.java:395-466) and of the whole shape pipeline (markers -> watershed ->
colorByIndexes -> BGR2GRAY) against the CPU oracles (oracle/shape_oracle.py, ws_oracle),
bit-exact on every intermediate (blurred gray, Canny edges, marker mask), the int32 markers and
the contour count, through the C ABI."""
import os

import numpy as np
import pytest

import msegment
from msegment import synth
from msegment.jrandom import generate_bgr_palette
from oracle import shape_oracle as so
from oracle import ws_oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "small_cases.npz")


def _torch():
    import torch

    return torch


def smooth_blobs(H, W, seed, n=12):
    """Soft-edged discs on a gradient: edges with weak tails, rings, holes, touching shapes."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    img = np.zeros((H, W, 3), np.float64)
    img += (xx / max(W, 1) * 60)[..., None]
    for _ in range(n):
        cy, cx = rng.uniform(0, H), rng.uniform(0, W)
        rad = rng.uniform(3, max(4, min(H, W) / 4))
        col = rng.uniform(0, 255, 3)
        d = np.sqrt((yy - cy) ** 2 + (xx - cx) ** 2)
        a = np.clip(rad - d, 0, 1)[..., None]
        img = img * (1 - a) + col * a
    img += rng.normal(0, 2, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def frames():
    out = []
    g = np.load(GOLDEN)
    out.append(("hkp_184", g["hkp_184x184__img"]))
    out.append(("mosaic_256", g["mosaic_256x256_s0__img"]))
    out.append(("mosaic_noise_96x80", g["mosaic_noise_96x80_s11__img"]))
    out.append(("mosaic_cells4", synth.frame("mosaic", 96, 128, 5, cells=4)[0]))
    for k, (H, W) in enumerate([(150, 200), (257, 300), (61, 77), (370, 129), (33, 500)]):
        out.append(("blobs_%dx%d" % (H, W), smooth_blobs(H, W, 40 + k)))
    out.append(("random_40x48", g["random_40x48_s9__img"]))
    return out


FRAMES = frames()


def stage_gpu(seg, img, ksize=None):
    torch = _torch()
    H, W = img.shape[:2]
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(np.ascontiguousarray(img)).to(dev)
    mk = torch.empty((H, W), dtype=torch.int32, device=dev)
    blur = torch.empty((H, W), dtype=torch.uint8, device=dev)
    edges = torch.empty_like(blur)
    mask = torch.empty_like(blur)
    depth, ncomp = seg.shape_markers_dev(t, mk, ksize=ksize, blur=blur, edges=edges, mask=mask)
    torch.cuda.synchronize()
    return {"blur": blur.cpu().numpy(), "edges": edges.cpu().numpy(), "mask": mask.cpu().numpy(),
            "markers": mk.cpu().numpy(), "depth": depth, "ncomp": ncomp}


def _check(got, want, name):
    for key in ("blur", "edges", "mask", "markers"):
        if not np.array_equal(got[key], want[key]):
            bad = int((got[key] != want[key]).sum())
            raise AssertionError("%s: %s differs at %d pixels" % (name, key, bad))
    assert (got["ncomp"], got["depth"]) == (want["ncomp"], want["depth"]), name


@pytest.mark.parametrize("name,img", FRAMES, ids=[f[0] for f in FRAMES])
def test_shape_stage_matches_oracle(seg, name, img):
    _check(stage_gpu(seg, img), so.shape_stages(img), name)


@pytest.mark.parametrize("ksize", [1, 3, 9, 21, 31])
def test_shape_stage_explicit_median_sizes(seg, ksize):
    img = smooth_blobs(140, 190, 7)
    _check(stage_gpu(seg, img, ksize), so.shape_stages(img, ksize), "k%d" % ksize)


@pytest.mark.parametrize("shape", [(1, 1), (2, 5), (3, 3), (5, 1), (1, 64), (7, 9)])
def test_shape_stage_tiny_frames(seg, shape):
    rng = np.random.default_rng(shape[0] * 31 + shape[1])
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    _check(stage_gpu(seg, img), so.shape_stages(img), "tiny%s" % (shape,))


def test_shape_stage_flat_frame_has_no_contour(seg):
    img = np.full((64, 80, 3), 77, np.uint8)
    got = stage_gpu(seg, img)
    assert got["depth"] == 0 and got["ncomp"] == 0 and not got["markers"].any()
    torch = _torch()
    ps = msegment.PictureService(segmenter=seg, seed=1)
    assert ps.shape_auto_marker_watershed(img) is None  # the reference returns null (:448-451)


def test_shape_markers_host_api(seg):
    img = FRAMES[0][1]
    mk, depth, ncomp = seg.shape_markers(img)
    want = so.shape_stages(img)
    assert np.array_equal(mk, want["markers"]) and (depth, ncomp) == (want["depth"], want["ncomp"])
    # strided (non-contiguous) view of a larger frame
    big = np.zeros((img.shape[0], img.shape[1] + 9, 3), np.uint8)
    big[:, 4:4 + img.shape[1]] = img
    mk2, d2, _ = seg.shape_markers(big[:, 4:4 + img.shape[1]])
    assert np.array_equal(mk2, want["markers"]) and d2 == want["depth"]


@pytest.mark.parametrize("colored", [False, True])
def test_shape_pipeline_matches_oracle(seg, colored):
    """markers -> this.watershed(src, markers, depth, colored) (:455) -> bw_result (:460-462)."""
    img = FRAMES[4][1]
    want = so.shape_stages(img)
    ps = msegment.PictureService(segmenter=seg, seed=5)
    res = ps.shape_auto_marker_watershed(img, ("COLORED",) if colored else ())
    labels = ws_oracle.watershed(img, want["markers"])
    assert res.depth == want["depth"]
    assert np.array_equal(res.labels, labels)
    pal = generate_bgr_palette(want["depth"], 5) if colored else None
    col = ws_oracle.colorize(labels, want["depth"], pal)
    assert np.array_equal(res.dst, col)
    assert np.array_equal(res.bw, ws_oracle.bgr2gray(col))


def test_shape_stage_large_frame_invariants(seg):
    """2048^2: no oracle run at this size -- structural invariants of the GPU result."""
    img = smooth_blobs(2048, 2048, 99, n=300)
    got = stage_gpu(seg, img)
    mk, n = got["markers"], got["ncomp"]
    assert n > 0 and mk.max() == n and mk.min() == 0
    assert np.array_equal(mk > 0, got["mask"] > 0)
    # numbering: first 2x2 block of label l precedes that of l + 1
    r, c = np.nonzero(mk)
    bkey = (r >> 1) * 1024 + (c >> 1)
    first = np.full(n + 1, 1 << 40, np.int64)
    np.minimum.at(first, mk[r, c], bkey)
    assert np.all(np.diff(first[1:]) > 0)
    # the oracle on a crop of the mask agrees with the GPU mask-only steps there
    crop = got["mask"][:300, :300]
    lab, nc = so.components(crop)
    assert nc > 0
