"""GPU parity of the NOT_CONNECTED_MARKERS marker stage (PictureService.java:468-842) and of the
whole NC pipeline (marker stage -> watershed -> colorByIndexes -> BGR2GRAY) against the CPU
oracles (oracle/nc_oracle.py, oracle/ws_oracle.py), bit-exact, through the C ABI."""
import numpy as np
import pytest

import msegment
from msegment import _lib, synth
from msegment.jrandom import JavaRandom
from oracle import nc_oracle as O
from oracle import ws_oracle

pytestmark = pytest.mark.gpu

GISTO = _lib.MSG_NC_GISTO_DIAP


def _torch():
    import torch

    return torch


def _dev(a):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


@pytest.mark.parametrize("shape", [(1, 1), (1, 3), (3, 5), (7, 1), (97, 131), (256, 256), (1023, 1025)])
def test_gray_hist_matches_oracle(seg, shape):
    torch = _torch()
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    g = torch.zeros(shape, dtype=torch.uint8, device="cuda:0")
    hist = seg.gray_hist_dev(_dev(img), g)
    torch.cuda.synchronize()
    want = O.gray(img)
    assert np.array_equal(g.cpu().numpy(), want)
    assert np.array_equal(hist, O.hist256(want))


def test_gray_hist_uniform_and_mosaic_4096(seg):
    torch = _torch()
    # a constant frame (one bin takes every count: worst-case atomic contention) and the
    # BASELINE config-3 mosaic
    for img in (np.full((4096, 4096, 3), 77, np.uint8), synth.mosaic_image(4096, 4096, 2, noise=3)):
        g = torch.empty(img.shape[:2], dtype=torch.uint8, device="cuda:0")
        hist = seg.gray_hist_dev(_dev(img), g)
        torch.cuda.synchronize()
        want = O.gray(img)
        assert np.array_equal(g.cpu().numpy(), want)
        assert np.array_equal(hist, O.hist256(want))
        assert hist.sum() == img.shape[0] * img.shape[1]


@pytest.mark.parametrize("shape", [(1, 1), (5, 3), (64, 64), (333, 517)])
def test_markers_from_table(seg, shape):
    torch = _torch()
    rng = np.random.default_rng(shape[1])
    gray = rng.integers(0, 256, shape, dtype=np.uint8)
    lut = rng.integers(-3, 40, 256).astype(np.int32)
    m = torch.full(shape, 12345, dtype=torch.int32, device="cuda:0")
    seg.nc_markers_dev(_dev(gray), lut, m)
    torch.cuda.synchronize()
    assert np.array_equal(m.cpu().numpy(), O.markers(gray, lut))


@pytest.mark.parametrize("opts", [0, GISTO])
@pytest.mark.parametrize("kind,shape,depth", [("mosaic_noise", (256, 256), 4), ("mosaic", (300, 411), 8),
                                              ("random", (128, 96), 2)])
def test_marker_stage_matches_oracle(seg, opts, kind, shape, depth):
    torch = _torch()
    img, _, _ = synth.frame(kind, shape[0], shape[1], 5)
    g, h, lv, mk = O.marker_stage(img, depth, gisto_diap=bool(opts))
    m = torch.empty(shape, dtype=torch.int32, device="cuda:0")
    gray = torch.empty(shape, dtype=torch.uint8, device="cuda:0")
    got = seg.nc_marker_stage_dev(_dev(img), depth, m, opts, gray=gray)
    torch.cuda.synchronize()
    assert got == lv
    assert np.array_equal(gray.cpu().numpy(), g)
    assert np.array_equal(m.cpu().numpy(), mk)
    # context scratch for gray
    m2 = torch.empty(shape, dtype=torch.int32, device="cuda:0")
    assert seg.nc_marker_stage_dev(_dev(img), depth, m2, opts) == lv
    torch.cuda.synchronize()
    assert np.array_equal(m2.cpu().numpy(), mk)


@pytest.mark.parametrize("k", [1, 3, 5, 9, 15])
@pytest.mark.parametrize("kind,shape", [("mosaic_noise", (211, 307)), ("random", (64, 96))])
def test_marker_stage_median_blur(seg, k, kind, shape):
    """MEDIAN_BLUR (PictureService.java:481-483): medianBlur(srcGray, k), then histogram, levels
    and markers from the blurred gray."""
    torch = _torch()
    img, _, _ = synth.frame(kind, shape[0], shape[1], 9)
    g, h, lv, mk = O.marker_stage(img, 4, median_blur=k)
    m = torch.empty(shape, dtype=torch.int32, device="cuda:0")
    gray = torch.empty(shape, dtype=torch.uint8, device="cuda:0")
    got = seg.nc_marker_stage_dev(_dev(img), 4, m, _lib.MSG_NC_MEDIAN_BLUR | _lib.MSG_NC_MASK(k), gray=gray)
    torch.cuda.synchronize()
    assert np.array_equal(gray.cpu().numpy(), g)
    assert got == lv
    assert np.array_equal(m.cpu().numpy(), mk)


def test_marker_stage_median_blur_even_mask(seg):
    torch = _torch()
    img, _, _ = synth.frame("mosaic_noise", 32, 32, 9)
    m = torch.empty((32, 32), dtype=torch.int32, device="cuda:0")
    with pytest.raises(msegment.MsegError) as e:
        seg.nc_marker_stage_dev(_dev(img), 4, m, _lib.MSG_NC_MEDIAN_BLUR | _lib.MSG_NC_MASK(4))
    assert e.value.code == _lib.MSG_EINVAL


@pytest.mark.parametrize("d", [0, 1, 3, 5, 8, 15])
@pytest.mark.parametrize("kind,shape", [("mosaic_noise", (211, 307)), ("random", (64, 96)), ("mosaic", (5, 7))])
def test_marker_stage_bilateral(seg, d, kind, shape):
    """BILATERIAL (PictureService.java:488-495): bilateralFilter(srcGray, dst, d, 2d, 2d), then
    histogram, levels and markers from dst; bit-exact against oracle/nc_oracle.bilateral (fp32,
    the same summation order; d = 0 is radius cvRound(1.5), the 5x7 frame folds its border
    twice at d = 15)."""
    torch = _torch()
    img, _, _ = synth.frame(kind, shape[0], shape[1], 9)
    g, h, lv, mk = O.marker_stage(img, 4, bilateral_d=d)
    m = torch.empty(shape, dtype=torch.int32, device="cuda:0")
    gray = torch.empty(shape, dtype=torch.uint8, device="cuda:0")
    try:
        got = seg.nc_marker_stage_dev(_dev(img), 4, m, _lib.MSG_NC_BILATERAL | _lib.MSG_NC_MASK(d), gray=gray)
    except msegment.MsegError as e:  # a filtered frame with no level: the reference throws too
        assert e.code == _lib.MSG_ESTATE and not lv
        return
    torch.cuda.synchronize()
    assert np.array_equal(gray.cpu().numpy(), g)
    assert got == lv
    assert np.array_equal(m.cpu().numpy(), mk)


def test_bilateral_non_square_partial_blocks(seg):
    """A 777 x 1000 frame (width not a multiple of 64: partial blocks; rows and columns reflect at
    both ends) through d = 9 bit-exact -- the large-frame check of the test below on a frame that
    is neither square nor block-aligned."""
    torch = _torch()
    img = synth.mosaic_image(777, 1000, 4, noise=3)
    g, h, lv, mk = O.marker_stage(img, 4, bilateral_d=9)
    m = torch.empty((777, 1000), dtype=torch.int32, device="cuda:0")
    gray = torch.empty((777, 1000), dtype=torch.uint8, device="cuda:0")
    assert seg.nc_marker_stage_dev(_dev(img), 4, m, _lib.MSG_NC_BILATERAL | _lib.MSG_NC_MASK(9), gray=gray) == lv
    torch.cuda.synchronize()
    assert np.array_equal(gray.cpu().numpy(), g)
    assert np.array_equal(m.cpu().numpy(), mk)


def test_bilateral_1024_and_median_precedence(seg):
    """A 1024^2 noisy mosaic through the BILATERIAL branch (d = 9: a 69-tap disc) bit-exact, and
    MEDIAN_BLUR winning when both flags are set (the reference's if / else-if)."""
    torch = _torch()
    img = synth.mosaic_image(1024, 1024, 4, noise=3)
    g, h, lv, mk = O.marker_stage(img, 4, bilateral_d=9)
    assert not np.array_equal(g, O.gray(img))
    m = torch.empty((1024, 1024), dtype=torch.int32, device="cuda:0")
    gray = torch.empty((1024, 1024), dtype=torch.uint8, device="cuda:0")
    assert seg.nc_marker_stage_dev(_dev(img), 4, m, _lib.MSG_NC_BILATERAL | _lib.MSG_NC_MASK(9), gray=gray) == lv
    torch.cuda.synchronize()
    assert np.array_equal(gray.cpu().numpy(), g)
    assert np.array_equal(m.cpu().numpy(), mk)
    g2, _, lv2, mk2 = O.marker_stage(img[:256, :256], 4, median_blur=5)
    m2 = torch.empty((256, 256), dtype=torch.int32, device="cuda:0")
    both = _lib.MSG_NC_MEDIAN_BLUR | _lib.MSG_NC_BILATERAL | _lib.MSG_NC_MASK(5)
    assert seg.nc_marker_stage_dev(_dev(img[:256, :256]), 4, m2, both) == lv2
    torch.cuda.synchronize()
    assert np.array_equal(m2.cpu().numpy(), mk2)


def test_marker_stage_multi_otsu(seg):
    torch = _torch()
    # three flat patches -> three flex levels -> the multi-Otsu override (k = 3)
    img = np.zeros((64, 96, 3), np.uint8)
    img[:, :32] = (20, 30, 40)
    img[:, 32:64] = (90, 100, 110)
    img[:, 64:] = (200, 210, 220)
    g, h, lv, mk = O.marker_stage(img, 4, multi_otsu_opt=True)
    assert len(O.flex_levels(h, 4)) == 3
    m = torch.empty((64, 96), dtype=torch.int32, device="cuda:0")
    assert seg.nc_marker_stage_dev(_dev(img), 4, m, _lib.MSG_NC_MULTI_OTSU) == lv
    torch.cuda.synchronize()
    assert np.array_equal(m.cpu().numpy(), mk)


def test_marker_stage_errors(seg):
    torch = _torch()
    img = np.full((8, 8, 3), 255, np.uint8)  # one bin at 255: never emitted -> no level
    m = torch.empty((8, 8), dtype=torch.int32, device="cuda:0")
    with pytest.raises(msegment.MsegError) as e:
        seg.nc_marker_stage_dev(_dev(img), 4, m)
    assert e.value.code == _lib.MSG_ESTATE
    buf = torch.empty(8 * 8 * 4 + 16, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(msegment.MsegError) as e:  # misaligned marker buffer
        seg.nc_markers_dev(_dev(np.zeros((8, 8), np.uint8)), np.zeros(256, np.int32), buf[4:].view(torch.int32))
    assert e.value.code == _lib.MSG_EINVAL


def _oracle_nc(img, depth, opts, seed, mask=3):
    """notConnectedMarkers end to end on the CPU oracles, with the reference's Random draws."""
    gisto, otsu, colored = "GISTO_DIAP" in opts, "MULTI_OTSU" in opts, "COLORED" in opts
    g, h, lv, mk = O.marker_stage(img, depth, gisto_diap=gisto, multi_otsu_opt=otsu,
                                  median_blur=mask if "MEDIAN_BLUR" in opts else 0,
                                  bilateral_d=mask if "BILATERIAL" in opts else None)
    n = len(lv)
    rnd = JavaRandom(seed)
    draw = lambda: [rnd.next_int(156) + 100 for _ in range(3)]  # noqa: E731
    step_pal = np.array([draw() for _ in range(n)], np.uint8).reshape(-1, 3)
    pal = np.array([draw() for _ in range(n)], np.uint8).reshape(-1, 3) if colored else None
    labels = ws_oracle.watershed(img, mk)
    dst = ws_oracle.colorize(labels, n, pal)
    return dst, ws_oracle.bgr2gray(dst), labels, lv, ws_oracle.colorize(mk, n, step_pal)


@pytest.mark.parametrize("opts", [("COLORED",), ("COLORED", "GISTO_DIAP"), (), ("MEDIAN_BLUR", "COLORED"),
                                  ("MEDIAN_BLUR", "BILATERIAL"),
                                  ("BILATERIAL",), ("BILATERIAL", "GISTO_DIAP", "COLORED")])
def test_not_connected_markers_pipeline(opts):
    img, _, _ = synth.frame("mosaic_noise", 192, 160, 11)
    ps = msegment.PictureService(seed=2024)
    r = ps.not_connected_markers(img, 4, opts, colored_markers=True, filter_mask_size=5)
    dst, bw, labels, lv, cm = _oracle_nc(img, 4, opts, 2024, mask=5)
    assert r.levels == lv
    assert np.array_equal(r.labels, labels)
    assert np.array_equal(r.colored_markers, cm)
    assert np.array_equal(r.dst, dst)
    assert np.array_equal(r.bw, bw)


def test_not_connected_markers_4096_properties(seg):
    """Config-3 size: the marker stage bit-exact against the (numpy-fast) oracle stage, and the
    flood's size-independent properties on its output."""
    torch = _torch()
    img = synth.mosaic_image(4096, 4096, 2, noise=3)
    g, h, lv, mk = O.marker_stage(img, 4, gisto_diap=True)
    d_img = _dev(img)
    m = torch.empty((4096, 4096), dtype=torch.int32, device="cuda:0")
    assert seg.nc_marker_stage_dev(d_img, 4, m, GISTO) == lv
    torch.cuda.synchronize()
    assert np.array_equal(m.cpu().numpy(), mk)
    n = len(lv)
    dst = torch.empty((4096, 4096, 3), dtype=torch.uint8, device="cuda:0")
    seg.watershed_colorize_dev(d_img, m, m, n, None, dst)
    torch.cuda.synchronize()
    lab = m.cpu().numpy()
    assert (lab[0, :] == -1).all() and (lab[-1, :] == -1).all()
    assert (lab[:, 0] == -1).all() and (lab[:, -1] == -1).all()
    inner = lab[1:-1, 1:-1]
    seeds = mk[1:-1, 1:-1] > 0
    assert np.array_equal(inner[seeds], mk[1:-1, 1:-1][seeds])  # seeds keep their label
    assert set(np.unique(inner)) <= set(range(-1, n + 1))


def test_host_buffer_marker_stage(seg):
    """msg_nc_marker_stage (the JNI shim's entry point): host buffers in and out."""
    img, _, _ = synth.frame("mosaic_noise", 211, 173, 9)
    for opts in (0, GISTO):
        g, h, lv, mk = O.marker_stage(img, 3, gisto_diap=bool(opts))
        markers, got = seg.nc_marker_stage(img, 3, opts)
        assert got == lv
        assert np.array_equal(markers, mk)
    with pytest.raises(msegment.MsegError) as e:
        seg.nc_marker_stage(np.full((4, 4, 3), 255, np.uint8), 3)
    assert e.value.code == _lib.MSG_ESTATE
