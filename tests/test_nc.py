"""NOT_CONNECTED_MARKERS marker stage (PictureService.java:468-842), CPU side.

* known-answer tests for the level logic, derived by hand from PictureService.java:574-640 /
  :650-722 / :781-828 and model/BrightLevel.java (each case says which lines it walks through);
* the oracle restatement (oracle/nc_oracle.py) against those answers;
* the library's host code (nc_levels.cpp through the C ABI: msg_nc_levels, msg_nc_marker_lut --
  host-only entry points, no GPU needed) against the oracle on random histograms.
"""
import numpy as np
import pytest

import msegment
from msegment import _lib
from oracle import nc_oracle as O

GISTO = _lib.MSG_NC_GISTO_DIAP
OTSU = _lib.MSG_NC_MULTI_OTSU


def H(**bins):
    h = np.zeros(256, dtype=np.int64)
    for k, v in bins.items():
        lo, _, hi = k[1:].partition("_")
        h[int(lo): int(hi or lo) + 1] = v
    return h


# (histogram, depth, expected flex levels)
KAT_LEVELS = [
    # two plateaus: a level extends while the running mean stays in [m/2, 3m/2] (:608-626),
    # closes on an empty bin (:590-598); a level's count adds its first bin twice (:604, :625)
    (H(b10_19=100, b30=5), 4, [(10, 19, 1100), (30, 30, 10)]),
    # block size limit 256/depth = 2 (:578, :617-623): closes every 2 bins
    (H(b50_54=10), 128, [(50, 51, 30), (52, 53, 20), (54, 54, 10)]),
    # mean jump 10 -> 55 > 15: split (:627-634)
    (H(b60=10, b61=100), 4, [(60, 60, 20), (61, 61, 100)]),
    # empty bin 0 followed by a non-empty bin 1: the initial block [hist[0]] = [0] gives
    # old mean 0, the band [0, 0] excludes the new mean, so an inverted level (1, 0) is emitted
    (H(b1=10), 4, [(1, 0, 10), (1, 1, 10)]),
    # the block still open at bin 255 is never emitted (the loop ends without a flush)
    (H(b10=3, b255=9), 4, [(10, 10, 6)]),
]


@pytest.mark.parametrize("hist,depth,want", KAT_LEVELS)
def test_oracle_flex_levels_known_answers(hist, depth, want):
    assert [l.tup() for l in O.flex_levels(hist, depth)] == want


@pytest.mark.parametrize("hist,depth,want", KAT_LEVELS)
def test_library_flex_levels_known_answers(hist, depth, want):
    assert msegment.nc_levels(hist, 64, 64, depth) == want


def test_known_answer_marker_tables():
    lv = [(10, 19, 1100), (30, 30, 10), (1, 0, 10), (1, 1, 10)]
    # means (BrightLevel.getMeanLevel): 10 + 9/2 = 14; 30; (1,0): range -1 -> 1 + (-1)/2 = 1; 1
    want = np.zeros(256, np.int32)
    want[14], want[30], want[1] = 1, 2, 3
    assert np.array_equal(O.marker_lut(lv), want)
    assert np.array_equal(msegment.nc_marker_lut(lv), want)
    # GISTO_DIAP (getMeanDiap(3)): (10,19) -> [11, 17]; (30,30) -> itself; (1,0) -> itself
    # (matches nothing); (1,1) -> itself, so brightness 1 goes to the 4th level
    want = np.zeros(256, np.int32)
    want[11:18], want[30], want[1] = 1, 2, 4
    assert np.array_equal(O.marker_lut(lv, True), want)
    assert np.array_equal(msegment.nc_marker_lut(lv, GISTO), want)


def test_known_answer_multi_otsu_single_level():
    # one flex level -> one threshold t; overrides [(0, t-1)], then last.end = 255 (:698-712)
    h = H(b10_19=100)
    assert O.levels(h, 10, 100, 4, multi_otsu_opt=True) == [(0, 255, 1000)]
    assert msegment.nc_levels(h, 10, 100, 4, OTSU) == [(0, 255, 1000)]


def test_errors_where_the_reference_throws():
    empty = np.zeros(256, np.int64)
    with pytest.raises(msegment.MsegError) as e:
        msegment.nc_levels(empty, 4, 4, 4)
    assert e.value.code == _lib.MSG_ESTATE
    with pytest.raises(ValueError):
        O.levels(empty, 4, 4, 4)
    with pytest.raises(msegment.MsegError) as e:
        msegment.nc_levels(H(b3=1), 1, 1, 0)  # 256 / 0
    assert e.value.code == _lib.MSG_EINVAL
    # 8 separated spikes -> 8 flex levels: otsuPart would enumerate ~C(128, 8) splits
    many = H(**{"b%d" % (10 * k + 5): 7 for k in range(8)})
    assert len(O.flex_levels(many, 4)) == 8
    with pytest.raises(msegment.MsegError) as e:
        msegment.nc_levels(many, 8, 7, 4, OTSU)
    assert e.value.code == _lib.MSG_ERANGE


def test_float_rounding_of_large_bins():
    # calcHist's CV_32F output read back with (int): 2^24 + 1 -> 2^24
    h = H(b100=(1 << 24) + 1, b101=(1 << 24) + 3)
    assert [l.tup() for l in O.flex_levels(h, 4)] == msegment.nc_levels(h, 1 << 13, 1 << 12, 4)
    assert O.flex_levels(h, 4)[0].count == (1 << 24) * 2 + (1 << 24) + 4


def _without_int_wrap(monkeypatch, fn):
    """The same oracle call with Python's unbounded ints in place of Java's 32-bit wrap."""
    with monkeypatch.context() as mp:
        mp.setattr(O, "_i32", lambda x: x)
        return fn()


def test_multi_otsu_wraps_bin_index_times_count(monkeypatch):
    # otsuPart's `ii * intensity` (PictureService.java:958) is an int product: reduced bin 125
    # (grey 250) holding 20 M pixels gives 2.5e9, which wraps negative in Java, and moves the
    # thresholds (frames of >= ~17 M pixels with a bright mode reach this)
    h = H(b10=3_000_000, b160=2_000_000, b250=20_000_000)
    rows, cols = 1000, int(h.sum()) // 1000
    want = [(0, 159, 3_000_000), (160, 161, 2_000_000), (162, 255, 20_000_000)]
    assert O.levels(h, rows, cols, 4, multi_otsu_opt=True) == want
    assert msegment.nc_levels(h, rows, cols, 4, OTSU) == want
    assert _without_int_wrap(monkeypatch, lambda: O.levels(h, rows, cols, 4, multi_otsu_opt=True)) != want


def test_multi_otsu_wraps_pixel_count(monkeypatch):
    # pixNum = rows * cols (PictureService.java:656) is an int: 65536 x 32768 wraps to -2^31
    h = np.zeros(256, np.int64)
    h[10:20], h[30], h[200:210] = 100, 5, 50
    want = [(0, -1, 0), (0, 255, 1505)]
    assert O.levels(h, 65536, 32768, 4, multi_otsu_opt=True) == want
    assert msegment.nc_levels(h, 65536, 32768, 4, OTSU) == want
    assert _without_int_wrap(monkeypatch, lambda: O.levels(h, 65536, 32768, 4, multi_otsu_opt=True)) != want


def _random_hist(rng, kind):
    if kind == "dense":
        h = rng.integers(0, 5000, 256)
    elif kind == "sparse":
        h = rng.integers(0, 5000, 256) * (rng.random(256) < 0.3)
    elif kind == "smooth":
        x = np.arange(256)
        h = (4000 * np.exp(-((x - rng.integers(0, 256)) / rng.integers(5, 80)) ** 2)).astype(np.int64)
        h += rng.integers(0, 3, 256)
    else:  # "image": the histogram of a small random mosaic
        img = rng.integers(0, 256, (8, 8, 3), dtype=np.uint8).repeat(8, 0).repeat(8, 1)
        h = O.hist256(O.gray(img))
    return h.astype(np.int64)


@pytest.mark.parametrize("kind", ["dense", "sparse", "smooth", "image"])
def test_library_levels_match_oracle_random(kind):
    rng = np.random.default_rng(1234 + len(kind))
    for it in range(150):
        h = _random_hist(rng, kind)
        depth = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 16, 64, 255, 256, 300]))
        try:
            want = [l.tup() for l in O.flex_levels(h, depth)]
        except ZeroDivisionError:
            continue
        if not want:
            with pytest.raises(msegment.MsegError):
                msegment.nc_levels(h, 100, 100, depth)
            continue
        got = msegment.nc_levels(h, 100, 100, depth)
        assert got == want, (kind, it, depth)
        for opt in (0, GISTO):
            assert np.array_equal(msegment.nc_marker_lut(got, opt), O.marker_lut(want, bool(opt)))


def test_library_multi_otsu_matches_oracle_random():
    rng = np.random.default_rng(77)
    seen = set()
    tries = 0
    while len(seen) < 3 or tries < 40:
        tries += 1
        assert tries < 2000
        # 1..3 separated plateaus -> k = 1..3 flex levels
        k = int(rng.integers(1, 4))
        h = np.zeros(256, np.int64)
        starts = np.sort(rng.choice(np.arange(2, 250, 12), k, replace=False))
        for s in starts:
            h[s: s + int(rng.integers(1, 8))] = int(rng.integers(1, 3000))
        lv = O.flex_levels(h, 2)
        if not 1 <= len(lv) <= 3:
            continue
        seen.add(len(lv))
        rows, cols = int(rng.integers(1, 200)), int(rng.integers(1, 200))
        want = O.levels(h, rows, cols, 2, multi_otsu_opt=True)
        got = msegment.nc_levels(h, rows, cols, 2, OTSU)
        assert got == want
        for opt in (0, GISTO):
            assert np.array_equal(msegment.nc_marker_lut(got, opt), O.marker_lut(want, bool(opt)))


def _bilateral_scalar(g, d):
    """Pixel-by-pixel restatement of bilateralFilter_8u (one channel) with fp32 scalars and
    OpenCV's borderInterpolate loop, written independently of the vectorised oracle."""
    import math

    f = np.float32
    H, W = g.shape
    sigma = 2.0 * d if d > 0 else 1.0
    r = d // 2 if d > 0 else int(round(1.5 * sigma))
    r = max(r, 1)
    cw = [f(math.exp(i * i * (-0.5 / (sigma * sigma)))) for i in range(256)]
    taps = [(i, j, f(math.exp(math.sqrt(i * i + j * j) ** 2 * (-0.5 / (sigma * sigma)))))
            for i in range(-r, r + 1) for j in range(-r, r + 1) if math.sqrt(i * i + j * j) <= r]

    def refl(p, n):
        while n > 1 and not 0 <= p < n:
            p = -p if p < 0 else 2 * n - 2 - p
        return 0 if n == 1 else p

    out = np.empty_like(g)
    for y in range(H):
        for x in range(W):
            v0 = int(g[y, x])
            ws = []
            for dy, dx, sw in taps:
                v = int(g[refl(y + dy, H), refl(x + dx, W)])
                w = f(cw[abs(v - v0)] * sw)
                ws.append((w, f(w * f(v))))
            s = f(0)
            t = f(0)
            n4 = len(ws) // 4 * 4
            for k in range(0, n4, 4):
                (w0, p0), (w1, p1), (w2, p2), (w3, p3) = ws[k:k + 4]
                t = f(t + f(f(w0 + w1) + f(w2 + w3)))
                s = f(s + f(f(p0 + p1) + f(p2 + p3)))
            for w, p in ws[n4:]:
                s = f(s + p)
                t = f(t + w)
            out[y, x] = int(np.rint(f(s / t)))
    return out


@pytest.mark.parametrize("d", [0, 1, 2, 3, 5, 8, 13])
def test_oracle_bilateral_matches_scalar_restatement(d):
    """The BILATERIAL pre-filter (PictureService.java:488-495): the vectorised oracle against a
    pixel loop, on noise (every tap weight in play) and on a frame smaller than the disc."""
    rng = np.random.default_rng(d)
    for shape in ((9, 13), (3, 2), (1, 5)):
        g = rng.integers(0, 256, shape, dtype=np.uint8)
        assert np.array_equal(O.bilateral(g, d), _bilateral_scalar(g, d)), shape


def test_oracle_bilateral_known_answers():
    # a flat plane is a fixed point; a step edge keeps its sides (colour weights at distance 200
    # are exp(-200^2 / 50) ~ 0); d <= 0 gives radius cvRound(1.5) = 2, a 13-tap disc
    assert np.array_equal(O.bilateral(np.full((6, 7), 93, np.uint8), 5), np.full((6, 7), 93, np.uint8))
    step = np.zeros((8, 8), np.uint8)
    step[:, 4:] = 200
    assert np.array_equal(O.bilateral(step, 5), step)
    radius, cw, taps = O.bilateral_tables(0)
    assert radius == 2 and len(taps) == 13 and cw[0] == 1.0
    radius, cw, taps = O.bilateral_tables(5)
    assert radius == 2 and len(taps) == 13 and cw.dtype == np.float32
    assert O.bilateral_tables(9)[0] == 4 and len(O.bilateral_tables(9)[2]) == 49
    # one bright pixel among dark ones is pulled only slightly (colour weight exp(-100^2/200))
    g = np.full((5, 5), 10, np.uint8)
    g[2, 2] = 110
    out = O.bilateral(g, 3)
    assert out[2, 2] == 110 and out[0, 0] == 10


def test_nc_option_flags():
    """AlgorithmOptions -> msg_nc_marker_stage bits (PictureService.java:469-495): MEDIAN_BLUR wins
    over BILATERIAL (if / else-if), the mask size rides in bits 8-15, a BILATERIAL size <= 0 acts
    as 0 (bilateralFilter: sigma <= 0 -> 1, radius 2), one above 255 is rejected."""
    from msegment.picture_service import nc_option_flags

    assert nc_option_flags((), 3) == 0
    assert nc_option_flags(("GISTO_DIAP", "MULTI_OTSU", "COLORED"), 3) == _lib.MSG_NC_GISTO_DIAP | OTSU
    assert nc_option_flags(("MEDIAN_BLUR", "BILATERIAL"), 5) == _lib.MSG_NC_MEDIAN_BLUR | _lib.MSG_NC_MASK(5)
    assert nc_option_flags(("BILATERIAL",), 9) == _lib.MSG_NC_BILATERAL | (9 << 8)
    assert nc_option_flags(("BILATERIAL",), -4) == _lib.MSG_NC_BILATERAL
    assert np.array_equal(O.bilateral_tables(-4)[2], O.bilateral_tables(0)[2])
    with pytest.raises(msegment.MsegError):
        nc_option_flags(("BILATERIAL",), 256)
    # MEDIAN_BLUR: medianBlur asserts ksize % 2 == 1 (C++ remainder: -1 % 2 == -1), so negative
    # and even sizes throw in the reference; 257 is a valid median there but does not fit the
    # option bits -- all rejected, none wrapped by the & 0xff packing (-1 -> 255, 257 -> 1)
    assert nc_option_flags(("MEDIAN_BLUR",), 1) == _lib.MSG_NC_MEDIAN_BLUR | (1 << 8)
    assert nc_option_flags(("MEDIAN_BLUR",), 255) == _lib.MSG_NC_MEDIAN_BLUR | (255 << 8)
    for k in (-1, -255, 0, 4, 256, 257):
        with pytest.raises(msegment.MsegError):
            nc_option_flags(("MEDIAN_BLUR",), k)
        with pytest.raises(msegment.MsegError):
            nc_option_flags(("MEDIAN_BLUR", "BILATERIAL"), k)
