"""CPU tests of the SHAPE_METHOD marker-stage oracle (oracle/shape_oracle.py): known answers
derived by hand from PictureService.shapeAutoMarkerWatershed (PictureService.java:395-466) and
from the documented OpenCV 3.4.2 operators it calls."""
import numpy as np
import pytest

from oracle import shape_oracle as so


@pytest.mark.parametrize("rows,cols,k", [
    (2, 5, 1), (3, 3, 5), (100, 300, 5), (101, 360, 3), (256, 256, 7), (360, 500, 9),
    (480, 640, 9), (720, 1280, 11), (1080, 1920, 11), (1081, 2000, 5), (4096, 4096, 21),
])
def test_blur_mask_size(rows, cols, k):
    # :877-899 -- min side, scale by range, (int) truncation, even -> +1
    assert so.blur_mask_size(rows, cols) == k


def test_median_replicate_border():
    g = np.array([[0, 0, 9], [0, 9, 9], [9, 9, 9]], np.uint8)
    m = so.median(g, 3)
    # corner (0,0): replicated window {0,0,0,0,0,9,0,0,9... } -> rows [0,0,0],[0,0,0],[0,0,9]
    assert m[0, 0] == 0
    assert m[2, 2] == 9
    assert m[1, 1] == 9  # window has five 9s
    assert np.array_equal(so.median(g, 1), g)


def test_canny_vertical_step():
    # cols 0-2 = 0, cols 3-5 = 100: dx = 400 at cols 2 and 3; NMS keeps col 2 only (m > left,
    # m >= right), and 400 > high -> every row of col 2 is an edge
    g = np.zeros((5, 6), np.uint8)
    g[:, 3:] = 100
    e = so.canny(g)
    want = np.zeros((5, 6), np.uint8)
    want[:, 2] = 255
    assert np.array_equal(e, want)


def test_canny_hysteresis_weak_chain():
    # a faint ramp (weak candidates) is kept only where it touches a strong edge
    g = np.zeros((9, 12), np.uint8)
    g[:, 6:] = 2          # dx = 8 at the step: weak (5 < 8 <= 50)
    cls = so.canny_classes(g)
    assert cls[:, 5].tolist() == [1] * 9 and cls.sum() == 9
    assert not so.canny(g).any()          # no strong pixel: nothing survives
    # hysteresis: a weak chain joined to a strong candidate through a diagonal step survives,
    # an isolated weak run does not
    cls = np.zeros((5, 6), np.uint8)
    cls[0:3, 1] = 1
    cls[3, 2] = 2
    cls[0:2, 4] = 1
    e = so.hysteresis(cls)
    assert e[0:3, 1].all() and e[3, 2] == 255 and not e[:, 4].any() and e.sum() == 4 * 255


def test_components_block_order():
    # raster order would number (0,3) first; the first 2x2 block of (1,0) comes first
    m = np.zeros((4, 6), np.uint8)
    m[1, 0] = 255
    m[0, 3] = 255
    lab, n = so.components(m)
    assert n == 2 and lab[1, 0] == 1 and lab[0, 3] == 2


def test_components_8_connected():
    m = np.zeros((4, 4), np.uint8)
    m[0, 0] = m[1, 1] = m[2, 2] = 1      # a diagonal chain is one component
    m[3, 0] = 1
    lab, n = so.components(m)
    assert n == 2 and lab[0, 0] == lab[2, 2] == 1 and lab[3, 0] == 2


@pytest.mark.parametrize("pattern,count", [
    (["00000", "01110", "01010", "01110", "00000"], 2),   # ring: outer + hole
    (["1001", "0000", "1001"], 4),                         # four dots
    (["11111", "10111", "11011", "11111"], 3),             # diagonal bg pixels: two 4-holes
    (["111", "101", "111"], 2),                            # touching the frame: padded outside
    (["000", "000"], 0),
])
def test_contour_count(pattern, count):
    m = np.array([[int(ch) for ch in row] for row in pattern], np.uint8) * 255
    assert so.contour_count(m) == count


def test_ring_is_dilation_difference():
    e = np.zeros((15, 15), np.uint8)
    e[7, 7] = 255
    r = so.ring(e)
    # dilate3 covers the 3x3 block, dilate5 of that the 7x7 block: ring = 7x7 minus 3x3
    want = np.zeros((15, 15), np.uint8)
    want[4:11, 4:11] = 255
    want[6:9, 6:9] = 0
    assert np.array_equal(r, want)


def test_shape_stages_mosaic():
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "opencv-msegment_amd"))
    from msegment import synth

    img, _, _ = synth.frame("mosaic", 96, 128, 5, cells=4)
    s = so.shape_stages(img)
    assert s["ksize"] == 5
    assert s["ncomp"] >= 1 and s["depth"] >= s["ncomp"]
    assert set(np.unique(s["mask"])) <= {0, 255}
    assert s["markers"].max() == s["ncomp"]
