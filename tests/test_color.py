"""CPU known answers for the COLOR_METHOD marker-stage oracle (oracle/color_oracle.py,
oracle/ws_oracle.c: oracle_chamfer5), each derived by hand from the OpenCV 3.4.2 routine the
step restates (PictureService.java:301-366).  Unpinned against a real OpenCV build."""
import numpy as np

from oracle import color_oracle as C
from oracle import ws_oracle


def test_sharpen_is_a_column_kernel_with_reflect101():
    # one channel pattern down a single column: 9 s(y) - sum of the 8 vertical neighbours
    col = np.array([10, 20, 30, 40, 50, 60, 70, 80, 90, 100], np.int64)
    img = np.zeros((10, 3, 3), np.uint8)
    img[:, 1, 0] = col
    out = C.sharpen(img)
    refl = lambda p: C._reflect101(p, 10)  # noqa: E731
    for y in range(10):
        want = 9 * col[y] - sum(col[refl(y + k)] for k in (-4, -3, -2, -1, 1, 2, 3, 4))
        assert out[y, 1, 0] == min(255, max(0, want))
    assert not out[:, [0, 2]].any()  # no horizontal taps
    assert C._reflect101(-1, 10) == 1 and C._reflect101(10, 10) == 8 and C._reflect101(-4, 2) == 0


def _java_check_pixel_rgb(px, r, g, b):
    """PixelUtil.checkPixelRGB (PixelUtil.java:19): Java's byte is signed, so a channel of 0xFF
    reads -1 and is compared, widened to int, with the int literal 255."""
    sb = np.asarray(px, np.uint8).astype(np.int8).astype(np.int64)
    return bool(sb[0] == r and sb[1] == g and sb[2] == b)


def test_white_to_black_loop_is_a_no_op_in_java():
    # PictureService.java:309-318 calls checkPixelRGB(vec3b, 255, 255, 255): never true
    assert not _java_check_pixel_rgb((255, 255, 255), 255, 255, 255)
    assert _java_check_pixel_rgb((255, 255, 255), -1, -1, -1)  # what it would have needed
    assert _java_check_pixel_rgb((0, 7, 127), 0, 7, 127)  # bytes below 0x80 compare as expected
    # so an all-white frame keeps its white pixels: 9*255 - 8*255 = 255 in every channel
    img = np.full((5, 5, 3), 255, np.uint8)
    assert (C.sharpen(img) == 255).all()
    # and a white pixel in a dark column is sharpened as white (not as black)
    img = np.zeros((9, 1, 3), np.uint8)
    img[4, 0] = 255
    out = C.sharpen(img)
    assert (out[4, 0] == 255).all() and not out[[0, 1, 2, 3, 5, 6, 7, 8], 0].any()


def test_otsu_first_maximum():
    g = np.zeros((4, 8), np.uint8)
    g[:, 4:] = 200
    assert C.otsu(g) == 0.0  # every split in [0, 199] is equally good: the first wins
    g2 = np.array([[10, 10, 10, 50, 50, 90, 90, 90]], np.uint8)
    assert C.otsu(g2) in (10.0, 50.0)
    assert C.otsu(np.full((3, 3), 7, np.uint8)) == 0.0  # one class: no split


def test_chamfer5_weights():
    bw = np.full((9, 9), 255, np.uint8)
    bw[4, 4] = 0
    d = ws_oracle.chamfer5(bw)
    assert d[4, 4] == 0 and d[4, 5] == 65536 and d[5, 5] == 91750 and d[5, 6] == 143976
    assert d[4, 6] == 2 * 65536 and d[6, 6] == 2 * 91750 and d[6, 7] == 143976 + 91750
    assert (d == d[::-1, ::-1]).all() and (d == d.T).all()


def test_circle_spans_of_radius_3():
    assert C.circle_spans(5, 5, 3) == {5: (2, 8), 4: (3, 7), 6: (3, 7), 3: (3, 7), 7: (3, 7), 2: (5, 5), 8: (5, 5)}


def test_contour_order_reverse_discovery():
    pk = np.zeros((20, 30), np.uint8)
    pk[12:16, 2:6] = 1   # discovered second (lower)
    pk[3:6, 20:25] = 1   # discovered first
    m, depth = C.contour_markers(pk)
    assert depth == 2
    assert (m[12:16, 2:6] == 1).all() and (m[3:6, 20:25] == 2).all()
    assert m[0, 0] == 0 and m[5, 5] == 255  # the circle((5,5), 3, 255)


def test_contour_hole_drawn_after_its_component():
    pk = np.zeros((30, 30), np.uint8)
    pk[10:20, 10:20] = 1
    pk[13:17, 13:17] = 0  # a hole
    m, depth = C.contour_markers(pk)
    assert depth == 2  # component + hole
    assert m[10, 10] == 1 and m[15, 15] == 2
    assert m[12, 15] == 2 and m[13, 12] == 2  # hole border pixels (4-adjacent) carry the hole
    assert m[12, 12] == 1  # diagonal only: not on the hole's border
