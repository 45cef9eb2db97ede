"""Known answers for the COLOR_METHOD contour step (PictureService.java:356-364), worked out by hand.

findContours(RETR_CCOMP, CHAIN_APPROX_NONE) on the dilated peaks, then for every contour i
drawContours(markers, contours, i, i + 1, FILLED, 8, hierarchy, INT_MAX): contour i and its
hierarchy children filled together (even-odd), later contours overwriting earlier ones.  The
derivations below follow Suzuki-Abe border following as OpenCV 3.4 implements it:

  * the image is padded with a zero frame first (copyMakeBorder in cv::findContours), so a
    background region open to the image edge is never a hole;
  * outer borders are found at their first pixel in raster order, a hole border at the
    foreground pixel left of the hole's first pixel; RETR_CCOMP keeps two levels (every outer
    border is top level, even one lying inside another component's hole);
  * cvInsertNodeIntoTree prepends, so siblings are listed in reverse discovery order and the
    output is the depth-first walk (outer border, then its holes);
  * a hole border traced with 8-connectivity visits the foreground pixels 4-adjacent to the hole
    (corners are skipped by the diagonal steps), so filling a hole's polygon covers the hole,
    those pixels and anything inside the hole; filling an outer border together with its holes
    (even-odd) covers the component but not its holes' interiors.

The objects sit at columns >= 10 so that the circle((5,5), 3) stamp of :364 does not touch
them; the circle itself is checked separately.  These pin oracle/color_oracle.contour_markers;
the GPU stage is checked against that oracle in tests/test_gpu_color.py.
"""
import numpy as np
import pytest

from oracle import color_oracle

H, W = 12, 20


def _grid(rows):
    return np.array([[int(ch) for ch in r] for r in rows], dtype=np.int32)


def _pk(cells):
    pk = np.zeros((H, W), np.uint8)
    for (r0, r1, c0, c1) in cells:
        pk[r0:r1 + 1, c0:c1 + 1] = 1
    return pk


def _ring(r0, r1, c0, c1):
    return [(r0, r0, c0, c1), (r1, r1, c0, c1), (r0, r1, c0, c0), (r0, r1, c1, c1)]


# Case A: a ring (rows 2-6, cols 11-15) around a 3x3 hole.  Contours: [ring outer, hole].
# Contour 0 (outer + hole, even-odd) paints the ring 1; contour 1 (the hole) paints the hole and
# the ring pixels 4-adjacent to it 2.  The four corners are not on the hole border: they stay 1.
CASE_RING = (
    _ring(2, 6, 11, 15),
    ["0000000000",
     "0000000000",
     "0122210000",
     "0222220000",
     "0222220000",
     "0222220000",
     "0122210000",
     "0000000000",
     "0000000000",
     "0000000000",
     "0000000000",
     "0000000000"],
    2)

# Case B: a ring (rows 1-9, cols 10-18) with a 3x3 island (rows 4-6, cols 13-15) in its hole.
# Discovery: ring outer (row 1), ring hole (row 2), island (row 4).  Top level, reversed:
# [island, ring]; the walk: island 0, ring 1, hole 2.  Island -> 1, then ring + hole -> 2 (the
# island is outside that even-odd fill), then the hole's polygon -> 3 over the hole, its border
# pixels and the island.  Ring corners stay 2.
CASE_RING_ISLAND = (
    _ring(1, 9, 10, 18) + [(4, 6, 13, 15)],
    ["0000000000",
     "2333333320",
     "3333333330",
     "3333333330",
     "3333333330",
     "3333333330",
     "3333333330",
     "3333333330",
     "3333333330",
     "2333333320",
     "0000000000",
     "0000000000"],
    3)

# Case C: one block (rows 2-6, cols 10-16) with two one-pixel holes, (4,12) and (4,14), whose
# borders share the pixel (4,13).  Discovery: A = (4,12) then B = (4,14); children reversed:
# [block 0, B 1, A 2].  Block -> 1; B's diamond (4,14) + its 4 neighbours -> 2; A's diamond -> 3,
# which overwrites the shared pixel (4,13).
CASE_TWO_HOLES = (
    [(2, 6, 10, 16)],
    ["0000000000",
     "0000000000",
     "1111111000",
     "1131211000",
     "1333221000",
     "1131211000",
     "1111111000",
     "0000000000",
     "0000000000",
     "0000000000",
     "0000000000",
     "0000000000"],
    3)

# Case D: components touching the frame.  A thick U (legs cols 11-12 and 15-16, rows 0-5; bottom
# rows 4-5) whose bay (rows 0-3, cols 13-14) opens on the top edge: no hole (the zero frame
# reaches it).  A block in the bottom-right corner (rows 7-11, cols 16-19) with a one-pixel hole
# at (9,18).  Discovery: U (row 0), block (row 7); reversed: [block 0, its hole 1, U 2].
# Block -> 1; the hole's diamond (9,18), (8,18), (10,18), (9,17), (9,19) -> 2; U -> 3.
CASE_FRAME = (
    [(0, 5, 11, 12), (0, 5, 15, 16), (4, 5, 11, 16), (7, 11, 16, 19)],
    ["0330033000",
     "0330033000",
     "0330033000",
     "0330033000",
     "0333333000",
     "0333333000",
     "0000000000",
     "0000001111",
     "0000001121",
     "0000001222",
     "0000001121",
     "0000001111"],
    3)


def _holes(pk, cells):
    for (r, c) in cells:
        pk[r, c] = 0
    return pk


@pytest.mark.parametrize("case", ["ring", "ring_island", "two_holes", "frame"])
def test_contour_markers_known_answers(case):
    cells, rows, depth = {"ring": CASE_RING, "ring_island": CASE_RING_ISLAND,
                          "two_holes": CASE_TWO_HOLES, "frame": CASE_FRAME}[case]
    pk = _pk(cells)
    if case == "two_holes":
        pk = _holes(pk, [(4, 12), (4, 14)])
    if case == "frame":
        pk = _holes(pk, [(9, 18)])
    m, d = color_oracle.contour_markers(pk)
    assert d == depth
    np.testing.assert_array_equal(m[:, 10:], _grid(rows))
    # nothing is painted left of the objects except the circle stamp
    left = m[:, :10]
    assert set(np.unique(left).tolist()) <= {0, 255}


def test_circle_stamp_known_answer():
    """circle((5,5), 3, 255, FILLED) with LINE_8 runs cv::Circle's integer walk (drawing.cpp):
    err = 0, dx = 3, dy = 0, plus = 1, minus = 5; each step fills rows 5 -/+ dy over x 5 -/+ dx
    and rows 5 -/+ dx over x 5 -/+ dy, then dy += 1, err += plus, plus += 2,
    mask = (err <= 0) - 1, err -= minus & mask, dx += mask, minus -= mask & 2.  By hand:
    (dx, dy) = (3, 0): row 5 x 2-8, rows 2 and 8 x 5;  -> err -4, dx 2, minus 3
    (dx, dy) = (2, 1): rows 4 and 6 x 3-7, rows 3 and 7 x 4-6;  -> err -1, dx 2
    (dx, dy) = (2, 2): rows 3 and 7 x 3-7 (twice);  -> dx 1 < dy 3, done."""
    m, d = color_oracle.contour_markers(np.zeros((H, W), np.uint8))
    assert d == 0
    want = np.zeros((H, W), np.int32)
    for y, (x0, x1) in {2: (5, 5), 3: (3, 7), 4: (3, 7), 5: (2, 8), 6: (3, 7), 7: (3, 7), 8: (5, 5)}.items():
        want[y, x0:x1 + 1] = 255
    np.testing.assert_array_equal(m, want)
