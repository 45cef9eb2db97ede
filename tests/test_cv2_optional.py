"""Optional pinning of the oracles against a real OpenCV: skipped unless `cv2`
(>= 3.4) is importable -- it is not in this image, so parity stays "unpinned" here.  On a machine
that has it, these tests diff the CPU restatements (never the product) against OpenCV itself:
cv2.watershed (PictureService.java:909) and the SHAPE_METHOD operators (:404-452)."""
import numpy as np
import pytest

cv2 = pytest.importorskip("cv2")

from msegment import synth  # noqa: E402
from oracle import shape_oracle as so  # noqa: E402
from oracle import ws_oracle  # noqa: E402

FRAMES = [synth.frame(kind, h, w, s)[:2] for kind, h, w, s in
          [("mosaic", 64, 80, 1), ("mosaic_noise", 96, 64, 2), ("random", 40, 48, 3)]]


@pytest.mark.parametrize("k", range(len(FRAMES)))
def test_watershed_oracle_vs_cv2(k):
    img, m = FRAMES[k]
    want = m.copy()
    cv2.watershed(np.ascontiguousarray(img), want)
    assert np.array_equal(ws_oracle.watershed(img, m), want)


@pytest.mark.parametrize("k", range(len(FRAMES)))
def test_shape_operators_vs_cv2(k):
    img = FRAMES[k][0]
    g = cv2.cvtColor(img, cv2.COLOR_BGR2GRAY)
    assert np.array_equal(so.gray(img), g)
    for ks in (3, 5, 7):
        assert np.array_equal(so.median(g, ks), cv2.medianBlur(g, ks))
    assert np.array_equal(so.canny(g), cv2.Canny(g, 5, 50))
    mask = so.median(so.ring(so.canny(g)), 3)
    n, lab = cv2.connectedComponents(mask, connectivity=8, ltype=cv2.CV_32S)
    mine, nm = so.components(mask)
    assert nm == n - 1 and np.array_equal(mine, lab)
    res = cv2.findContours(mask.copy(), cv2.RETR_CCOMP, cv2.CHAIN_APPROX_NONE)
    contours = res[-2]
    assert so.contour_count(mask) == len(contours)
