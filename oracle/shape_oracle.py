"""CPU restatement of the SHAPE_METHOD marker stage -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module; the
product (libmsegment: shape_kernels.hip) never does.

Follows PictureService.shapeAutoMarkerWatershed in the reference
(src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java:395-466) step by step.
The Java glue is in-tree; the image operators are OpenCV 3.4.2 ([ext], pom.xml:38-43), restated
from their documented algorithms (numpy + scipy.ndimage as independent tools):

  blur_mask_size()   calculateSizeOfSquareBlurMask                      :877-899
  gray()             cvtColor(src, srcGray, COLOR_BGR2GRAY)             :404-405
  median()           medianBlur(srcGray, srcGray, k): exact k x k median, BORDER_REPLICATE  :408
  canny()            Canny(brdGray, brdGray, 5, 50): 3x3 Sobel (BORDER_REPLICATE), L1
                     magnitude, non-maximum suppression with OpenCV's tan(22.5)/tan(67.5)
                     fixed-point sectors (CANNY_SHIFT 15), hysteresis = candidates 8-connected
                     to a candidate above the high threshold                :415-416
  ring()             dilate 3x3 -> dilate 5x5 -> subtract (saturating)     :426-429
                     (dilation ignores the outside: morphologyDefaultBorderValue)
  median(.., 3)      medianBlur(markerMask, markerMask, 3)                  :435
  components()       connectedComponents(markerMask, markers, 8, CV_32S): 8-connected
                     components of the non-zero pixels, numbered 1.. in the order of the first
                     2x2 block (block-raster order) that holds one of their pixels -- the order
                     in which OpenCV's default 8-way labeller (BBDT, Grana et al.) creates the
                     smallest provisional label of each component          :441
  contour_count()    findContours(markerMask, RETR_CCOMP).size(): one outer border per
                     8-connected component + one hole border per 4-connected background
                     component that does not touch the (zero-padded) image border  :447-452
  shape_markers()    the whole stage: (markers int32, depth = contour count); depth 0 means
                     the reference returns null (no contours)               :448-451

Parity status: the Java glue is pinned by reading it; every OpenCV operator is restated from
its documented algorithm and is UNPINNED against a real OpenCV 3.4.2 build (none exists in this
image; an IPP-enabled build could differ in Canny).  GPU parity is bit-exact against this file.
"""
import numpy as np
from scipy import ndimage

CANNY_SHIFT = 15
TG22 = int(0.4142135623730950488016887242097 * (1 << CANNY_SHIFT) + 0.5)  # 13573


def blur_mask_size(rows, cols):
    """calculateSizeOfSquareBlurMask (PictureService.java:877-899), Java int/double semantics."""
    m = cols if cols <= rows else rows
    if m < 3:
        return 1
    if m <= 100:
        return 5
    if m <= 360:
        scale = 0.025
    elif m <= 480:
        scale = 0.02
    elif m <= 720:
        scale = 0.015
    elif m <= 1080:
        scale = 0.01
    else:
        scale = 0.005
    r = int(m * scale)  # Double.intValue(): truncation toward zero
    return r + 1 if r % 2 == 0 else r


def gray(bgr):
    b = bgr[..., 0].astype(np.uint32)
    g = bgr[..., 1].astype(np.uint32)
    r = bgr[..., 2].astype(np.uint32)
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def median(img, k):
    """medianBlur: exact median of the k x k window, BORDER_REPLICATE (k = 1: copy)."""
    img = np.asarray(img, dtype=np.uint8)
    if k <= 1:
        return img.copy()
    return ndimage.median_filter(img, size=k, mode="nearest")


def sobel(g):
    """3x3 Sobel dx, dy (CV_16S), BORDER_REPLICATE."""
    p = np.pad(g.astype(np.int32), 1, mode="edge")
    H, W = g.shape
    s = lambda dr, dc: p[1 + dr:1 + dr + H, 1 + dc:1 + dc + W]  # noqa: E731
    dx = (s(-1, 1) - s(-1, -1)) + 2 * (s(0, 1) - s(0, -1)) + (s(1, 1) - s(1, -1))
    dy = (s(1, -1) - s(-1, -1)) + 2 * (s(1, 0) - s(-1, 0)) + (s(1, 1) - s(-1, 1))
    return dx, dy


def canny_classes(g, low=5, high=50):
    """Per pixel: 0 not a candidate, 1 candidate (passed NMS, m > low), 2 candidate with
    m > high.  Magnitudes outside the frame are 0 (OpenCV's zeroed magnitude border)."""
    dx, dy = sobel(g)
    mag = np.abs(dx) + np.abs(dy)
    H, W = g.shape
    mp = np.zeros((H + 2, W + 2), np.int64)
    mp[1:-1, 1:-1] = mag
    M = lambda dr, dc: mp[1 + dr:1 + dr + H, 1 + dc:1 + dc + W]  # noqa: E731
    m = mag.astype(np.int64)
    xs = np.abs(dx).astype(np.int64)
    ys = np.abs(dy).astype(np.int64)
    x = xs * TG22
    y = ys << CANNY_SHIFT
    horiz = y < x
    tg67 = x + (xs << (CANNY_SHIFT + 1))
    vert = (~horiz) & (y > tg67)
    diag = (~horiz) & (~vert)
    same = (dx ^ dy) >= 0  # s = +1: up-left / down-right; s = -1: up-right / down-left
    keep_h = (m > M(0, -1)) & (m >= M(0, 1))
    keep_v = (m > M(-1, 0)) & (m >= M(1, 0))
    keep_d = np.where(same, (m > M(-1, -1)) & (m > M(1, 1)), (m > M(-1, 1)) & (m > M(1, -1)))
    keep = (m > low) & ((horiz & keep_h) | (vert & keep_v) | (diag & keep_d))
    out = np.zeros((H, W), np.uint8)
    out[keep] = 1
    out[keep & (m > high)] = 2
    return out


def hysteresis(cls):
    """255 where a candidate is 8-connected (through candidates) to a strong candidate."""
    lab, n = ndimage.label(cls > 0, structure=np.ones((3, 3), bool))
    strong = np.zeros(n + 1, bool)
    strong[np.unique(lab[cls == 2])] = True
    strong[0] = False
    return np.where(strong[lab], 255, 0).astype(np.uint8)


def canny(g, low=5, high=50):
    return hysteresis(canny_classes(g, low, high))


def dilate(img, k):
    """dilate with a k x k rectangle; the outside never wins (non-negative images)."""
    return ndimage.maximum_filter(np.asarray(img, np.uint8), size=k, mode="constant", cval=0)


def ring(edges):
    d3 = dilate(edges, 3)
    d5 = dilate(d3, 5)
    return np.clip(d5.astype(np.int32) - d3.astype(np.int32), 0, 255).astype(np.uint8)


def components(mask):
    """connectedComponents(mask, 8, CV_32S) with OpenCV's numbering (first 2x2 block)."""
    fg = np.asarray(mask) != 0
    lab, n = ndimage.label(fg, structure=np.ones((3, 3), bool))
    out = np.zeros(fg.shape, np.int32)
    if n == 0:
        return out, 0
    H, W = fg.shape
    r, c = np.nonzero(fg)
    bkey = (r >> 1).astype(np.int64) * ((W + 1) >> 1) + (c >> 1)
    first = np.full(n + 1, np.iinfo(np.int64).max, np.int64)
    np.minimum.at(first, lab[r, c], bkey)
    order = np.argsort(first[1:], kind="stable")  # component ids sorted by first block
    newid = np.zeros(n + 1, np.int32)
    newid[order + 1] = np.arange(1, n + 1, dtype=np.int32)
    out[r, c] = newid[lab[r, c]]
    return out, n


def contour_count(mask):
    """findContours(mask, RETR_CCOMP, CHAIN_APPROX_NONE).size() on a zero-padded copy."""
    fg = np.asarray(mask) != 0
    _, nfg = ndimage.label(fg, structure=np.ones((3, 3), bool))
    bg = ~np.pad(fg, 1, constant_values=False)
    blab, nbg = ndimage.label(bg, structure=ndimage.generate_binary_structure(2, 1))
    return nfg + (nbg - 1)


def shape_stages(bgr, ksize=None):
    """Every intermediate of the stage: dict of gray, blur, edges, mask, markers, ncomp, depth."""
    bgr = np.asarray(bgr, np.uint8)
    H, W = bgr.shape[:2]
    k = blur_mask_size(H, W) if ksize is None else ksize
    g = gray(bgr)
    b = median(g, k)
    e = canny(b)
    mask = median(ring(e), 3)
    mk, n = components(mask)
    return {"ksize": k, "gray": g, "blur": b, "edges": e, "mask": mask, "markers": mk, "ncomp": n,
            "depth": contour_count(mask)}


def shape_markers(bgr, ksize=None):
    s = shape_stages(bgr, ksize)
    return s["markers"], s["depth"]
