"""CPU oracle of the COLOR_METHOD marker stage -- TEST INFRASTRUCTURE ONLY.

PictureService.colorAutoMarkerWatershed (PictureService.java:301-392), the caller that builds the
flood's seeds for the colour method, restated step by step from OpenCV 3.4.2's documented
algorithms (OpenCV is an un-vendored Maven dependency, pom.xml:38-43: nothing here is pinned
against a real OpenCV build -- "parity unpinned"):

  :308-318  the "white -> black" loop is a NO-OP in Java: PixelUtil.checkPixelRGB
            (PixelUtil.java:19) compares the signed byte of each channel (0xFF reads -1) with
            int 255, which is never equal -- white pixels stay white
  :323-333  filter2D(src, CV_32F, MatOfFloat(1,1,1,1,-8,1,1,1,1)) -- a 9x1 COLUMN kernel,
            BORDER_REFLECT_101 -- then src - laplacian, saturated to CV_8UC3: exact integers,
            res = clamp(9 s(y) - sum_{0<|k|<=4} s(y+k), 0, 255) per channel; the result
            REPLACES src (it is what the watershed floods, :379)
  :338/938  bw = threshold(BGR2GRAY(src), 40, 255, BINARY | OTSU): Otsu's threshold in double
            arithmetic (getThreshVal_Otsu_8u), gray > t -> 255
  :343/1018 distanceTransform(bw, DIST_L2, 5) (oracle/ws_oracle.c: oracle_chamfer5) and
            normalize(0, 1, NORM_MINMAX) in float
  :348-350  threshold(0.4, 1.0, BINARY) on the float image, dilate 3x3 (ones)
  :356-364  findContours(RETR_CCOMP, CHAIN_APPROX_NONE) + drawContours(i, i + 1, FILLED, 8,
            hierarchy, INT_MAX) + circle((5,5), 3, 255, FILLED); depth = contours.size()

The contour step is restated through connected components (the part an OpenCV build could
disagree with): outer borders = 8-connected foreground components, holes = 4-connected
background components not touching the frame.  Suzuki's raster scan discovers a component at its
first pixel and a hole at the pixel left of its first pixel; cvInsertNodeIntoTree prepends, so
siblings come out in reverse discovery order, and the list is the depth-first walk (outer
contour, then its holes).  Filling contour i (its holes by the even-odd rule) covers the
component and the border pixels of its holes; a hole's own fill covers the hole and its border
pixels (foreground pixels 4-adjacent to it) and whatever it encloses; later contours overwrite.
"""
import numpy as np
from scipy import ndimage

from oracle import nc_oracle, ws_oracle


def _reflect101(p, n):
    if n == 1:
        return 0
    while p < 0 or p >= n:
        p = -p if p < 0 else 2 * n - 2 - p
    return p


def sharpen(bgr):
    """:323-333: src - filter2D(9x1 Laplacian), saturated (white pixels kept: :309-318 is a no-op)."""
    s = np.asarray(bgr, dtype=np.int64).copy()
    H = s.shape[0]
    acc = 9 * s
    for k in (-4, -3, -2, -1, 1, 2, 3, 4):
        idx = np.array([_reflect101(y + k, H) for y in range(H)], dtype=np.int64)
        acc = acc - s[idx]
    return np.clip(acc, 0, 255).astype(np.uint8)


def otsu(gray):
    """OpenCV getThreshVal_Otsu_8u: the first threshold of maximal between-class variance."""
    h = np.bincount(np.asarray(gray, dtype=np.uint8).ravel(), minlength=256).astype(np.int64)
    n = int(h.sum())
    scale = 1.0 / n
    mu = 0.0
    for i in range(256):
        mu += i * float(h[i])
    mu *= scale
    mu1 = 0.0
    q1 = 0.0
    max_sigma = 0.0
    max_val = 0.0
    eps = float(np.finfo(np.float32).eps)
    for i in range(256):
        p_i = float(h[i]) * scale
        mu1 *= q1
        q1 += p_i
        q2 = 1.0 - q1
        if min(q1, q2) < eps or max(q1, q2) > 1.0 - eps:
            continue
        mu1 = (mu1 + i * p_i) / q1
        mu2 = (mu - q1 * mu1) / q2
        sigma = q1 * q2 * (mu1 - mu2) * (mu1 - mu2)
        if sigma > max_sigma:
            max_sigma = sigma
            max_val = float(i)
    return max_val


def peaks(bw):
    """:343-353: chamfer distance, min-max normalised in float, > 0.4, dilate 3x3 -> 0/1."""
    t0 = ws_oracle.chamfer5(bw)
    d = t0.astype(np.float32) * np.float32(1.0 / 65536)
    lo, hi = float(d.min()), float(d.max())
    if hi - lo > np.finfo(np.float64).eps:
        sc = 1.0 / (hi - lo)
        v = d * np.float32(sc)
        if lo != 0.0:
            v = v + np.float32(-lo * sc)
    else:
        v = np.zeros_like(d)
    th = (v > np.float32(0.4)).astype(np.uint8)
    return ndimage.maximum_filter(th, size=3, mode="constant", cval=0)


def circle_spans(cx, cy, r):
    """cv::circle(FILLED, LINE_8) spans: OpenCV's integer circle walk, {row: (x0, x1)}."""
    spans = {}

    def hline(y, x0, x1):
        a, b = spans.get(y, (x0, x1))
        spans[y] = (min(a, x0), max(b, x1))

    err, dx, dy, plus, minus = 0, r, 0, 1, (r << 1) - 1
    while dx >= dy:
        hline(cy - dy, cx - dx, cx + dx)
        hline(cy + dy, cx - dx, cx + dx)
        hline(cy - dx, cx - dy, cx + dy)
        hline(cy + dx, cx - dy, cx + dy)
        dy += 1
        err += plus
        plus += 2
        mask = (1 if err <= 0 else 0) - 1
        err -= minus & mask
        dx += mask
        minus -= mask & 2
    return spans


def contour_markers(pk):
    """:356-364 restated through components (module docstring); returns (markers, depth)."""
    pk = np.asarray(pk, dtype=np.uint8)
    H, W = pk.shape
    fg = pk != 0
    comp, nc = ndimage.label(fg, structure=np.ones((3, 3), int))
    bgl, nb = ndimage.label(~fg, structure=[[0, 1, 0], [1, 1, 1], [0, 1, 0]])
    flat = np.arange(H * W).reshape(H, W)
    first_c = ndimage.minimum(flat, comp, index=np.arange(1, nc + 1)) if nc else []
    first_b = ndimage.minimum(flat, bgl, index=np.arange(1, nb + 1)) if nb else []
    border = set(np.unique(np.concatenate([bgl[0], bgl[-1], bgl[:, 0], bgl[:, -1]])).tolist()) - {0}
    holes = [b + 1 for b in range(nb) if (b + 1) not in border]
    # discovery keys and parents
    ckey = {c + 1: int(first_c[c]) for c in range(nc)}
    hkey = {h: int(first_b[h - 1]) - 1 for h in holes}
    hpar = {h: int(comp.flat[int(first_b[h - 1]) - 1]) for h in holes}
    kids = {}
    for h in holes:
        kids.setdefault(hpar[h], []).append(h)
    order = []
    for c in sorted(ckey, key=lambda c: -ckey[c]):
        order.append(("c", c))
        for h in sorted(kids.get(c, []), key=lambda h: -hkey[h]):
            order.append(("h", h))
    idx = {o: i for i, o in enumerate(order)}
    # the hole enclosing each component: the background region left of its first pixel
    enc_hole = {}
    for c in ckey:
        f = ckey[c]
        b = int(bgl.flat[f - 1]) if f % W else 0
        enc_hole[c] = b if b in hpar else 0

    memo = {}

    def enc(c):  # highest index among the holes enclosing component c (transitively), -1 none
        if c in memo:
            return memo[c]
        h = enc_hole[c]
        v = -1 if h == 0 else max(idx[("h", h)], enc(hpar[h]))
        memo[c] = v
        return v

    lab_c = np.zeros(nc + 1, np.int64)
    for c in ckey:
        lab_c[c] = 1 + max(idx[("c", c)], enc(c))
    lab_hfill = np.zeros(nb + 1, np.int64)
    lab_hbord = np.zeros(nb + 1, np.int64)
    for h in holes:
        lab_hfill[h] = 1 + max(idx[("h", h)], enc(hpar[h]))
        lab_hbord[h] = 1 + idx[("h", h)]
    m = np.where(fg, lab_c[comp], lab_hfill[bgl])
    # foreground pixels 4-adjacent to a hole carry that hole's fill too
    hb = np.where(fg, 0, lab_hbord[bgl])
    up = np.zeros_like(hb)
    up[1:] = np.maximum(up[1:], hb[:-1])
    up[:-1] = np.maximum(up[:-1], hb[1:])
    up[:, 1:] = np.maximum(up[:, 1:], hb[:, :-1])
    up[:, :-1] = np.maximum(up[:, :-1], hb[:, 1:])
    m = np.where(fg, np.maximum(m, up), m)
    for y, (x0, x1) in circle_spans(5, 5, 3).items():
        if 0 <= y < H:
            a, b = max(0, x0), min(W - 1, x1)
            if a <= b:
                m[y, a:b + 1] = 255
    return m.astype(np.int32), len(order)


def stages(bgr):
    """Every intermediate: sharp (the flood's src), gray, otsu, bw, peaks, markers, depth."""
    sh = sharpen(bgr)
    g = nc_oracle.gray(sh)
    t = otsu(g)
    bw = np.where(g > t, 255, 0).astype(np.uint8)
    pk = peaks(bw)
    mk, depth = contour_markers(pk)
    return {"sharp": sh, "gray": g, "otsu": t, "bw": bw, "peaks": pk, "markers": mk, "depth": depth}


def color_markers(bgr):
    s = stages(bgr)
    return s["sharp"], s["markers"], s["depth"]
