"""CPU restatement of the NOT_CONNECTED_MARKERS marker stage -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module; the
product (libmsegment: nc_kernels.hip + nc_levels.cpp) never does.

Follows PictureService.notConnectedMarkers in the reference
(src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java), statement by
statement, in plain Python with Java's semantics made explicit:

  gray()             cvtColor(src, COLOR_BGR2GRAY)                        :476-478
                     OpenCV 3.4.2's 8-bit fixed point (yuv_shift 14; the non-IPP path)
  hist256()          calcHist(srcGray, 256 bins, [0, 256)) read back with (int) from CV_32F :565
  flex_levels()      "Collecting ranges"                                   :574-640
  multi_otsu()       the MULTI_OTSU override + otsuPart                   :650-722, :945-996
  marker_lut()       "ALLOCATE TO LAYERS" + the marker-map sum            :781-828
  markers()          lut[gray]
  bilateral()        the BILATERIAL pre-filter bilateralFilter(srcGray, d, 2d, 2d)  :488-495
                     (OpenCV 3.4.2 bilateralFilter_8u, non-IPP, fp32; parity unpinned)

Parity status: the level logic and the marker allocation are in-tree Java (pinned by reading
it: the known-answer tests in tests/test_nc.py are derived by hand from those lines); the gray
conversion is OpenCV's documented fixed-point formula, unpinned against a real OpenCV build
(none exists in this image; an IPP-enabled OpenCV may round differently).
"""
import numpy as np


def _i32(x):
    """Java int wrap-around."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def _f32_int(x):
    """(int) of a value stored in a CV_32F Mat."""
    return int(np.float32(x))


def gray(bgr):
    b = bgr[..., 0].astype(np.uint32)
    g = bgr[..., 1].astype(np.uint32)
    r = bgr[..., 2].astype(np.uint32)
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def hist256(gray_img):
    return np.bincount(np.asarray(gray_img).reshape(-1), minlength=256).astype(np.int64)


class BrightLevel:
    """model/BrightLevel.java"""

    def __init__(self, start, end, count):
        self.start, self.end, self.count = start, end, count

    def clone(self):
        return BrightLevel(self.start, self.end, self.count)

    def mean_level(self):
        if self.start == self.end:
            return self.start
        rng = self.end - self.start
        if rng == 1:
            return self.start
        return self.start + int(rng / 2)  # Java int division truncates toward zero

    def mean_diap(self, rng):
        diam = self.end - self.start
        if diam <= rng * 2:
            return BrightLevel(self.start, self.end, self.count)
        mean = self.mean_level()
        s = mean - rng + 1 if mean - rng < self.start else mean - rng
        e = mean + rng - 1 if mean + rng > self.end else mean + rng
        return BrightLevel(s, e, e - s + 1)

    def tup(self):
        return (self.start, self.end, self.count)


def _mean_i(values):
    """MathUtil.meanI: Double mean, .intValue()."""
    if not values:
        return 0  # NaN.intValue()
    m = 0.0
    for v in values:
        m += float(v)
    return int(m / len(values))


def flex_levels(hist, depth):
    """PictureService.java:574-640 on the (int) histogram values."""
    h = [_f32_int(v) for v in hist]
    block_limit = 256 // depth
    f = []
    block = [h[0]]
    temp = BrightLevel(0, 0, h[0])
    for i in range(1, 256):
        prev, curr = h[i - 1], h[i]
        if curr == 0:
            if prev != 0:
                temp.end = i - 1
                f.append(temp.clone())
            temp = BrightLevel(i, i, curr)
            block = []
            continue
        if prev == 0:
            temp = BrightLevel(i, i, curr)
        with_cur = list(block) + [curr]
        coeff = 0.5
        old_mean = curr if not block else _mean_i(block)
        new_mean = _mean_i(with_cur)
        min_t = old_mean - old_mean * coeff
        max_t = old_mean + old_mean * coeff
        if min_t <= new_mean <= max_t:
            if len(block) >= block_limit:
                temp.end = i - 1
                f.append(temp.clone())
                temp = BrightLevel(i, i, curr)
                block = [curr]
                continue
            block.append(curr)
            temp.count = _i32(temp.count + curr)
            continue
        temp.end = i - 1
        f.append(temp.clone())
        temp = BrightLevel(i, i, curr)
        block = [curr]
    return f


def _otsu_part(k, wk, mk, m, mt, pixnum, hsize, hist, start, step):
    """otsuPart, PictureService.java:945-996 -> (maxVar, idxMaxVar, deepers)."""
    if step >= k:
        return None
    max_var = 0.0
    max_idx = start
    max_deep_idx = 0
    max_deepers = []
    for ii in range(start, hsize):
        intensity = hist[ii]
        wk[step] += intensity / float(pixnum)
        mk[step] += _i32(ii * intensity) / float(pixnum)
        m[step] = mk[step] / wk[step] if wk[step] != 0.0 else (
            float("nan") if mk[step] == 0.0 else float("inf") * (1 if mk[step] > 0 else -1))
        if step > 0:
            wks = 0.0
            mks = 0.0
            for q in range(step + 1):
                wks += wk[q]
                mks += mk[q]
            wk[step + 1] = 1 - wks
            mk[step + 1] = mt - mks
        if step == k - 1:
            var = 0.0
            for q in range(step + 1):
                var += wk[q] * (m[q] - mt) * (m[q] - mt)
            if max_var < var:
                max_var = var
                max_idx = ii
        else:
            d = _otsu_part(k, wk, mk, m, mt, pixnum, hsize, hist, ii + 1, step + 1)
            if d[0] > max_var:
                max_idx = ii
                max_var = d[0]
                max_deep_idx = d[1]
                max_deepers = d[2]
    if step == k - 1:
        return (max_var, max_idx, [])
    max_deepers = list(max_deepers) + [max_deep_idx]
    return (max_var, max_idx, max_deepers)


def multi_otsu(hist, rows, cols, levels):
    """PictureService.java:650-722: the override levels."""
    h = [_f32_int(v) for v in hist]
    reduced = [_f32_int(h[i] + h[i + 1]) for i in range(0, 256, 2)]
    k = len(levels)
    if k == 0:
        raise ValueError("otsuPart returns null (NullPointerException in the reference)")
    pixnum = _i32(rows * cols)
    mt = 0.0
    for i in range(128):
        mt += i * (reduced[i] / float(pixnum))
    wk = [0.0] * (k + 1)
    mk = [0.0] * (k + 1)
    m = [0.0] * (k + 1)
    r = _otsu_part(k, wk, mk, m, mt, pixnum, 128, reduced, 0, 0)
    th = list(r[2]) + [r[1]]
    th.sort()
    th = [255 if t * (256 // 128) >= 256 else t * (256 // 128) for t in th]
    ov = []
    begin = 0
    for t in th:
        ov.append(BrightLevel(begin, t - 1, 0))
        begin = t
    ov[-1].end = 255
    for i in range(256):
        for o in ov:
            if o.start <= i <= o.end:
                o.count = _i32(o.count + h[i])
    return ov


def levels(hist, rows, cols, depth, gisto_diap=False, multi_otsu_opt=False):
    lv = flex_levels(hist, depth)
    if multi_otsu_opt:
        lv = multi_otsu(hist, rows, cols, lv)
    if not lv:
        raise ValueError("no brightness level (NoSuchElementException in the reference)")
    return [l.tup() for l in lv]


def marker_lut(levels_, gisto_diap=False):
    lv = [BrightLevel(*t) for t in levels_]
    lut = np.zeros(256, dtype=np.int32)
    for b in range(256):
        for idx, l in enumerate(lv, start=1):
            if gisto_diap:
                d = l.mean_diap(3)
                if d.start <= b <= d.end:
                    lut[b] = idx
                    break
            elif b == l.mean_level():
                lut[b] = idx
                break
    return lut


def markers(gray_img, lut):
    return lut[np.asarray(gray_img)].astype(np.int32)


def _reflect101(p, n):
    """borderInterpolate(p, n, BORDER_REFLECT_101), the loop form (borders wider than the
    frame fold again)."""
    if 0 <= p < n:
        return p
    if n == 1:
        return 0
    while not 0 <= p < n:
        p = -p if p < 0 else 2 * n - 2 - p
    return p


def bilateral_tables(d):
    """bilateralFilter_8u's set-up for bilateralFilter(srcGray, dst, d, 2d, 2d) (the BILATERIAL
    branch, PictureService.java:488-490; OpenCV 3.4.2 imgproc bilateralFilter_8u): sigmas <= 0
    become 1, radius = d / 2 (d <= 0: cvRound(1.5 sigma_space)), at least 1; the colour table
    (float)exp(i*i*c) and the disc of taps (dy, dx, (float)exp(r*r*s)) with r = sqrt(dy^2 + dx^2)
    <= radius, row-major.  Returns (radius, colour weights f32[256], [(dy, dx, f32 weight)])."""
    import math

    sc = ss = float(2 * int(d))
    if sc <= 0:
        sc = ss = 1.0
    gcc = -0.5 / (sc * sc)
    gsc = -0.5 / (ss * ss)
    radius = int(d) // 2 if d > 0 else int(np.rint(ss * 1.5))
    radius = max(radius, 1)
    cw = np.array([np.float32(math.exp((i * i) * gcc)) for i in range(256)], np.float32)
    taps = []
    for i in range(-radius, radius + 1):
        for j in range(-radius, radius + 1):
            r = math.sqrt(float(i) * i + float(j) * j)
            if r > radius:
                continue
            taps.append((i, j, np.float32(math.exp(r * r * gsc))))
    return radius, cw, taps


def bilateral(g, d):
    """bilateralFilter(srcGray, dst, d, 2d, 2d) on an 8-bit gray plane, BORDER_REFLECT_101, in
    fp32 as OpenCV 3.4.2's non-IPP x86 path computes it: taps in groups of four, each group's
    weights w = colour[|v - v0|] * space and products w * v summed pairwise ((0+1)+(2+3), the
    SSE3 horizontal adds) into the running sums, the last maxk % 4 taps added one at a time;
    dst = cvRound(sum / wsum).  Parity unpinned: an IPP-enabled OpenCV runs IPP's own filter."""
    g = np.asarray(g, np.uint8)
    H, W = g.shape
    radius, cw, taps = bilateral_tables(d)
    if H == 0 or W == 0:
        return g.copy()
    rows = np.array([_reflect101(p, H) for p in range(-radius, H + radius)])
    cols = np.array([_reflect101(p, W) for p in range(-radius, W + radius)])
    pad = g[np.ix_(rows, cols)].astype(np.int32)
    v0 = g.astype(np.int32)

    def tap(k):
        dy, dx, sw = taps[k]
        v = pad[radius + dy:radius + dy + H, radius + dx:radius + dx + W]
        w = cw[np.abs(v - v0)] * sw
        return w, w * v.astype(np.float32)

    s = np.zeros((H, W), np.float32)
    ws = np.zeros((H, W), np.float32)
    n4 = len(taps) // 4 * 4
    for k in range(0, n4, 4):
        (w0, p0), (w1, p1), (w2, p2), (w3, p3) = (tap(k + i) for i in range(4))
        ws = ws + ((w0 + w1) + (w2 + w3))
        s = s + ((p0 + p1) + (p2 + p3))
    for k in range(n4, len(taps)):
        w, p = tap(k)
        s = s + p
        ws = ws + w
    return np.rint(s / ws).astype(np.uint8)


def marker_stage(bgr, depth, gisto_diap=False, multi_otsu_opt=False, median_blur=0, bilateral_d=None):
    """gray, hist, levels, markers of one BGR frame.  median_blur = k > 0: the MEDIAN_BLUR branch
    (PictureService.java:481-483), medianBlur(srcGray, k) before the histogram (restated as the
    exact k x k median with replicated borders, oracle/shape_oracle.median); else bilateral_d = d
    (not None): the BILATERIAL branch (:488-495), bilateral(srcGray, d)."""
    g = gray(bgr)
    if median_blur:
        from oracle import shape_oracle
        g = shape_oracle.median(g, int(median_blur))
    elif bilateral_d is not None:
        g = bilateral(g, int(bilateral_d))
    h = hist256(g)
    lv = levels(h, bgr.shape[0], bgr.shape[1], depth, gisto_diap, multi_otsu_opt)
    return g, h, lv, markers(g, marker_lut(lv, gisto_diap))
