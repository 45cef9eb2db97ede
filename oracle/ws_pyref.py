"""Independent pure-Python restatement of the hot path -- TEST INFRASTRUCTURE ONLY.

Second, structurally different restatement of OpenCV 3.4.2 ``cv::watershed`` ([ext]
modules/imgproc/src/segmentation.cpp, called from the reference at
``src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java:909``) used to
cross-check ``oracle/ws_oracle.c`` on small inputs.  Where the C oracle uses 256 FIFO
arrays with a moving ``active`` level, this one uses a single binary heap keyed by
``(level, push_sequence)``, which is the priority order the 256-bucket FIFO implements
("a strict priority queue on key (level, push-time)").  Pure Python:
keep inputs small (<= ~256x256).

Only tests/ may import this module.
"""
import heapq

import numpy as np

WSHED = -1
IN_QUEUE = -2


def _cdiff(img, a, b):
    pa = img[a]
    pb = img[b]
    return max(abs(int(pa[0]) - int(pb[0])), abs(int(pa[1]) - int(pb[1])),
               abs(int(pa[2]) - int(pb[2])))


def watershed(bgr, markers):
    """Return a new int32 label map; ``bgr`` is (H, W, 3) uint8, ``markers`` (H, W) int32."""
    bgr = np.asarray(bgr, dtype=np.uint8)
    m = np.array(markers, dtype=np.int32, copy=True)
    H, W = m.shape
    if H == 0 or W == 0:
        return m
    img = bgr.reshape(H * W, 3)
    lab = m.reshape(-1).tolist()
    # frame (PictureService.java:909 -> segmentation.cpp border pass)
    for c in range(W):
        lab[c] = WSHED
        lab[(H - 1) * W + c] = WSHED
    for r in range(H):
        lab[r * W] = WSHED
        lab[r * W + W - 1] = WSHED
    raw = lab[:]  # interior raw values; frame already WSHED

    heap = []
    seq = 0
    for r in range(1, H - 1):
        for c in range(1, W - 1):
            p = r * W + c
            if lab[p] < 0:
                lab[p] = 0
            if lab[p] != 0:
                continue
            best = None
            for q in (p - 1, p + 1, p - W, p + W):
                # a neighbour counts only if its RAW value is positive (frame is WSHED)
                if raw[q] > 0:
                    d = _cdiff(img, p, q)
                    best = d if best is None else min(best, d)
            if best is not None:
                heapq.heappush(heap, (best, seq, p))
                seq += 1
                lab[p] = IN_QUEUE

    while heap:
        _, _, p = heapq.heappop(heap)
        label = 0
        for q in (p - 1, p + 1, p - W, p + W):
            t = lab[q]
            if t > 0:
                if label == 0:
                    label = t
                elif t != label:
                    label = WSHED
        lab[p] = label
        if label == WSHED:
            continue
        for q in (p - 1, p + 1, p - W, p + W):
            if lab[q] == 0:
                heapq.heappush(heap, (_cdiff(img, p, q), seq, q))
                seq += 1
                lab[q] = IN_QUEUE
    return np.array(lab, dtype=np.int32).reshape(H, W)


def colorize(labels, depth, palette=None):
    """colorByIndexes (PictureService.java:913-936); palette None = colored=false (white)."""
    labels = np.asarray(labels)
    H, W = labels.shape
    out = np.zeros((H, W, 3), dtype=np.uint8)
    for r in range(H):
        for c in range(W):
            idx = int(labels[r, c])
            if 0 < idx <= depth:
                out[r, c] = (255, 255, 255) if palette is None else palette[idx - 1]
    return out
