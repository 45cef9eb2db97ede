"""Deterministic synthetic inputs for the watershed hot path.

Counter-based splitmix64 hashing, so any frame is regenerated from (kind, size, seed) on the
GPU box instead of being shipped.  Frames are BGR uint8 (H, W, 3) plus int32 seed markers
(H, W), the two Mats PictureService.watershed receives (PictureService.java:908).

Kinds:
  mosaic        64 x 64 grid of uniform-colour cells; one 3x3 seed per cell at a jittered
                centre, label = cell index + 1  
  mosaic_noise  the same + per-channel noise in [0, noise], saturated (ordering stress case)
  random        uniform-random BGR with the mosaic's seeds (worst case for the exact flood)
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def hash3(seed, stream, idx):
    """64-bit hash of (seed, stream, idx); idx may be an array (< 2**32)."""
    key = (np.uint64(seed & 0xFFFFFF) << np.uint64(40)) | (np.uint64(stream & 0xFF) << np.uint64(32))
    return splitmix64(np.asarray(idx, dtype=np.uint64) ^ key)


def _cells(H, W, cells):
    ch = max(1, H // cells)
    cw = max(1, W // cells)
    ncr = (H + ch - 1) // ch
    ncc = (W + cw - 1) // cw
    return ch, cw, ncr, ncc


def seeds(H, W, seed, cells=64):
    """int32 markers: one s x s seed block per cell (s = 3, or 1 for cells under 5 px)."""
    m = np.zeros((H, W), dtype=np.int32)
    if H == 0 or W == 0:
        return m
    ch, cw, ncr, ncc = _cells(H, W, cells)
    s = 3 if min(ch, cw) >= 5 else 1
    ids = np.arange(ncr * ncc, dtype=np.uint64)
    h = hash3(seed, 2, ids)
    ar = max(0, min(ch // 4, (ch - s) // 2))
    ac = max(0, min(cw // 4, (cw - s) // 2))
    jr = (h & np.uint64(0xFFFF)).astype(np.int64) % (2 * ar + 1) - ar
    jc = ((h >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64) % (2 * ac + 1) - ac
    ci = (ids // np.uint64(ncc)).astype(np.int64)
    cj = (ids % np.uint64(ncc)).astype(np.int64)
    r0 = ci * ch + ch // 2 + jr - s // 2
    c0 = cj * cw + cw // 2 + jc - s // 2
    lab = (ids + np.uint64(1)).astype(np.int32)
    for dr in range(s):
        for dc in range(s):
            rr = r0 + dr
            cc = c0 + dc
            ok = (rr >= 0) & (rr < H) & (cc >= 0) & (cc < W)
            # blocks stay inside their own cell, so no two seeds write the same pixel
            m[rr[ok], cc[ok]] = lab[ok]
    return m


def mosaic_image(H, W, seed, cells=64, noise=0):
    img = np.zeros((H, W, 3), dtype=np.uint8)
    if H == 0 or W == 0:
        return img
    ch, cw, ncr, ncc = _cells(H, W, cells)
    ids = np.arange(ncr * ncc, dtype=np.uint64)
    h = hash3(seed, 0, ids)
    pal = np.stack([(h >> np.uint64(8 * k)) & np.uint64(255) for k in range(3)], axis=1).astype(np.uint8)
    rows = (np.arange(H) // ch)[:, None]
    cols = (np.arange(W) // cw)[None, :]
    img[:] = pal[rows * ncc + cols]
    if noise > 0:
        pix = np.arange(H * W, dtype=np.uint64)
        hn = hash3(seed, 1, pix)
        nz = np.stack([((hn >> np.uint64(8 * k)) & np.uint64(255)).astype(np.int32) % (noise + 1)
                       for k in range(3)], axis=1).reshape(H, W, 3)
        img = np.minimum(img.astype(np.int32) + nz, 255).astype(np.uint8)
    return img


def random_image(H, W, seed):
    pix = np.arange(H * W, dtype=np.uint64)
    h = hash3(seed, 3, pix)
    return np.stack([((h >> np.uint64(8 * k)) & np.uint64(255)).astype(np.uint8) for k in range(3)],
                    axis=1).reshape(H, W, 3)


def frame(kind, H, W, seed, noise=3, cells=64):
    """(bgr, markers, depth) for a synthetic frame; depth = number of seed labels."""
    if kind == "mosaic":
        img = mosaic_image(H, W, seed, cells)
    elif kind == "mosaic_noise":
        img = mosaic_image(H, W, seed, cells, noise=noise)
    elif kind == "random":
        img = random_image(H, W, seed)
    else:
        raise ValueError("unknown synthetic kind %r" % kind)
    m = seeds(H, W, seed, cells)
    _, _, ncr, ncc = _cells(max(H, 1), max(W, 1), cells)
    return img, m, ncr * ncc
