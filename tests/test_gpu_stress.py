"""GPU parity stress: many randomized frames built to exercise every batching path of the engine
(multi-segment batches, interrupt cuts, segment cuts, small-batch kernel vs. multi-block
kernels, dense seeds, negative markers), bit-exact against the CPU oracle."""
import numpy as np
import pytest

from oracle import ws_oracle
from msegment import synth

pytestmark = pytest.mark.gpu


def _terraced(rng, H, W, levels):
    """Few distinct colours in blobs: many ties, several bucket levels, plateaus + steps."""
    base = rng.integers(0, levels, ((H + 7) // 8, (W + 7) // 8, 1))
    img = np.kron(base, np.ones((8, 8, 1), dtype=np.int64))[:H, :W]
    img = np.repeat(img, 3, axis=2) * (255 // max(levels - 1, 1))
    jitter = rng.integers(0, 3, (H, W, 3)) * (rng.random((H, W, 1)) < 0.05)
    return np.clip(img + jitter, 0, 255).astype(np.uint8)


def _markers(rng, H, W, density, nlab):
    m = np.zeros((H, W), np.int32)
    k = max(1, int(H * W * density))
    rr = rng.integers(0, H, k)
    cc = rng.integers(0, W, k)
    m[rr, cc] = rng.integers(-2, nlab + 1, k)
    return m


def _check(seg, img, m, tag):
    out = m.copy()
    seg.watershed(img, out)
    want = ws_oracle.watershed(img, m)
    if not np.array_equal(out, want):
        bad = np.argwhere(out != want)
        raise AssertionError("%s: %d pixels differ, first %s gpu=%d cpu=%d" % (
            tag, len(bad), bad[0].tolist(), out[tuple(bad[0])], want[tuple(bad[0])]))


@pytest.mark.parametrize("seed", range(6))
def test_terraced_frames(seg, seed):
    rng = np.random.default_rng(1000 + seed)
    for t in range(6):
        H, W = int(rng.integers(40, 300)), int(rng.integers(40, 300))
        img = _terraced(rng, H, W, int(rng.integers(2, 9)))
        m = _markers(rng, H, W, float(rng.choice([0.0005, 0.003, 0.02])), int(rng.integers(2, 40)))
        _check(seg, img, m, "terraced s%d t%d %dx%d" % (seed, t, H, W))


@pytest.mark.parametrize("seed", range(4))
def test_gradients_and_noise(seg, seed):
    rng = np.random.default_rng(2000 + seed)
    for t in range(4):
        H, W = int(rng.integers(64, 257)), int(rng.integers(64, 257))
        yy, xx = np.mgrid[0:H, 0:W]
        g = (xx * rng.integers(1, 4) + yy * rng.integers(0, 3)) % 256
        img = np.stack([g, (g * 3) % 256, 255 - g], axis=2).astype(np.int64)
        img += rng.integers(0, int(rng.integers(1, 12)), (H, W, 3))
        img = np.clip(img, 0, 255).astype(np.uint8)
        m = _markers(rng, H, W, 0.002, 12)
        _check(seg, img, m, "gradient s%d t%d" % (seed, t))


def test_large_batches_cross_small_limit(seg):
    """Plateau frames whose generations straddle the small-batch size limit."""
    rng = np.random.default_rng(7)
    for H, W in [(700, 900), (1200, 500)]:
        img = _terraced(rng, H, W, 3)
        m = _markers(rng, H, W, 0.00002, 6)
        _check(seg, img, m, "big plateau %dx%d" % (H, W))


@pytest.mark.parametrize("kind", ["mosaic", "mosaic_noise", "random"])
def test_synthetic_medium(seg, kind):
    for s in range(3):
        img, m, _ = synth.frame(kind, 384, 320, 40 + s, cells=16)
        _check(seg, img, m, "%s s%d" % (kind, s))


@pytest.mark.parametrize("H,W", [(37, 2500), (5, 3077), (1029, 7), (130, 1025)])
def test_wide_and_narrow_frames(seg, H, W):
    """Several raster chunks per row (phase-1 compaction, RSEG = 1024 columns) with a partial last
    one, partial 4x4 tiles on both axes, and single-tile-column frames."""
    rng = np.random.default_rng(H * 7919 + W)
    img = _terraced(rng, H, W, 4)
    m = _markers(rng, H, W, 0.004, 9)
    _check(seg, img, m, "shape %dx%d" % (H, W))
