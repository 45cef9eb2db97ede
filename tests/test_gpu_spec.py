"""GPU parity of the speculative generations (csrc/spec_kernels.hip): the interrupt-dense regime
(textured frames, scattered seeds, real photographs) against the CPU oracle, bit-exact, with the
engine's counters checked so that the tests fail if the frames stop reaching it."""
import numpy as np
import pytest

from oracle import ws_oracle
from msegment import synth

pytestmark = pytest.mark.gpu


@pytest.fixture
def spec_seg(seg):
    seg.set_speculative(True)
    yield seg
    seg.set_speculative(True)


def _run(seg, img, m):
    out = m.copy()
    seg.watershed(img, out)
    return out, seg.stats()


def _assert_exact(out, want, tag):
    if not np.array_equal(out, want):
        bad = np.argwhere(out != want)
        raise AssertionError("%s: %d pixels differ, first %s gpu=%d cpu=%d" % (
            tag, len(bad), bad[0].tolist(), out[tuple(bad[0])], want[tuple(bad[0])]))


@pytest.mark.parametrize("kind,S,seed", [("mosaic_noise", 256, 1), ("mosaic_noise", 512, 7),
                                         ("mosaic_noise", 1024, 1), ("random", 256, 3)])
def test_noise_frames_reach_the_engine(spec_seg, kind, S, seed):
    img, m, _ = synth.frame(kind, S, S, seed)
    out, st = _run(spec_seg, img, m)
    _assert_exact(out, ws_oracle.watershed(img, m), "%s %d s%d" % (kind, S, seed))
    assert st["spec_generations"] > 0 and st["spec_rounds"] >= 2 * st["spec_generations"]
    assert st["pops"] > 0


@pytest.mark.parametrize("H,W,noise", [(301, 517, 3), (97, 1023, 9), (640, 123, 1), (5, 900, 6)])
def test_ragged_noise_frames(spec_seg, H, W, noise):
    img = synth.mosaic_image(H, W, 11, cells=16, noise=noise)
    m = synth.seeds(H, W, 11, cells=16)
    out, _ = _run(spec_seg, img, m)
    _assert_exact(out, ws_oracle.watershed(img, m), "ragged %dx%d noise %d" % (H, W, noise))


@pytest.mark.parametrize("seed", range(4))
def test_scattered_seeds_and_wide_levels(spec_seg, seed):
    """Seeds everywhere (the NC pipeline's kind of marker map) on gradients with noise: long
    cascades through many levels, so executions overflow and the serial fallback runs."""
    rng = np.random.default_rng(7000 + seed)
    H, W = int(rng.integers(200, 420)), int(rng.integers(200, 420))
    yy, xx = np.mgrid[0:H, 0:W]
    g = (xx * int(rng.integers(1, 3)) + yy) % 256
    img = np.stack([g, (g * 5) % 256, 255 - g], axis=2).astype(np.int64)
    img = np.clip(img + rng.integers(0, int(rng.integers(2, 40)), (H, W, 3)), 0, 255).astype(np.uint8)
    m = np.zeros((H, W), np.int32)
    k = int(H * W * float(rng.choice([0.002, 0.01, 0.05])))
    m[rng.integers(0, H, k), rng.integers(0, W, k)] = rng.integers(1, 50, k)
    out, _ = _run(spec_seg, img, m)
    _assert_exact(out, ws_oracle.watershed(img, m), "scattered s%d %dx%d" % (seed, H, W))


def test_real_photo_crop_with_fallbacks(spec_seg):
    """album.jpg pixels (decoded, tests/golden) with the shape method's seeds: cascades larger
    than a lane's capacity are handed to serial pops and the regime resumes after them."""
    import os
    from PIL import Image

    path = os.path.join(os.path.dirname(__file__), "golden", "album_1500x1500.png")
    rgb = np.asarray(Image.open(path).convert("RGB"))
    img = np.ascontiguousarray(rgb[200:900, 300:1000, ::-1])
    m = np.ascontiguousarray(spec_seg.shape_markers(img)[0])
    out, st = _run(spec_seg, img, m)
    _assert_exact(out, ws_oracle.watershed(img, m), "album crop")
    assert st["spec_generations"] > 0


def test_engine_off_gives_the_same_labels(seg):
    img, m, _ = synth.frame("mosaic_noise", 384, 384, 5)
    seg.set_speculative(True)
    on, st_on = _run(seg, img, m)
    seg.set_speculative(False)
    try:
        off, st_off = _run(seg, img, m)
    finally:
        seg.set_speculative(True)
    assert st_on["spec_generations"] > 0 and st_off["spec_generations"] == 0
    assert np.array_equal(on, off)
    _assert_exact(on, ws_oracle.watershed(img, m), "on/off")


def test_repeated_calls_reuse_round_tags(spec_seg):
    """Claims are tagged by round and never cleared between calls: repeated floods of different
    frames in one context must not read each other's claims."""
    for k in range(6):
        kind = ("mosaic_noise", "random")[k % 2]
        img, m, _ = synth.frame(kind, 192 + 32 * k, 160 + 16 * k, 40 + k)
        out, _ = _run(spec_seg, img, m)
        _assert_exact(out, ws_oracle.watershed(img, m), "repeat %d" % k)


def test_batch_api_in_flight(spec_seg):
    frames = [synth.frame("mosaic_noise", 320, 320, 60 + k) for k in range(6)]
    imgs = [f[0] for f in frames]
    mks = [f[1].copy() for f in frames]
    spec_seg.watershed_batch(list(zip(imgs, mks)))
    for k, f in enumerate(frames):
        _assert_exact(mks[k], ws_oracle.watershed(f[0], f[1]), "batch %d" % k)
