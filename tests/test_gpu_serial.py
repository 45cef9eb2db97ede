"""GPU parity of k_serial -- the serial-pop regime in a kernel of its own, queue bookkeeping in
registers and LDS records, stores deferred behind the next pop's loads (csrc/ws_kernels.hip) -- against the CPU oracle and against serial pops inside the
one-workgroup loop, on the inputs that live in that regime: real photographs (album.jpg pixels with
the shape method's seeds), scattered notConnectedMarkers-like seeds, noisy frames with the
speculative engine off (so every interrupt-dense stretch is popped serially)."""
import os

import numpy as np
import pytest

from msegment import synth
from oracle import ws_oracle

pytestmark = pytest.mark.gpu


def _run(seg, img, m):
    out = m.copy()
    seg.watershed(img, out)
    return out


def _exact(out, want, tag):
    if not np.array_equal(out, want):
        bad = np.argwhere(out != want)
        raise AssertionError("%s: %d pixels differ, first %s gpu=%d cpu=%d" % (
            tag, len(bad), bad[0].tolist(), out[tuple(bad[0])], want[tuple(bad[0])]))


def _album(seg, y0, y1, x0, x1):
    from PIL import Image

    rgb = np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "golden", "album_1500x1500.png")).convert("RGB"))
    img = np.ascontiguousarray(rgb[y0:y1, x0:x1, ::-1])
    return img, np.ascontiguousarray(seg.shape_markers(img)[0])


def _frames(seg):
    out = [("album_crop",) + _album(seg, 300, 900, 200, 1000)]
    rng = np.random.default_rng(17)
    for k in range(3):
        H, W = int(rng.integers(150, 400)), int(rng.integers(150, 400))
        yy, xx = np.mgrid[0:H, 0:W]
        g = (xx + 2 * yy) % 256
        img = np.stack([g, (g * 3) % 256, 255 - g], axis=2).astype(np.int64)
        img = np.clip(img + rng.integers(0, 12, (H, W, 3)), 0, 255).astype(np.uint8)
        m = np.zeros((H, W), np.int32)
        n = int(H * W * 0.01)
        m[rng.integers(0, H, n), rng.integers(0, W, n)] = rng.integers(1, 9, n)
        out.append(("scattered_%d" % k, img, m))
    img, m, _ = synth.frame("mosaic_noise", 384, 320, 21)
    out.append(("mosaic_noise", img, m))
    img, m, _ = synth.frame("random", 200, 230, 22)
    out.append(("random", img, m))
    return out


@pytest.mark.parametrize("spec", [False, True])
def test_serial_kernel_matches_oracle_and_inloop_pops(seg, spec):
    seg.set_speculative(spec)
    try:
        for name, img, m in _frames(seg):
            want = ws_oracle.watershed(img, m)
            seg.set_serial_kernel(True)
            seg.set_profiling(True)
            seg.kernel_profile(reset=True)
            try:
                a = _run(seg, img, m)
                prof = seg.kernel_profile(reset=True)
            finally:
                seg.set_profiling(False)
                seg.set_serial_kernel(False)
            b = _run(seg, img, m)
            _exact(a, want, "%s serial kernel (spec %s)" % (name, spec))
            _exact(b, want, "%s in-loop serial pops (spec %s)" % (name, spec))
            if name == "album_crop" and not spec:
                assert prof.get("k_serial", (0, 0))[0] > 0, "album crop never reached k_serial"
    finally:
        seg.set_speculative(True)


def test_serial_kernel_full_album_with_diag(seg):
    """The whole 1500^2 photograph (the reference's album.jpg) with the shape method's seeds, the
    regime split reported (msg_set_diag 3) and the labels exact."""
    img, m = _album(seg, 0, 1500, 0, 1500)
    want = ws_oracle.watershed(img, m)
    seg.set_diag(3)
    seg.set_serial_kernel(True)
    try:
        out = _run(seg, img, m)
        d = seg.stats()["diag"]
    finally:
        seg.set_diag(False)
        seg.set_serial_kernel(False)
    _exact(out, want, "album")
    assert d[3] > 0  # serial pops ran (in k_serial)
