"""CPU: host logic -- synthetic generator determinism, Java RNG restatement, golden digests of
the generator, and that the msegment package never reaches the oracle."""
import hashlib
import json
import os

import numpy as np

from msegment import synth
from msegment.jrandom import JavaRandom, generate_bgr_palette

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_java_random_known_values():
    assert JavaRandom(0)._next(32) == -1155484576          # new Random(0).nextInt()
    assert JavaRandom(42)._next(32) == -1170105035         # new Random(42).nextInt()
    r = JavaRandom(42)
    assert [r.next_int(10) for _ in range(5)] == [0, 3, 8, 4, 0]


def test_palette_range():
    pal = generate_bgr_palette(500, 7)
    assert pal.shape == (500, 3) and pal.min() >= 100 and pal.max() <= 255


def test_synth_deterministic_and_shapes():
    a = synth.frame("mosaic", 300, 200, 3)
    b = synth.frame("mosaic", 300, 200, 3)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    img, m, depth = a
    assert img.shape == (300, 200, 3) and m.shape == (300, 200) and m.dtype == np.int32
    labs = np.unique(m[m > 0])
    assert len(labs) == depth  # one seed per cell, none overwritten


def test_synth_matches_committed_digests():
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        dg = json.load(f)
    for key in ("mosaic_1024x1024_s1", "random_512x512_s3"):
        kind, size, s = key.rsplit("_", 2)
        H, W = map(int, size.split("x"))
        img, m, depth = synth.frame(kind, H, W, int(s[1:]))
        assert hashlib.sha256(img.tobytes()).hexdigest() == dg[key]["img_sha256"]
        assert hashlib.sha256(m.tobytes()).hexdigest() == dg[key]["markers_sha256"]
        assert depth == dg[key]["depth"]


def test_product_package_never_imports_oracle():
    pkg = os.path.join(ROOT, "opencv-msegment_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dp, f), encoding="utf-8", errors="replace").read()
                assert "ws_oracle" not in src and "ws_pyref" not in src and "liboracle" not in src, f


def _unbound_segmenter():
    """A Segmenter whose context was never created (no GPU here): any call that reached the library
    would fail on the null handle, so an MsegError(MSG_EINVAL) raised here comes from the binding's
    own argument checks."""
    import msegment
    from msegment import _lib

    s = msegment.Segmenter.__new__(msegment.Segmenter)
    s._L = _lib.load()
    s._h = None
    s.device = 0
    return s


def test_batch_rejects_short_palette_and_size_mismatch():
    import pytest

    from msegment import MsegError, _lib

    seg = _unbound_segmenter()
    img, m, _ = synth.frame("mosaic", 16, 24, 1)
    with pytest.raises(MsegError) as e:  # 4 colours needed, 3 given: C would read past the buffer
        seg.watershed_batch([(img, m.copy())], depth=4, palette=np.zeros((3, 3), np.uint8))
    assert e.value.code == _lib.MSG_EINVAL and "palette" in str(e.value)
    with pytest.raises(MsegError) as e:  # rows and cols come from the markers: the image must agree
        seg.watershed_batch([(img[:15], m.copy())], depth=4)
    assert e.value.code == _lib.MSG_EINVAL and "sizes differ" in str(e.value)
    with pytest.raises(MsegError) as e:
        seg.watershed_batch([(img, m.astype(np.int64))])
    assert e.value.code == _lib.MSG_EINVAL


def test_nc_pipeline_digest_reproduces():
    """The committed digest the NC pipeline's bench line is checked against
    (make_golden.py --pipelines) is what the oracles produce on that frame today."""
    from oracle import nc_oracle, ws_oracle

    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        dg = json.load(f)["nc_mosaic_4096x4096_s2_d4_GISTO_DIAP"]
    img, _, _ = synth.frame("mosaic", 4096, 4096, 2)
    _, _, lv, mk = nc_oracle.marker_stage(img, 4, gisto_diap=True)
    assert len(lv) == dg["depth"]
    assert hashlib.sha256(np.ascontiguousarray(mk, np.int32).tobytes()).hexdigest() == dg["markers_sha256"]
    assert hashlib.sha256(ws_oracle.watershed(img, mk).tobytes()).hexdigest() == dg["labels_sha256"]
