"""CPU: the oracle against the hand-derived known answers, the
independent Python restatement, and the committed golden fixtures."""
import os

import numpy as np
import pytest

from oracle import ws_oracle, ws_pyref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def kat1():
    img = np.zeros((5, 5, 3), np.uint8)
    m = np.zeros((5, 5), np.int32)
    m[1, 1] = 1
    m[3, 3] = 2
    want = np.array([[-1, -1, -1, -1, -1], [-1, 1, 1, -1, -1], [-1, 1, -1, 2, -1],
                     [-1, -1, 2, 2, -1], [-1, -1, -1, -1, -1]], np.int32)
    return img, m, want


@pytest.mark.parametrize("impl", [ws_oracle.watershed, ws_pyref.watershed])
def test_kat1_uniform_two_seeds(impl):
    img, m, want = kat1()
    assert np.array_equal(impl(img, m), want)


@pytest.mark.parametrize("impl", [ws_oracle.watershed, ws_pyref.watershed])
def test_kat2_frame_marker_is_destroyed(impl):
    m = np.zeros((3, 3), np.int32)
    m[0, 0] = 5
    out = impl(np.zeros((3, 3, 3), np.uint8), m)
    want = np.full((3, 3), -1, np.int32)
    want[1, 1] = 0
    assert np.array_equal(out, want)


@pytest.mark.parametrize("impl", [ws_oracle.watershed, ws_pyref.watershed])
def test_kat3_negative_interior_becomes_zero(impl):
    m = np.zeros((3, 3), np.int32)
    m[1, 1] = -7
    out = impl(np.zeros((3, 3, 3), np.uint8), m)
    assert out[1, 1] == 0 and (out[[0, 2], :] == -1).all() and (out[:, [0, 2]] == -1).all()


@pytest.mark.parametrize("impl", [ws_oracle.watershed, ws_pyref.watershed])
@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (2, 2), (7, 1), (2, 9), (9, 2)])
def test_kat4_thin_frames_all_wshed(impl, shape):
    m = np.ones(shape, np.int32) * 3
    out = impl(np.zeros(shape + (3,), np.uint8), m)
    assert (out == -1).all()


def test_empty_frames():
    for shape in [(0, 0), (0, 5), (5, 0)]:
        out = ws_oracle.watershed(np.zeros(shape + (3,), np.uint8), np.zeros(shape, np.int32))
        assert out.shape == shape


def test_oracle_matches_pyref_random():
    rng = np.random.default_rng(1)
    for t in range(60):
        H, W = rng.integers(1, 30, 2)
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        if t % 3 == 0:
            img = (img // 128 * 128).astype(np.uint8)
        elif t % 3 == 1:
            img = (img // 16).astype(np.uint8)
        m = np.zeros((H, W), np.int32)
        for _ in range(int(rng.integers(0, 12))):
            m[rng.integers(0, H), rng.integers(0, W)] = rng.integers(-4, 6)
        assert np.array_equal(ws_oracle.watershed(img, m), ws_pyref.watershed(img, m)), t


def test_output_value_set_and_frame():
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    m = np.zeros((40, 50), np.int32)
    m[10, 10], m[30, 40], m[5, 45] = 1, 2, 3
    out = ws_oracle.watershed(img, m)
    assert set(np.unique(out)) <= {-1, 0, 1, 2, 3}
    assert (out[0] == -1).all() and (out[-1] == -1).all()
    assert (out[:, 0] == -1).all() and (out[:, -1] == -1).all()


def test_colorize_rules():
    lab = np.array([[-1, 0, 1, 2, 3, 4]], np.int32)
    pal = np.array([[10, 20, 30], [40, 50, 60], [70, 80, 90]], np.uint8)
    out = ws_oracle.colorize(lab, 3, pal)
    assert out[0].tolist() == [[0, 0, 0], [0, 0, 0], [10, 20, 30], [40, 50, 60], [70, 80, 90], [0, 0, 0]]
    white = ws_oracle.colorize(lab, 2, None)
    assert white[0].tolist() == [[0, 0, 0], [0, 0, 0], [255] * 3, [255] * 3, [0, 0, 0], [0, 0, 0]]
    assert np.array_equal(ws_pyref.colorize(lab, 3, pal), out)


def test_gray_on_black_and_white_is_exact():
    bw = np.array([[[0, 0, 0], [255, 255, 255]]], np.uint8)
    assert ws_oracle.bgr2gray(bw).tolist() == [[0, 255]]


def test_golden_small_cases():
    z = np.load(os.path.join(GOLD, "small_cases.npz"))
    names = list(z["__names"])
    assert len(names) >= 15
    for n in names:
        img, m = z[n + "__img"], z[n + "__markers"]
        lab = ws_oracle.watershed(img, m)
        assert np.array_equal(lab, z[n + "__labels"]), n
        d = int(z[n + "__depth"])
        assert np.array_equal(ws_oracle.colorize(lab, d, z[n + "__palette"]), z[n + "__color"]), n
        assert np.array_equal(ws_oracle.colorize(lab, d, None), z[n + "__white"]), n
        assert np.array_equal(ws_oracle.bgr2gray(z[n + "__color"]), z[n + "__gray"]), n
