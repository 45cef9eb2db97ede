"""The console entry point (msegment.cli) against App.java:14-31 and the reference's output naming
(OutFileNameGenerator.java:14-16).  CPU tests drive it with a stand-in service (argument handling,
echo, naming, the null-contour branch); the GPU test runs the real colour and shape pipelines through it and
compares the written PNGs with a direct PictureService call on the same picture."""
import io
import os

import numpy as np
import pytest

from msegment import cli
from msegment.picture_service import ColorResult, ShapeResult


class _FakeService:
    def __init__(self, res, cres=None):
        self.res = res
        self.cres = cres
        self.seen = None

    def color_auto_marker_watershed(self, src):
        self.seen = src
        if self.cres is not None:
            return self.cres
        h, w = src.shape[:2]
        z = np.zeros((h, w, 3), np.uint8)
        return ColorResult(z, z[:, :, 0], np.zeros((h, w), np.int32), 0, z)

    def shape_auto_marker_watershed(self, src):
        self.seen = src
        return self.res


def _write_picture(tmp_path, name="pic.test.png", h=24, w=40):
    rng = np.random.default_rng(5)
    bgr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    cli.write_png(os.path.join(str(tmp_path), name), bgr)
    return bgr


def test_generate_png_name():
    assert cli.generate_png("SHAPE_METHOD_hkp", 1, "result") == "SHAPE_METHOD_hkp_00001_result.png"
    assert cli.image_file_name("album.big.jpg") == "album"


@pytest.mark.parametrize("argv", [[], ["a"], ["a", "b"], ["a", "b", "c", "d"]])
def test_wrong_arg_count(argv):
    out = io.StringIO()
    assert cli.run(argv, out=out, service=_FakeService(None)) == 1
    assert out.getvalue().strip() == "error parsing args"


def test_missing_picture(tmp_path):
    out = io.StringIO()
    rc = cli.run([str(tmp_path), str(tmp_path), "nope.png"], out=out, service=_FakeService(None))
    assert rc == 2
    lines = out.getvalue().splitlines()
    assert lines[:3] == ["arg 0: %s" % tmp_path, "arg 1: %s" % tmp_path, "arg 2: nope.png"]
    assert "error with file stream" in lines[3]


def test_reads_bgr_and_saves_named_outputs(tmp_path):
    bgr = _write_picture(tmp_path)
    h, w = bgr.shape[:2]
    dst = np.full((h, w, 3), 7, np.uint8)
    bw = np.full((h, w), 9, np.uint8)
    cdst = np.full((h, w, 3), 5, np.uint8)
    cbw = np.full((h, w), 6, np.uint8)
    svc = _FakeService(ShapeResult(dst, bw, np.zeros((h, w), np.int32), 3),
                       ColorResult(cdst, cbw, np.zeros((h, w), np.int32), 11, cdst))
    out = io.StringIO()
    rc = cli.run([str(tmp_path), str(tmp_path), "pic.test.png", "--save"], out=out, service=svc)
    assert rc == 0
    assert np.array_equal(svc.seen, bgr)          # imread order: BGR
    odir = os.path.join(str(tmp_path), "pic_output")
    names = sorted(os.listdir(odir))
    assert names == ["COLOR_METHOD_pic_00001_result.png", "COLOR_METHOD_pic_00002_bw_result.png",
                     "SHAPE_METHOD_pic_00001_result.png", "SHAPE_METHOD_pic_00002_bw_result.png"]
    from PIL import Image

    got = np.asarray(Image.open(os.path.join(odir, names[2])).convert("RGB"))[:, :, ::-1]
    assert np.array_equal(got, dst)
    assert np.array_equal(np.asarray(Image.open(os.path.join(odir, names[3]))), bw)
    got = np.asarray(Image.open(os.path.join(odir, names[0])).convert("RGB"))[:, :, ::-1]
    assert np.array_equal(got, cdst)
    assert np.array_equal(np.asarray(Image.open(os.path.join(odir, names[1]))), cbw)
    text = out.getvalue()
    assert "colorAutoMarkerWatershed: 24x40, depth 11" in text and "depth 3" in text
    assert text.index("colorAutoMarkerWatershed") < text.index("shapeAutoMarkerWatershed")  # App.java:28-29


def test_no_contours_returns_quietly(tmp_path):
    _write_picture(tmp_path)
    out = io.StringIO()
    rc = cli.run([str(tmp_path), str(tmp_path), "pic.test.png", "--save"], out=out,
                 service=_FakeService(None))
    assert rc == 0 and "contours is empty" in out.getvalue()
    odir = os.path.join(str(tmp_path), "pic_output")
    assert sorted(os.listdir(odir)) == ["COLOR_METHOD_pic_00001_result.png", "COLOR_METHOD_pic_00002_bw_result.png"]


@pytest.mark.gpu
def test_cli_shape_pipeline_matches_service(tmp_path):
    """BASELINE config 1: a 256x256 PNG of the mosaic (seed 0) through the CLI."""
    from msegment.picture_service import PictureService

    from msegment import synth

    img, _, _ = synth.frame("mosaic", 256, 256, 0)
    cli.write_png(os.path.join(str(tmp_path), "m.png"), img)
    out = io.StringIO()
    rc = cli.run([str(tmp_path), str(tmp_path), "m.png", "--save", "--seed", "4"], out=out)
    assert rc == 0, out.getvalue()
    ref = PictureService(seed=4).shape_auto_marker_watershed(img)
    assert ref is not None
    odir = os.path.join(str(tmp_path), "m_output")
    from PIL import Image

    got = np.asarray(Image.open(os.path.join(odir, "SHAPE_METHOD_m_00001_result.png")).convert("RGB"))
    assert np.array_equal(got[:, :, ::-1], ref.dst)
    got_bw = np.asarray(Image.open(os.path.join(odir, "SHAPE_METHOD_m_00002_bw_result.png")))
    assert np.array_equal(got_bw, ref.bw)
    cref = PictureService(seed=4).color_auto_marker_watershed(img)
    got = np.asarray(Image.open(os.path.join(odir, "COLOR_METHOD_m_00001_result.png")).convert("RGB"))
    assert np.array_equal(got[:, :, ::-1], cref.dst)
    got_bw = np.asarray(Image.open(os.path.join(odir, "COLOR_METHOD_m_00002_bw_result.png")))
    assert np.array_equal(got_bw, cref.bw)
