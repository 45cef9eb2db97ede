"""ctypes wrapper around ``oracle/liboracle_ws.so`` -- TEST INFRASTRUCTURE ONLY.

The C restatement (``oracle/ws_oracle.c``) of OpenCV 3.4.2 ``cv::watershed`` (reached from
``PictureService.java:909``) and of ``PictureService.colorByIndexes``
(``PictureService.java:913-936``).  Only tests/, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, as the checker / the timed CPU baseline.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle_ws.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i32p = ctypes.POINTER(ctypes.c_int32)
        sz = ctypes.c_size_t
        L.oracle_watershed.argtypes = [u8p, sz, i32p, sz, ctypes.c_int, ctypes.c_int]
        L.oracle_watershed.restype = ctypes.c_int
        L.oracle_colorize.argtypes = [i32p, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      u8p, u8p, sz]
        L.oracle_colorize.restype = ctypes.c_int
        L.oracle_bgr2gray.argtypes = [u8p, sz, ctypes.c_int, ctypes.c_int, u8p, sz]
        L.oracle_bgr2gray.restype = ctypes.c_int
        L.oracle_chamfer5.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_chamfer5.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def watershed(bgr, markers):
    """Return a new int32 label map (input markers are not modified)."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    m = np.array(markers, dtype=np.int32, copy=True, order="C")
    H, W = m.shape
    assert bgr.shape == (H, W, 3)
    rc = lib().oracle_watershed(_p(bgr, ctypes.c_uint8), W * 3, _p(m, ctypes.c_int32), W * 4,
                                H, W)
    if rc != 0:
        raise RuntimeError("oracle_watershed failed: %d" % rc)
    return m


def colorize(labels, depth, palette=None):
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    H, W = labels.shape
    out = np.empty((H, W, 3), dtype=np.uint8)
    pal = None
    if palette is not None:
        pal = np.ascontiguousarray(palette, dtype=np.uint8).reshape(-1)
        assert pal.size >= depth * 3
    rc = lib().oracle_colorize(_p(labels, ctypes.c_int32), W * 4, H, W, int(depth),
                               _p(pal, ctypes.c_uint8) if pal is not None else None,
                               _p(out, ctypes.c_uint8), W * 3)
    if rc != 0:
        raise RuntimeError("oracle_colorize failed: %d" % rc)
    return out


def bgr2gray(bgr):
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W, _ = bgr.shape
    out = np.empty((H, W), dtype=np.uint8)
    lib().oracle_bgr2gray(_p(bgr, ctypes.c_uint8), W * 3, H, W, _p(out, ctypes.c_uint8), W)
    return out


def chamfer5(bw):
    """OpenCV 3.4.2 distanceTransform(DIST_L2, 5) raw fixed-point distances (uint32, x 2^-16)."""
    bw = np.ascontiguousarray(bw, dtype=np.uint8)
    H, W = bw.shape
    out = np.zeros((H, W), np.uint32)
    if H and W:
        rc = lib().oracle_chamfer5(_p(bw, ctypes.c_uint8), H, W, _p(out, ctypes.c_uint32))
        if rc:
            raise MemoryError("oracle_chamfer5: %d" % rc)
    return out
