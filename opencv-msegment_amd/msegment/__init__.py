"""msegment -- MI355X-native drop-in for the reference's watershed hot path.

Host-side mirror of the reference interface over libmsegment.so (include/msegment.h):

* :class:`Segmenter` -- one libmsegment context (one HIP stream + device workspace).
  ``watershed`` is ``Imgproc.watershed(src, markers)`` (PictureService.java:909): markers are
  rewritten IN PLACE with OpenCV's exact label map; ``colorize`` is ``colorByIndexes``
  (PictureService.java:913-936).
* :class:`PictureService` (picture_service.py) -- ``watershed(src, markers, depth, colored)``
  exactly as ``PictureService.watershed`` (PictureService.java:908-911).

Errors raise :class:`MsegError` (the ``CvException`` analogue); a missing HIP library raises
ImportError -- there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import MsegError, Stats

__all__ = ["Segmenter", "MsegError", "Stats", "PictureService", "nc_levels", "nc_marker_lut"]


def _levels_out(arr, n):
    return [(int(arr[k].start), int(arr[k].end), int(arr[k].count)) for k in range(n)]


def nc_levels(hist, rows, cols, depth, options=0):
    """Brightness levels of notConnectedMarkers from a 256-bin histogram (host code of the
    library, PictureService.java:574-722): list of (start, end, count)."""
    L = _lib.load()
    h = np.ascontiguousarray(np.asarray(hist, dtype=np.int32).reshape(256))
    arr = (_lib.BrightLevel * 256)()
    n = ctypes.c_int(0)
    rc = L.msg_nc_levels(ctypes.c_void_p(h.ctypes.data), int(rows), int(cols), int(depth),
                         int(options), arr, 256, ctypes.byref(n))
    if rc != 0:
        raise MsegError(rc, "msg_nc_levels failed")
    return _levels_out(arr, n.value)


def nc_marker_lut(levels, options=0):
    """Brightness -> marker table of ALLOCATE TO LAYERS (PictureService.java:781-828)."""
    L = _lib.load()
    n = len(levels)
    arr = (_lib.BrightLevel * max(n, 1))()
    for k, (s, e, c) in enumerate(levels):
        arr[k].start, arr[k].end, arr[k].count = int(s), int(e), int(c)
    lut = np.zeros(256, dtype=np.int32)
    rc = L.msg_nc_marker_lut(arr, n, int(options), ctypes.c_void_p(lut.ctypes.data))
    if rc != 0:
        raise MsegError(rc, "msg_nc_marker_lut failed")
    return lut


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _img_view(bgr):
    bgr = np.asarray(bgr)
    if bgr.dtype != np.uint8 or bgr.ndim != 3 or bgr.shape[2] != 3:
        raise MsegError(_lib.MSG_EINVAL, "src must be uint8 (H, W, 3) BGR (CV_8UC3)")
    if bgr.strides[2] != 1 or bgr.strides[1] != 3 or bgr.strides[0] < 0:
        bgr = np.ascontiguousarray(bgr)
    return bgr, bgr.strides[0] if bgr.shape[0] > 0 else bgr.shape[1] * 3


class Segmenter:
    """One libmsegment context on HIP device ``device``."""

    def __init__(self, device=0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        rc = self._L.msg_create(ctypes.byref(h), int(device), 0)
        if rc != 0:
            raise MsegError(rc, "msg_create(device=%d) failed" % device)
        self._h = h
        self.device = device

    # -- plumbing -------------------------------------------------------------------------
    def _check(self, rc):
        if rc != 0:
            raise MsegError(rc, self._L.msg_last_error(self._h).decode(errors="replace"))

    def close(self):
        if getattr(self, "_h", None):
            self._L.msg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_profiling(self, on=True):
        self._check(self._L.msg_set_profiling(self._h, 1 if on else 0))

    def kernel_profile(self, reset=True):
        """{kernel: (launches, total_ms)} from HIP events on the launch stream."""
        arr = (_lib.KernelProfile * _lib.NKERNELS)()
        n = self._L.msg_get_kernel_profile(self._h, arr, _lib.NKERNELS, 1 if reset else 0)
        if n < 0:
            self._check(n)
        return {arr[k].name.decode(): (arr[k].launches, arr[k].total_ms) for k in range(n)}

    def stats(self):
        s = Stats()
        self._check(self._L.msg_get_stats(self._h, ctypes.byref(s)))
        out = {k: getattr(s, k) for k, _ in Stats._fields_}
        out["diag"] = list(s.diag)
        return out

    def set_diag(self, on=True):
        """In-kernel counters; on=2 also injects k_resolve give-ups (tests of the re-run path);
        on=3 reports the one-workgroup loop's regime split instead, on=4 the cooperative cascade
        pop's phases (diagnostic build; msegment.h, msg_set_diag)."""
        self._check(self._L.msg_set_diag(self._h, int(on) if on in (2, 3, 4) else (1 if on else 0)))

    def set_fast_commit(self, on=True):
        """Two-launch iterations for large flood batches (default on); off = three launches."""
        self._check(self._L.msg_set_fast_commit(self._h, 1 if on else 0))

    def set_speculative(self, on=True):
        """Speculative generations for the interrupt-dense regime (default on); off = serial pops."""
        self._check(self._L.msg_set_speculative(self._h, 1 if on else 0))

    # -- host buffers (numpy) -------------------------------------------------------------
    def watershed(self, bgr, markers):
        """cv::watershed(bgr, markers): ``markers`` (int32 (H, W) ndarray) is rewritten in place."""
        self.watershed_colorize(bgr, markers, None)
        return markers

    def watershed_colorize(self, bgr, markers, depth, palette=None, gray=False):
        """Fused PictureService.watershed: labels in place, then colorByIndexes (+ BGR2GRAY).

        ``depth=None`` skips the colourise step.  ``palette`` = (depth, 3) uint8 BGR or None
        (colored=false: white).  Returns dst or (dst, gray)."""
        bgr, bstride = _img_view(bgr)
        if not isinstance(markers, np.ndarray) or markers.dtype != np.int32 or markers.ndim != 2:
            raise MsegError(_lib.MSG_EINVAL, "markers must be an int32 (H, W) ndarray (CV_32SC1)")
        H, W = markers.shape
        if bgr.shape[:2] != (H, W):
            raise MsegError(_lib.MSG_EINVAL, "src and markers sizes differ")
        work = markers
        if markers.strides[1] != 4 or markers.strides[0] < W * 4 or not markers.flags.writeable:
            work = np.ascontiguousarray(markers)
        mstride = work.strides[0] if H > 0 else W * 4
        dst = gr = pal = None
        if depth is not None:
            depth = int(depth)
            dst = np.empty((H, W, 3), dtype=np.uint8)
            if gray:
                gr = np.empty((H, W), dtype=np.uint8)
            if palette is not None:
                pal = np.ascontiguousarray(palette, dtype=np.uint8).reshape(-1, 3)
                if pal.shape[0] < depth:
                    raise MsegError(_lib.MSG_EINVAL, "palette has fewer than depth colours")
        rc = self._L.msg_watershed_colorize(
            self._h, _vp(bgr), bstride, _vp(work), mstride, H, W,
            depth if depth is not None else 0, _vp(pal), _vp(dst), W * 3, _vp(gr), W)
        self._check(rc)
        if work is not markers:
            markers[...] = work
        if depth is None:
            return markers
        return (dst, gr) if gray else dst

    def colorize(self, labels, depth, palette=None):
        """colorByIndexes(labels, depth, colored) -> (H, W, 3) uint8."""
        labels = np.ascontiguousarray(labels, dtype=np.int32)
        H, W = labels.shape
        dst = np.empty((H, W, 3), dtype=np.uint8)
        pal = None
        if palette is not None:
            pal = np.ascontiguousarray(palette, dtype=np.uint8).reshape(-1, 3)
        self._check(self._L.msg_colorize(self._h, _vp(labels), W * 4, H, W, int(depth), _vp(pal),
                                         _vp(dst), W * 3))
        return dst

    def watershed_batch(self, frames, depth=None, palette=None):
        """frames: list of (bgr, markers); every markers array is rewritten in place.  With a
        depth, also each frame's colorByIndexes (msg_watershed_colorize_batch): returns the list of
        colourised BGR frames (palette: depth x 3 BGR bytes, None = white)."""
        n = len(frames)
        keep = []
        bp = (ctypes.c_void_p * n)()
        bs = (ctypes.c_size_t * n)()
        mp = (ctypes.c_void_p * n)()
        ms = (ctypes.c_size_t * n)()
        rows = (ctypes.c_int * n)()
        cols = (ctypes.c_int * n)()
        for k, (bgr, m) in enumerate(frames):
            bgr, st = _img_view(bgr)
            if not isinstance(m, np.ndarray) or m.dtype != np.int32 or m.ndim != 2 or not m.flags.c_contiguous:
                raise MsegError(_lib.MSG_EINVAL, "batch markers must be C-contiguous int32 (H, W)")
            if bgr.shape[:2] != m.shape:  # rows and cols come from the markers alone
                raise MsegError(_lib.MSG_EINVAL, "frame %d: src and markers sizes differ" % k)
            keep.append(bgr)
            bp[k] = bgr.ctypes.data
            bs[k] = st
            mp[k] = m.ctypes.data
            ms[k] = m.shape[1] * 4
            rows[k], cols[k] = m.shape
        if depth is None:
            self._check(self._L.msg_watershed_batch(self._h, n, bp, bs, mp, ms, rows, cols))
            return None
        depth = int(depth)
        pal = None
        if palette is not None:  # the library reads 3 * depth bytes from it
            pal = np.ascontiguousarray(palette, dtype=np.uint8).reshape(-1, 3)
            if pal.shape[0] < depth:
                raise MsegError(_lib.MSG_EINVAL, "palette has fewer than depth colours")
        dsts = [np.empty(m.shape + (3,), np.uint8) for _, m in frames]
        dp = (ctypes.c_void_p * n)(*[d.ctypes.data for d in dsts])
        ds = (ctypes.c_size_t * n)(*[d.shape[1] * 3 for d in dsts])
        self._check(self._L.msg_watershed_colorize_batch(self._h, n, bp, bs, mp, ms, rows, cols, int(depth),
                                                          pal.ctypes.data if pal is not None else None, dp, ds))
        return dsts

    def set_batch_inflight(self, k):
        """Floods kept in flight by the batch calls (1..8; 1 = back to back)."""
        self._check(self._L.msg_set_batch_inflight(self._h, int(k)))

    def set_batch_devices(self, devices=()):
        """Spread the host-buffer batch calls over a device list (msg_set_batch_devices): frames
        [n*j/D, n*(j+1)/D) run on devices[j]; () = this context's own device."""
        devs = [int(d) for d in devices]
        arr = (ctypes.c_int * max(1, len(devs)))(*devs)
        self._check(self._L.msg_set_batch_devices(self._h, len(devs), arr if devs else None))

    def set_batch_floods(self, mode=1):
        """Many floods per launch in the batch calls (msegment.h msg_set_batch_floods): 0 off, 1 every
        flood serial to its end in one kernel (one wave per flood), 2 plateaus handed to batches, 3
        automatic (the library's default: a probe flood per frame size picks 0 or 1)."""
        self._check(self._L.msg_set_batch_floods(self._h, int(mode)))

    def set_resolve_grid(self, blocks=0):
        """Blocks per k_resolve launch (0 = the default); a performance knob only."""
        self._check(self._L.msg_set_resolve_grid(self._h, int(blocks)))

    # -- device-resident buffers (torch tensors on this device) ---------------------------
    @staticmethod
    def _stream(stream):
        if stream is None:
            import torch
            return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        return ctypes.c_void_p(int(stream))

    def watershed_dev(self, bgr, markers_in, labels=None, stream=None):
        """Device-resident flood: uint8 (H, W, 3) + int32 (H, W) -> int32 labels (may alias)."""
        H, W = markers_in.shape
        if labels is None:
            labels = markers_in
        for t in (bgr, markers_in, labels):
            if not t.is_contiguous():
                raise MsegError(_lib.MSG_EINVAL, "device tensors must be contiguous")
        self._check(self._L.msg_watershed_dev(self._h, ctypes.c_void_p(bgr.data_ptr()),
                                              ctypes.c_void_p(markers_in.data_ptr()),
                                              ctypes.c_void_p(labels.data_ptr()), H, W,
                                              self._stream(stream)))
        return labels

    def colorize_dev(self, labels, depth, palette=None, dst=None, gray=None, stream=None):
        H, W = labels.shape
        self._check(self._L.msg_colorize_dev(
            self._h, ctypes.c_void_p(labels.data_ptr()), H, W, int(depth),
            ctypes.c_void_p(palette.data_ptr()) if palette is not None else None,
            ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(gray.data_ptr()) if gray is not None else None,
            self._stream(stream)))
        return dst

    def watershed_colorize_dev(self, bgr, markers_in, labels, depth, palette, dst, gray=None,
                               stream=None):
        H, W = markers_in.shape
        self._check(self._L.msg_watershed_colorize_dev(
            self._h, ctypes.c_void_p(bgr.data_ptr()), ctypes.c_void_p(markers_in.data_ptr()),
            ctypes.c_void_p(labels.data_ptr()), H, W, int(depth),
            ctypes.c_void_p(palette.data_ptr()) if palette is not None else None,
            ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(gray.data_ptr()) if gray is not None else None,
            self._stream(stream)))
        return dst

    def watershed_colorize_batch_dev(self, bgrs, markers_in, labels, depth, palette, dsts, stream=None):
        """Device-resident batch (BASELINE config 5 on one GPU): lists of torch tensors, frame k
        reads bgrs[k], markers_in[k] and writes labels[k], dsts[k]; several floods in flight."""
        n = len(bgrs)
        if not (len(markers_in) == len(labels) == len(dsts) == n):
            raise MsegError(_lib.MSG_EINVAL, "batch lists differ in length")
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
        rows = (ctypes.c_int * n)(*[int(m.shape[0]) for m in markers_in])
        cols = (ctypes.c_int * n)(*[int(m.shape[1]) for m in markers_in])
        self._check(self._L.msg_watershed_colorize_batch_dev(
            self._h, n, arr(bgrs), arr(markers_in), arr(labels), rows, cols, int(depth),
            ctypes.c_void_p(palette.data_ptr()) if palette is not None else None, arr(dsts),
            self._stream(stream)))
        return dsts

    # -- NOT_CONNECTED_MARKERS marker stage (PictureService.java:468-842) ------------------
    def gray_hist_dev(self, bgr, gray, stream=None):
        """srcGray = BGR2GRAY(bgr) into ``gray`` (uint8 (H, W) tensor) + its 256-bin histogram."""
        H, W = bgr.shape[:2]
        hist = np.zeros(256, dtype=np.int32)
        self._check(self._L.msg_gray_hist_dev(self._h, ctypes.c_void_p(bgr.data_ptr()), H, W,
                                              ctypes.c_void_p(gray.data_ptr()),
                                              ctypes.c_void_p(hist.ctypes.data), self._stream(stream)))
        return hist

    def nc_marker_stage(self, bgr, depth, options=0):
        """Host-buffer marker stage: uint8 (H, W, 3) BGR -> (int32 (H, W) markers, levels)."""
        bgr, bstride = _img_view(bgr)
        H, W = bgr.shape[:2]
        markers = np.zeros((H, W), dtype=np.int32)
        arr = (_lib.BrightLevel * 256)()
        n = ctypes.c_int(0)
        self._check(self._L.msg_nc_marker_stage(self._h, _vp(bgr), bstride, H, W, int(depth),
                                                int(options), _vp(markers), max(W, 1) * 4, arr, 256,
                                                ctypes.byref(n)))
        return markers, _levels_out(arr, n.value)

    def nc_markers_dev(self, gray, lut, markers, stream=None):
        H, W = gray.shape
        lut = np.ascontiguousarray(np.asarray(lut, dtype=np.int32).reshape(256))
        self._check(self._L.msg_nc_markers_dev(self._h, ctypes.c_void_p(gray.data_ptr()), H, W,
                                               ctypes.c_void_p(lut.ctypes.data),
                                               ctypes.c_void_p(markers.data_ptr()), self._stream(stream)))
        return markers

    def nc_marker_stage_dev(self, bgr, depth, markers, options=0, gray=None, stream=None):
        """gray + histogram -> levels -> markers (int32 (H, W) tensor); returns the levels."""
        H, W = bgr.shape[:2]
        arr = (_lib.BrightLevel * 256)()
        n = ctypes.c_int(0)
        self._check(self._L.msg_nc_marker_stage_dev(
            self._h, ctypes.c_void_p(bgr.data_ptr()), H, W, int(depth), int(options),
            ctypes.c_void_p(gray.data_ptr()) if gray is not None else None,
            ctypes.c_void_p(markers.data_ptr()), arr, 256, ctypes.byref(n), self._stream(stream)))
        return _levels_out(arr, n.value)

    def shape_markers(self, bgr, ksize=None):
        """Host-buffer SHAPE_METHOD marker stage (PictureService.java:402-452): uint8 (H, W, 3)
        BGR -> (int32 (H, W) markers, depth = contour count, component count)."""
        bgr, bstride = _img_view(bgr)
        H, W = bgr.shape[:2]
        markers = np.zeros((H, W), dtype=np.int32)
        depth, ncomp = ctypes.c_int(0), ctypes.c_int(0)
        self._check(self._L.msg_shape_markers(self._h, _vp(bgr), bstride, H, W, int(ksize or 0),
                                              _vp(markers), max(W, 1) * 4, ctypes.byref(depth),
                                              ctypes.byref(ncomp)))
        return markers, depth.value, ncomp.value

    def shape_markers_dev(self, bgr, markers, ksize=None, blur=None, edges=None, mask=None, stream=None):
        """Device form: markers (int32 (H, W) tensor) out; optional uint8 (H, W) tensors receive the
        blurred gray, the Canny edges and the marker mask.  Returns (depth, ncomp)."""
        H, W = bgr.shape[:2]
        depth, ncomp = ctypes.c_int(0), ctypes.c_int(0)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        self._check(self._L.msg_shape_markers_dev(self._h, ptr(bgr), H, W, int(ksize or 0), ptr(markers),
                                                  ctypes.byref(depth), ctypes.byref(ncomp), ptr(blur),
                                                  ptr(edges), ptr(mask), self._stream(stream)))
        return depth.value, ncomp.value

    def color_markers_dev(self, bgr, sharp, markers, stream=None):
        """COLOR_METHOD marker stage (PictureService.java:301-366) on device tensors: bgr (H, W, 3)
        uint8 in; sharp (H, W, 3) uint8 (the sharpened image the watershed floods) and markers
        (H, W) int32 out.  Returns depth (the contour count)."""
        H, W = bgr.shape[:2]
        depth = ctypes.c_int(0)
        self._check(self._L.msg_color_markers_dev(self._h, ctypes.c_void_p(bgr.data_ptr()), H, W,
                                                  ctypes.c_void_p(sharp.data_ptr()),
                                                  ctypes.c_void_p(markers.data_ptr()), ctypes.byref(depth),
                                                  self._stream(stream)))
        return depth.value

    def color_markers(self, bgr):
        """Host form: (sharp BGR uint8, markers int32, depth)."""
        bgr, st = _img_view(bgr)
        H, W = bgr.shape[:2]
        sharp = np.empty((H, W, 3), np.uint8)
        m = np.empty((H, W), np.int32)
        depth = ctypes.c_int(0)
        self._check(self._L.msg_color_markers(self._h, _vp(bgr), st, H, W, _vp(sharp), max(W, 1) * 3,
                                              _vp(m), max(W, 1) * 4, ctypes.byref(depth)))
        return sharp, m, depth.value

    def edge_weights_dev(self, bgr, wright, wdown, stream=None):
        H, W = bgr.shape[:2]
        self._check(self._L.msg_edge_weights_dev(self._h, ctypes.c_void_p(bgr.data_ptr()),
                                                 ctypes.c_void_p(wright.data_ptr()),
                                                 ctypes.c_void_p(wdown.data_ptr()), H, W,
                                                 self._stream(stream)))
        return wright, wdown


from .picture_service import PictureService  # noqa: E402
