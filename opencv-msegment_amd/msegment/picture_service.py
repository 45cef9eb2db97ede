"""Mirror of the reference's hot-path surface in ``PictureService`` over libmsegment.

Reference: src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java
  * ``private final Random rnd = new Random();``                          :64
  * ``generateBGRColor()`` -- each channel ``(byte)(rnd.nextInt(156)+100)``  :236-241
  * ``watershed(Mat src, Mat markers, Integer depth, boolean colored)``      :908-911
  * ``colorByIndexes(Mat markers, Integer depth, boolean colored)``          :913-936
  * ``bw_result`` = ``cvtColor(dst, COLOR_BGR2GRAY)``                        :376-379
  * ``notConnectedMarkers(ii, depth, filterMaskSize, options)``             :468-867
    (the caller that builds the flood's seeds from brightness levels; see not_connected_markers)
  * ``shapeAutoMarkerWatershed(ii, options)``                                :395-466
    (seeds from Canny edge rings; see shape_auto_marker_watershed)
  * ``colorAutoMarkerWatershed(ii, options)``                                :301-392
    (seeds from distance-transform peaks of the sharpened image; see color_auto_marker_watershed)

Same names, argument meaning and error behaviour: ``watershed`` rewrites ``markers`` in place
(like ``Imgproc.watershed``) and returns the colourised Mat; a type/size mismatch raises
``MsegError`` where OpenCV's CV_Assert would throw ``CvException``.
"""
import random
from collections import namedtuple

from .jrandom import JavaRandom

NcResult = namedtuple("NcResult", "dst bw labels levels colored_markers")
ShapeResult = namedtuple("ShapeResult", "dst bw labels depth")
ColorResult = namedtuple("ColorResult", "dst bw labels depth sharp")


def nc_option_flags(options, filter_mask_size):
    """msg_nc_marker_stage option bits for notConnectedMarkers' AlgorithmOptions
    (PictureService.java:469-495): GISTO_DIAP, MULTI_OTSU, and one pre-filter -- MEDIAN_BLUR wins
    over BILATERIAL (the reference's if / else-if) -- with filterMaskSize in bits 8-15.

    MEDIAN_BLUR: OpenCV 3.4.2's medianBlur asserts ``ksize % 2 == 1`` (C++ remainder, so every
    negative or even size throws CvException), so those raise MsegError here too; sizes above 255
    are valid in OpenCV but do not fit the option bits (MsegError, never a silent wrap).
    BILATERIAL: every size <= 0 behaves as 0 in bilateralFilter (sigma <= 0 -> 1, radius
    cvRound(1.5)), so it is passed as 0; sizes above 255 do not fit the option bits (MsegError).
    MSegmentNative.ncFilterBits is the same rule on the Java side."""
    from . import MsegError, _lib

    opts = set(options)
    flags = (_lib.MSG_NC_GISTO_DIAP if "GISTO_DIAP" in opts else 0) | (
        _lib.MSG_NC_MULTI_OTSU if "MULTI_OTSU" in opts else 0)
    k = int(filter_mask_size)
    if "MEDIAN_BLUR" in opts:
        if k < 1 or k % 2 != 1:
            raise MsegError(_lib.MSG_EINVAL, "MEDIAN_BLUR mask size %d: must be odd and >= 1 "
                            "(medianBlur's assertion)" % k)
        if k > 255:
            raise MsegError(_lib.MSG_EINVAL, "MEDIAN_BLUR mask size %d: at most 255" % k)
        flags |= _lib.MSG_NC_MEDIAN_BLUR | _lib.MSG_NC_MASK(k)
    elif "BILATERIAL" in opts:
        if k > 255:
            raise MsegError(_lib.MSG_EINVAL, "BILATERIAL mask size %d: at most 255" % k)
        flags |= _lib.MSG_NC_BILATERAL | _lib.MSG_NC_MASK(max(k, 0))
    return flags


class PictureService:
    def __init__(self, segmenter=None, seed=None, device=0):
        from . import Segmenter

        self.segmenter = segmenter if segmenter is not None else Segmenter(device)
        # Java's `new Random()` is unseeded; pass `seed` to reproduce a given Java palette.
        self.rnd = JavaRandom(seed if seed is not None else random.getrandbits(48))

    def generate_bgr_color(self):
        b = self.rnd.next_int(156) + 100
        g = self.rnd.next_int(156) + 100
        r = self.rnd.next_int(156) + 100
        return (b, g, r)

    def _palette(self, depth, colored):
        if not colored:
            return None  # all white (PictureService.java:921-922)
        import numpy as np

        return np.array([self.generate_bgr_color() for _ in range(depth)], dtype=np.uint8).reshape(-1, 3)

    def watershed(self, src, markers, depth, colored):
        """PictureService.watershed: Imgproc.watershed(src, markers); colorByIndexes(...)."""
        depth = int(depth)
        pal = self._palette(depth, colored)
        return self.segmenter.watershed_colorize(src, markers, depth, pal)

    def watershed_with_gray(self, src, markers, depth, colored):
        """watershed + the callers' bw_result (cvtColor BGR2GRAY), fused on the GPU."""
        depth = int(depth)
        pal = self._palette(depth, colored)
        return self.segmenter.watershed_colorize(src, markers, depth, pal, gray=True)

    def color_by_indexes(self, markers, depth, colored):
        depth = int(depth)
        return self.segmenter.colorize(markers, depth, self._palette(depth, colored))

    def not_connected_markers(self, src, depth, options=(), colored_markers=False, filter_mask_size=3):
        """PictureService.notConnectedMarkers (PictureService.java:468-867) on the GPU.

        ``options``: names of AlgorithmOptions (model/dic/AlgorithmOptions.java).  COLORED,
        GISTO_DIAP, MULTI_OTSU and MEDIAN_BLUR change the result; NO_SAVE_STEPS / BW_RESULT only
        concern saving step images, which is not part of this drop-in (every step image is
        skipped).  MEDIAN_BLUR = medianBlur(srcGray, filter_mask_size) before the histogram
        (:481-483; an even size raises MsegError(EINVAL), like medianBlur's assertion); else
        BILATERIAL = bilateralFilter(srcGray, dst, filter_mask_size, 2 filter_mask_size,
        2 filter_mask_size) (:488-495, fp32 as OpenCV 3.4.2's non-IPP path sums it).

        Same Random draws as the reference: colorByIndexes(markers, n, true) for the
        "colored_markers_summ" step (:830) draws n colours before the watershed's own
        colorByIndexes (:834) draws n more when COLORED.  Returns NcResult(dst = the result
        image, bw = its BGR2GRAY (:839-841), labels = the flooded marker map, levels, and the
        coloured marker image when ``colored_markers``).
        """
        import numpy as np
        import torch

        opts = set(options)
        flags = nc_option_flags(opts, filter_mask_size)
        colored = "COLORED" in opts
        src = np.ascontiguousarray(np.asarray(src, dtype=np.uint8))
        H, W = src.shape[:2]
        dev = torch.device("cuda", self.segmenter.device)
        d_src = torch.from_numpy(src).to(dev)
        markers = torch.empty((H, W), dtype=torch.int32, device=dev)
        seg = self.segmenter
        levels = seg.nc_marker_stage_dev(d_src, int(depth), markers, flags)
        n = len(levels)
        step_pal = self._palette(n, True)  # :830, drawn whether or not the step is saved
        cm = None
        if colored_markers:
            cm = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
            seg.colorize_dev(markers, n, torch.from_numpy(step_pal).to(dev), cm)
        pal = self._palette(n, colored)
        dst = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        bw = torch.empty((H, W), dtype=torch.uint8, device=dev)
        seg.watershed_colorize_dev(d_src, markers, markers, n,
                                   torch.from_numpy(pal).to(dev) if pal is not None else None, dst, bw)
        torch.cuda.synchronize(dev)
        return NcResult(dst.cpu().numpy(), bw.cpu().numpy(), markers.cpu().numpy(), levels,
                        cm.cpu().numpy() if cm is not None else None)

    def shape_auto_marker_watershed(self, src, options=()):
        """PictureService.shapeAutoMarkerWatershed (PictureService.java:395-466) on the GPU.

        gray -> medianBlur(calculateSizeOfSquareBlurMask) -> Canny(5, 50) -> dilate 3 / dilate 5
        / subtract -> medianBlur 3 -> connectedComponents(8) = markers; depth = the RETR_CCOMP
        contour count (:447-451) -- ``None`` when there is no contour, like the reference's
        ``return null``.  Then this.watershed(src, markers, depth, colored) (:455) and the
        bw_result (:460-462).  ``options``: COLORED changes the result; the save-step options do
        not apply here.  Returns ShapeResult(dst, bw, labels = the flooded markers, depth).
        """
        import numpy as np
        import torch

        colored = "COLORED" in set(options)
        src = np.ascontiguousarray(np.asarray(src, dtype=np.uint8))
        H, W = src.shape[:2]
        dev = torch.device("cuda", self.segmenter.device)
        d_src = torch.from_numpy(src).to(dev)
        markers = torch.empty((H, W), dtype=torch.int32, device=dev)
        seg = self.segmenter
        depth, _ = seg.shape_markers_dev(d_src, markers)
        if depth == 0:
            return None
        pal = self._palette(depth, colored)
        dst = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        bw = torch.empty((H, W), dtype=torch.uint8, device=dev)
        seg.watershed_colorize_dev(d_src, markers, markers, depth,
                                   torch.from_numpy(pal).to(dev) if pal is not None else None, dst, bw)
        torch.cuda.synchronize(dev)
        return ShapeResult(dst.cpu().numpy(), bw.cpu().numpy(), markers.cpu().numpy(), depth)

    def color_auto_marker_watershed(self, src, options=()):
        """PictureService.colorAutoMarkerWatershed (PictureService.java:301-392) on the GPU.

        src - 9x1 Laplacian (the sharpened image is what the watershed floods, :333; the
        white -> black loop :309-318 is a no-op in Java, PixelUtil.java:19's signed-byte compare), Otsu bw, distanceTransform peaks, contours -> markers and depth = the contour
        count (:355-364), then this.watershed(src, markers, depth, colored) (:378) and the
        bw_result (:384-386).  ``options``: COLORED changes the result; the save-step options do
        not apply here.  Returns ColorResult(dst, bw, labels = the flooded markers, depth, sharp).
        The contour numbering is unpinned against a real OpenCV build.
        """
        import numpy as np
        import torch

        colored = "COLORED" in set(options)
        src = np.ascontiguousarray(np.asarray(src, dtype=np.uint8))
        H, W = src.shape[:2]
        dev = torch.device("cuda", self.segmenter.device)
        d_src = torch.from_numpy(src).to(dev)
        sharp = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        markers = torch.empty((H, W), dtype=torch.int32, device=dev)
        seg = self.segmenter
        depth = seg.color_markers_dev(d_src, sharp, markers)
        pal = self._palette(depth, colored)
        dst = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        bw = torch.empty((H, W), dtype=torch.uint8, device=dev)
        seg.watershed_colorize_dev(sharp, markers, markers, depth,
                                   torch.from_numpy(pal).to(dev) if pal is not None else None, dst, bw)
        torch.cuda.synchronize(dev)
        return ColorResult(dst.cpu().numpy(), bw.cpu().numpy(), markers.cpu().numpy(), depth,
                           sharp.cpu().numpy())
