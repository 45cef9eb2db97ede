"""Mirror of the reference's hot-path surface in ``PictureService`` over libmsegment.

Reference: src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java
  * ``private final Random rnd = new Random();``                          :64
  * ``generateBGRColor()`` -- each channel ``(byte)(rnd.nextInt(156)+100)``  :236-241
  * ``watershed(Mat src, Mat markers, Integer depth, boolean colored)``      :908-911
  * ``colorByIndexes(Mat markers, Integer depth, boolean colored)``          :913-936
  * ``bw_result`` = ``cvtColor(dst, COLOR_BGR2GRAY)``                        :376-379

Same names, argument meaning and error behaviour: ``watershed`` rewrites ``markers`` in place
(like ``Imgproc.watershed``) and returns the colourised Mat; a type/size mismatch raises
``MsegError`` where OpenCV's CV_Assert would throw ``CvException``.
"""
import random

from .jrandom import JavaRandom


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
