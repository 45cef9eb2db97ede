"""java.util.Random restated (48-bit LCG), for the reference's palette generator.

PictureService keeps ``private final Random rnd = new Random();`` (PictureService.java:64) and
draws each label colour in ``generateBGRColor`` (PictureService.java:236-241) as
``(byte)(rnd.nextInt(156) + 100)`` for B, then G, then R.  With an explicit seed this module
reproduces the exact palette a Java run with ``new Random(seed)`` would draw, so colourised
outputs can be checked bit for bit (the reference itself is unseeded and not reproducible).
"""

_MULT = 0x5DEECE66D
_MASK = (1 << 48) - 1


class JavaRandom:
    def __init__(self, seed):
        self._seed = (seed ^ _MULT) & _MASK

    def _next(self, bits):
        self._seed = (self._seed * _MULT + 0xB) & _MASK
        r = self._seed >> (48 - bits)
        if r & (1 << (bits - 1)) and bits == 32:
            r -= 1 << 32
        return r

    def next_int(self, bound):
        if bound <= 0:
            raise ValueError("bound must be positive")
        if bound & (-bound) == bound:
            return (bound * self._next(31)) >> 31
        while True:
            bits = self._next(31)
            val = bits % bound
            # Java: while (bits - val + (bound-1) < 0) -- int32 overflow test
            if bits - val + (bound - 1) < (1 << 31):
                return val


def generate_bgr_palette(depth, seed):
    """depth x 3 BGR palette exactly as colorByIndexes(colored=true) would draw it."""
    import numpy as np

    rnd = JavaRandom(seed)
    pal = np.empty((max(depth, 0), 3), dtype=np.uint8)
    for i in range(max(depth, 0)):
        pal[i, 0] = rnd.next_int(156) + 100
        pal[i, 1] = rnd.next_int(156) + 100
        pal[i, 2] = rnd.next_int(156) + 100
    return pal
