"""CPU checks of the host/device-shared index arithmetic in csrc/ws_shared.h: the 4x4 tiled
layout (tix, nb_of), the phase-1 marker encoding, and the batch-window rule (next_wcap).
The header is compiled with g++ (HIP qualifiers defined away) into a small driver."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "opencv-msegment_amd", "csrc", "ws_shared.h")

DRIVER = r'''
#define __host__
#define __device__
struct int2 { int x, y; };  // HIP vector types used by the header's workspace pointers
struct int4 { int x, y, z, w; };
#include <cstdio>
#include <cstdlib>
#include <initializer_list>
#include "ws_shared.h"
using namespace msg;
int main() {
  int bad = 0;
  const int shapes[][2] = {{1, 1}, {3, 5}, {4, 4}, {7, 9}, {17, 33}, {64, 3}, {5, 1030}};
  for (auto& sh : shapes) {
    const int H = sh[0], W = sh[1], Wt = (W + 3) / 4, Ht = (H + 3) / 4;
    const long long np = (long long)Ht * Wt * 16;
    char* seen = (char*)calloc(np, 1);
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < W; ++c) {
        const long long t = tix(r, c, Wt);
        if (t < 0 || t >= np || seen[t]) ++bad;  // a bijection into the tile space
        seen[t] = 1;
        const int dr[4] = {0, 0, -1, 1}, dc[4] = {-1, 1, 0, 0};
        for (int d = 0; d < 4; ++d) {
          const int rr = r + dr[d], cc = c + dc[d];
          // neighbours inside the padded tile grid must match tix; outside they may land in
          // the one-tile-row margins but never further than one tile row + one tile away
          const long long n = nb_of(t, d, Wt);
          if (rr >= 0 && cc >= 0 && rr < Ht * 4 && cc < Wt * 4) {
            if (n != tix(rr, cc, Wt)) ++bad;
          } else if (n < -16ll * (Wt + 1) || n >= np + 16ll * (Wt + 1)) {
            ++bad;
          }
        }
      }
    free(seen);
  }
  for (int lv = 0; lv < 256; ++lv)
    if (!is_p1(p1_state(lv)) || (p1_state(lv) & 255) != lv) ++bad;
  for (int s : {0, 5, -1, -2, queued_state(0), queued_state(1 << 30)})
    if (is_p1(s)) ++bad;
  // window: interrupt cut -> max(WMIN, 2 x committed); full uncut window -> x4; else unchanged
  if (next_wcap(0, 100000, 3, true) != WMIN) ++bad;
  if (next_wcap(0, 100000, 5000, true) != 10000) ++bad;
  if (next_wcap(64, 64, 64, false) != 256) ++bad;
  if (next_wcap(256, 10, 10, false) != 256) ++bad;
  if (next_wcap(MERGE_CAP / 4, MERGE_CAP / 4, MERGE_CAP / 4, false) != 0) ++bad;
  if (next_wcap(0, 1 << 20, 1 << 20, false) != 0) ++bad;
  printf("bad=%d\n", bad);
  return bad != 0;
}
'''


def test_shared_index_arithmetic():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.cpp")
        exe = os.path.join(d, "t")
        open(src, "w").write(DRIVER)
        try:
            subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.dirname(HDR), src, "-o", exe])
        except OSError as e:  # no compiler: skip; a compile error of the header is a failure
            pytest.skip("g++ unavailable: %s" % e)
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout + out.stderr
