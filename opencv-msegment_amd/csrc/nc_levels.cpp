// nc_levels.cpp -- host side of the NOT_CONNECTED_MARKERS marker stage: brightness levels from
// the 256-bin histogram and the brightness -> marker table (include/msegment.h, msg_nc_levels /
// msg_nc_marker_lut).  256 bins of serial decisions: no GPU work here.
//
// Follows PictureService.notConnectedMarkers (src/main/java/ru/shayhulud/opencvcmsegment/
// service/PictureService.java) with Java's arithmetic: int division and int-wrapping products,
// IEEE doubles evaluated left to right (this file is built with -ffp-contract=off so no product
// is fused into an FMA), (int) casts that truncate toward zero.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/msegment.h"

namespace {

struct Level {  // model/BrightLevel.java
  int32_t start, end, count;
};

int32_t wrap_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
int32_t wrap_mul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

// MathUtil.meanI (MathUtil.java): double mean of the values, .intValue() (NaN -> 0)
int32_t mean_i(const std::vector<int32_t>& v) {
  double s = 0.0;
  for (int32_t x : v) s += (double)x;
  const double m = s / (double)v.size();
  if (m != m) return 0;
  if (m >= 2147483647.0) return 2147483647;
  if (m <= -2147483648.0) return (int32_t)(-2147483647 - 1);
  return (int32_t)m;
}

// BrightLevel.getMeanLevel
int32_t mean_level(const Level& l) {
  if (l.start == l.end) return l.start;
  const int32_t range = l.end - l.start;
  if (range == 1) return l.start;
  return l.start + range / 2;
}

// BrightLevel.getMeanDiap(range)
Level mean_diap(const Level& l, int32_t range) {
  const int32_t diam = l.end - l.start;
  if (diam <= range * 2) return l;
  const int32_t mean = mean_level(l);
  const int32_t s = mean - range < l.start ? mean - range + 1 : mean - range;
  const int32_t e = mean + range > l.end ? mean + range - 1 : mean + range;
  return Level{s, e, e - s + 1};
}

// "Collecting ranges" / flex thresholds, PictureService.java:574-640.  Note the reference's
// quirks, kept as they are: the block still open at bin 255 is never emitted, a level can close
// as (i, i-1) when a non-empty bin follows an empty bin 0, and a level's count adds its first
// bin twice.
std::vector<Level> flex_levels(const int32_t* h, int32_t depth) {
  const int32_t block_limit = 256 / depth;  // Double.valueOf(256 / depth).intValue()
  std::vector<Level> out;
  std::vector<int32_t> block{h[0]};
  Level temp{0, 0, h[0]};
  for (int i = 1; i < 256; ++i) {
    const int32_t prev = h[i - 1], curr = h[i];
    if (curr == 0) {
      if (prev != 0) {
        temp.end = i - 1;
        out.push_back(temp);
      }
      temp = Level{i, i, curr};
      block.clear();
      continue;
    }
    if (prev == 0) temp = Level{i, i, curr};
    std::vector<int32_t> with = block;
    with.push_back(curr);
    const double coeff = 0.5;
    const int32_t old_mean = block.empty() ? curr : mean_i(block);
    const int32_t new_mean = mean_i(with);
    const double min_t = (double)old_mean - (double)old_mean * coeff;
    const double max_t = (double)old_mean + (double)old_mean * coeff;
    if (min_t <= (double)new_mean && (double)new_mean <= max_t) {
      if ((int64_t)block.size() >= block_limit) {
        temp.end = i - 1;
        out.push_back(temp);
        temp = Level{i, i, curr};
        block.assign(1, curr);
      } else {
        block.push_back(curr);
        temp.count = wrap_add(temp.count, curr);
      }
      continue;
    }
    temp.end = i - 1;
    out.push_back(temp);
    temp = Level{i, i, curr};
    block.assign(1, curr);
  }
  return out;
}

// otsuPart (PictureService.java:945-996), including its shared wk/mk/m accumulators that are
// never reset between sibling calls.
struct OtsuStep {
  double max_var;
  int32_t idx;
  std::vector<int32_t> deepers;
};

struct Otsu {
  int k;
  std::vector<double> wk, mk, m;
  double mt;
  int32_t pixnum;
  const int32_t* hist;
  int hist_size;

  OtsuStep part(int start, int step) {
    double max_var = 0.0;
    int32_t max_idx = start, max_deep_idx = 0;
    std::vector<int32_t> max_deepers;
    for (int ii = start; ii < hist_size; ++ii) {
      const int32_t intensity = hist[ii];
      wk[step] += (double)intensity / (double)pixnum;
      mk[step] += (double)wrap_mul(ii, intensity) / (double)pixnum;
      m[step] = mk[step] / wk[step];
      if (step > 0) {
        double wks = 0.0, mks = 0.0;
        for (int q = 0; q < step + 1; ++q) {
          wks += wk[q];
          mks += mk[q];
        }
        wk[step + 1] = 1.0 - wks;
        mk[step + 1] = mt - mks;
      }
      if (step == k - 1) {
        double var = 0.0;
        for (int q = 0; q < step + 1; ++q) var += wk[q] * (m[q] - mt) * (m[q] - mt);
        if (max_var < var) {
          max_var = var;
          max_idx = ii;
        }
      } else {
        OtsuStep d = part(ii + 1, step + 1);
        if (d.max_var > max_var) {
          max_idx = ii;
          max_var = d.max_var;
          max_deep_idx = d.idx;
          max_deepers = std::move(d.deepers);
        }
      }
    }
    if (step == k - 1) return OtsuStep{max_var, max_idx, {}};
    max_deepers.push_back(max_deep_idx);
    return OtsuStep{max_var, max_idx, std::move(max_deepers)};
  }
};

// number of loop iterations otsuPart runs for k thresholds over n bins (the work it costs)
double otsu_iterations(int k, int n) {
  // it[s][start]: iterations of part(start, s) and below
  std::vector<std::vector<double>> it(k + 1, std::vector<double>(n + 2, 0.0));
  for (int s = k - 1; s >= 0; --s)
    for (int st = n; st >= 0; --st) {
      double t = 0.0;
      for (int ii = st; ii < n; ++ii) t += 1.0 + (s == k - 1 ? 0.0 : it[s + 1][ii + 1]);
      it[s][st] = t;
    }
  return k > 0 ? it[0][0] : 0.0;
}

}  // namespace

extern "C" {

int msg_nc_levels(const int32_t* hist256, int rows, int cols, int depth, unsigned options,
                  msg_bright_level* levels, int max_levels, int* n_levels) {
  if (!hist256 || !n_levels || rows < 0 || cols < 0) return MSG_EINVAL;
  if (max_levels > 0 && !levels) return MSG_EINVAL;
  if (depth <= 0) return MSG_EINVAL;  // 256 / depth: ArithmeticException in the reference
  *n_levels = 0;
  // calcHist's output is CV_32F and the reference reads it back with (int): counts above 2^24
  // come back rounded to float
  int32_t h[256];
  for (int i = 0; i < 256; ++i) {
    if (hist256[i] < 0) return MSG_EINVAL;
    h[i] = (int32_t)(float)hist256[i];
  }
  std::vector<Level> lv = flex_levels(h, depth);
  if (options & MSG_NC_MULTI_OTSU) {  // PictureService.java:650-722
    const int k = (int)lv.size();
    if (k == 0) return MSG_ESTATE;  // otsuPart returns null -> NullPointerException
    const int rhs = 128;            // reducedBrightHist rows (:557-563)
    int32_t red[128];
    for (int i = 0; i < 256; i += 2) red[i / 2] = (int32_t)(float)wrap_add(h[i], h[i + 1]);
    // the reference's exhaustive recursion visits ~C(128, k) splits: refuse what it could not
    // finish either (k >= 6 is > 5e9 iterations)
    if (otsu_iterations(k, rhs) > 2.0e9) return MSG_ERANGE;
    const int32_t pixnum = wrap_mul(rows, cols);
    double mt = 0.0;
    for (int i = 0; i < rhs; ++i) mt += (double)i * ((double)red[i] / (double)pixnum);
    Otsu o{k, std::vector<double>(k + 1, 0.0), std::vector<double>(k + 1, 0.0),
           std::vector<double>(k + 1, 0.0), mt, pixnum, red, rhs};
    OtsuStep r = o.part(0, 0);
    std::vector<int32_t> th = r.deepers;
    th.push_back(r.idx);
    std::stable_sort(th.begin(), th.end());
    for (auto& t : th) {
      const int32_t v = t * (256 / rhs);
      t = v >= 256 ? 255 : v;
    }
    std::vector<Level> ov;
    int32_t begin = 0;
    for (int32_t t : th) {
      ov.push_back(Level{begin, t - 1, 0});
      begin = t;
    }
    ov.back().end = 255;
    for (int i = 0; i < 256; ++i)
      for (auto& l : ov)
        if (l.start <= i && i <= l.end) l.count = wrap_add(l.count, h[i]);
    lv = std::move(ov);
  }
  // maxBlockValue = max(count) over an empty list: NoSuchElementException (:724-726)
  if (lv.empty()) return MSG_ESTATE;
  const int n = (int)lv.size();
  for (int i = 0; i < n && i < max_levels; ++i) {
    levels[i].start = lv[i].start;
    levels[i].end = lv[i].end;
    levels[i].count = lv[i].count;
  }
  *n_levels = n;
  return n <= max_levels ? MSG_OK : MSG_ERANGE;
}

int msg_nc_marker_lut(const msg_bright_level* levels, int n_levels, unsigned options,
                      int32_t* lut256) {
  if (!lut256 || n_levels < 0 || (n_levels > 0 && !levels)) return MSG_EINVAL;
  // ALLOCATE TO LAYERS, PictureService.java:781-821: the first level (in order) whose mean --
  // or mean band of +-3 with GISTO_DIAP -- holds the brightness marks the pixel and stops the
  // scan; the marker maps are then summed (:823-828), which leaves that one index
  for (int b = 0; b < 256; ++b) {
    lut256[b] = 0;
    for (int i = 0; i < n_levels; ++i) {
      const Level l{levels[i].start, levels[i].end, levels[i].count};
      bool hit;
      if (options & MSG_NC_GISTO_DIAP) {
        const Level d = mean_diap(l, 3);
        hit = d.start <= b && b <= d.end;
      } else {
        hit = b == mean_level(l);
      }
      if (hit) {
        lut256[b] = i + 1;
        break;
      }
    }
  }
  return MSG_OK;
}

}  // extern "C"
