// nc_kernels.hip -- gfx950 kernels of the NOT_CONNECTED_MARKERS marker stage, the caller that
// builds the flood's seeds in PictureService.notConnectedMarkers (PictureService.java:468-842):
//
//   srcGray = cvtColor(src, COLOR_BGR2GRAY)                          :476-478
//   brightHist = calcHist(srcGray, 256 bins, [0, 256))               :565
//   ... levels from the histogram (host, nc_levels.cpp)               :574-722
//   markers(i,j) = idx of the first level whose mean (or mean band)  :781-842
//                  equals srcGray(i,j), else 0; summed over the level maps (one term is nonzero)
//
// Both kernels stream: k_gray_hist reads 3 B/px and writes 1 B/px (+ 256 atomics per block),
// k_nc_markers reads 1 B/px and writes 4 B/px.  One thread = four pixels (three dword loads of
// BGR, one dword of gray), grid-strided, so 4-byte alignment of the frame buffers is required
// (checked on the host); markers are stored as int4, so that buffer needs 16-byte alignment.
// Plain (temporal) loads and stores: the flood that follows re-reads the frame and the markers,
// and at 4096^2 they fit the 256 MB MALL.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msg {

constexpr int GH_BS = 1024;   // k_gray_hist block (16 waves), one block per CU
constexpr int GH_COPIES = 2;  // LDS sub-histograms per wave (lane & 1), rows padded to 257 words
constexpr int GH_UNROLL = 4;  // 4-pixel groups per thread in flight (4 x 12 B loads)

// OpenCV's 8-bit BGR2GRAY (fixed point, yuv_shift 14): Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14
__device__ __forceinline__ uint32_t gray_of(uint32_t b, uint32_t g, uint32_t r) {
  return (1868u * b + 9617u * g + 4899u * r + 8192u) >> 14;
}

// Counts go to LDS sub-histograms (two per wave, rows skewed by one bank so the copies of a bin
// sit in different banks); a wave whose 256 pixels share one gray value adds them with a single
// ds_add (flat regions otherwise serialise 64 lanes on one address).  Each block then adds its
// 256 sums to hist with global atomics: with one block per CU that is 256 atomics per bin.
// (scripts/exp/hist_variants.hip: one sub-histogram per wave costs 3x on a flat frame; 4096
// blocks of global atomics, or a last-block reduction over per-block partials, cost 4x.)
// FROM_GRAY: `bgr` is already a gray plane (the MEDIAN_BLUR branch, :481-483, histograms the
// blurred srcGray): one dword of 4 pixels per group, no gray output.
template <bool FROM_GRAY>
__global__ __launch_bounds__(GH_BS) void k_gray_hist(const uint8_t* __restrict__ bgr, long long N,
                                                     uint8_t* __restrict__ gray,
                                                     unsigned* __restrict__ hist) {
  constexpr int ST = 257, NSUB = GH_BS / 64 * GH_COPIES;
  __shared__ unsigned sh[NSUB * ST];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int k = tid; k < NSUB * ST; k += GH_BS) sh[k] = 0;
  __syncthreads();
  unsigned* mine = sh + ((tid >> 6) * GH_COPIES + (lane & (GH_COPIES - 1))) * ST;
  const long long nq = N >> 2;  // full 4-pixel groups
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(bgr);
  const long long stride = (long long)gridDim.x * GH_BS * GH_UNROLL;
  for (long long q0 = (long long)blockIdx.x * GH_BS * GH_UNROLL + tid; q0 < nq; q0 += stride) {
    uint32_t w[GH_UNROLL][3];
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      const long long q = q0 + (long long)u * GH_BS;
      if (q < nq) {
        if (FROM_GRAY) {
          w[u][0] = b32[q];
        } else {
          w[u][0] = b32[3 * q];
          w[u][1] = b32[3 * q + 1];
          w[u][2] = b32[3 * q + 2];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      const long long q = q0 + (long long)u * GH_BS;
      if (q >= nq) break;
      uint32_t y0, y1, y2, y3;
      if (FROM_GRAY) {
        const uint32_t g4 = w[u][0];
        y0 = g4 & 255u;
        y1 = (g4 >> 8) & 255u;
        y2 = (g4 >> 16) & 255u;
        y3 = g4 >> 24;
      } else {
        // B0 G0 R0 B1 | G1 R1 B2 G2 | R2 B3 G3 R3
        const uint32_t w0 = w[u][0], w1 = w[u][1], w2 = w[u][2];
        y0 = gray_of(w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
        y1 = gray_of(w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
        y2 = gray_of((w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
        y3 = gray_of((w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
        reinterpret_cast<uint32_t*>(gray)[q] = y0 | (y1 << 8) | (y2 << 16) | (y3 << 24);
      }
      const uint32_t yw = __builtin_amdgcn_readfirstlane(y0);
      const unsigned nact = (unsigned)__popcll(__ballot(1));
      if (__all(y0 == yw && y1 == yw && y2 == yw && y3 == yw)) {
        if (lane == 0) atomicAdd(mine + yw, 4u * nact);
      } else {
        atomicAdd(mine + y0, 1u);
        atomicAdd(mine + y1, 1u);
        atomicAdd(mine + y2, 1u);
        atomicAdd(mine + y3, 1u);
      }
    }
  }
  if (blockIdx.x == 0 && tid < (int)(N & 3)) {  // ragged tail (< 4 pixels)
    const long long p = (nq << 2) + tid;
    uint32_t y;
    if (FROM_GRAY) {
      y = bgr[p];
    } else {
      y = gray_of(bgr[3 * p], bgr[3 * p + 1], bgr[3 * p + 2]);
      gray[p] = (uint8_t)y;
    }
    atomicAdd(mine + y, 1u);
  }
  __syncthreads();
  if (tid < 256) {
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < NSUB; ++k) s += sh[k * ST + tid];
    if (s) atomicAdd(hist + tid, s);
  }
}

struct NcLut {
  int32_t v[256];  // marker for each brightness (0 = no level's mean / mean band)
};

__global__ __launch_bounds__(256) void k_nc_markers(const uint8_t* __restrict__ gray, long long N,
                                                    int32_t* __restrict__ markers, NcLut lut) {
  __shared__ int32_t sl[256];
  sl[threadIdx.x] = lut.v[threadIdx.x];
  __syncthreads();
  const long long nq = N >> 2;
  const uint32_t* g32 = reinterpret_cast<const uint32_t*>(gray);
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
       q += (long long)gridDim.x * blockDim.x) {
    const uint32_t g = g32[q];
    int4 m;
    m.x = sl[g & 255u];
    m.y = sl[(g >> 8) & 255u];
    m.z = sl[(g >> 16) & 255u];
    m.w = sl[g >> 24];
    reinterpret_cast<int4*>(markers)[q] = m;
  }
  if (blockIdx.x == 0 && threadIdx.x < (int)(N & 3)) {
    const long long p = (nq << 2) + threadIdx.x;
    markers[p] = sl[gray[p]];
  }
}

// ---- BILATERIAL pre-filter: bilateralFilter(srcGray, dst, d, 2d, 2d) (:488-495) -------------
// OpenCV 3.4.2's bilateralFilter_8u for one channel, BORDER_REFLECT_101, in fp32 with the
// summation order of its x86 (SSE3) path: taps in groups of four, each group's weights and
// weighted values added pairwise ((0+1)+(2+3)) into the running sums, the last maxk % 4 taps one
// at a time, dst = cvRound(sum / wsum).  The tables are computed on the host with the same
// double-precision exp as OpenCV's set-up (the colour table goes to LDS, the taps are read with
// scalar loads: every lane walks the same disc).  One thread = one pixel, a wave = 64 columns of
// a row, so each tap's gather is one coalesced 64-byte row segment; blocks whose disc stays
// inside the frame skip the reflection.  No contraction into FMAs: the products round first.
struct BilColor {
  float v[256];
};
struct BilTap {
  float w;
  int dy, dx;
};
constexpr int BIL_ROWS = 4;  // block = 64 columns x 4 rows

__device__ __forceinline__ int reflect101(int p, int n) {  // borderInterpolate, REFLECT_101
  if ((unsigned)p < (unsigned)n) return p;
  if (n == 1) return 0;
  do {
    p = p < 0 ? -p : 2 * n - 2 - p;
  } while ((unsigned)p >= (unsigned)n);
  return p;
}

__global__ __launch_bounds__(64 * BIL_ROWS) void k_bilateral(const uint8_t* __restrict__ src,
                                                             uint8_t* __restrict__ dst, int H, int W,
                                                             const BilTap* __restrict__ taps,
                                                             int maxk, int radius, BilColor cw) {
#pragma clang fp contract(off)
  __shared__ float scw[256];
  scw[threadIdx.x] = cw.v[threadIdx.x];
  __syncthreads();
  const int x0 = blockIdx.x * 64, y0 = blockIdx.y * BIL_ROWS;
  const int x = x0 + (threadIdx.x & 63), y = y0 + (int)(threadIdx.x >> 6);
  if (x >= W || y >= H) return;
  const bool inside = x0 >= radius && y0 >= radius && x0 + 64 + radius <= W && y0 + BIL_ROWS + radius <= H;
  const int v0 = src[(size_t)y * W + x];
  auto sample = [&](const BilTap& t, float& w, float& p) {
    int yy = y + t.dy, xx = x + t.dx;
    if (!inside) {
      yy = reflect101(yy, H);
      xx = reflect101(xx, W);
    }
    const int v = src[(size_t)yy * W + xx];
    w = scw[abs(v - v0)] * t.w;
    p = w * (float)v;
  };
  float sum = 0.f, wsum = 0.f;
  int k = 0;
  for (; k + 4 <= maxk; k += 4) {
    float w0, w1, w2, w3, p0, p1, p2, p3;
    sample(taps[k], w0, p0);
    sample(taps[k + 1], w1, p1);
    sample(taps[k + 2], w2, p2);
    sample(taps[k + 3], w3, p3);
    wsum += (w0 + w1) + (w2 + w3);
    sum += (p0 + p1) + (p2 + p3);
  }
  for (; k < maxk; ++k) {
    float w, p;
    sample(taps[k], w, p);
    sum += p;
    wsum += w;
  }
  dst[(size_t)y * W + x] = (uint8_t)__float2int_rn(__fdiv_rn(sum, wsum));
}

}  // namespace msg
