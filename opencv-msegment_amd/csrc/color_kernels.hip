// color_kernels.hip -- gfx950 kernels of the COLOR_METHOD marker stage, the caller that builds the
// flood's seeds in PictureService.colorAutoMarkerWatershed (PictureService.java:301-366):
//
//   src - filter2D(9x1 Laplacian), saturate                      :308-333   k_cm_sharpen
//     (the white -> black loop at :309-318 never fires: PixelUtil.checkPixelRGB, PixelUtil.java:19,
//      compares Java's signed byte -- 0xFF reads -1 -- with int 255, so white stays white)
//   bw = BGR2GRAY + threshold(OTSU)                              :338, :938 k_gray_hist + host Otsu
//   distanceTransform(bw, DIST_L2, 5)                            :343, :1020 k_cm_dt_init, k_cm_dt_sweep
//   normalize(NORM_MINMAX), threshold(0.4), dilate(3x3)          :1021, :348-350 k_cm_minmax, k_cm_peaks, k_cm_dilate3
//   findContours(RETR_CCOMP) + drawContours + circle             :356-364   CCL (shape_kernels.hip),
//                                                                           k_cm_regions, host order, k_cm_paint
//
// Exact restatements (the CPU checker lives under oracle/, test-only): the sharpen is
// integer arithmetic; the chamfer distance is the min-plus closure of the 5x5 mask, which the
// two-pass raster scan of OpenCV computes and which in-place relaxation sweeps reach as well
// (values only decrease and every value is a path length); normalisation and the 0.4 threshold
// use the same float operations (no contraction).  The contour order is restated through
// components: unpinned against a real OpenCV build.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msg {

constexpr unsigned CM_HV = 65536u, CM_DG = 91750u, CM_LG = 143976u;  // 1, 1.4, 2.1969 in Q16
constexpr unsigned CM_INIT = 0x7fffffffu >> 2;                      // OpenCV's INIT_DIST0

__device__ __forceinline__ int cm_reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = (p < 0) ? -p : 2 * n - 2 - p;
  return p;
}

// res(y, x, c) = clamp(9 s(y) - sum_{0 < |k| <= 4} s(reflect101(y + k)), 0, 255), s = the source
// pixel as it is (the reference's white -> black loop is a no-op in Java, see the header).  One
// thread per pixel.
__global__ __launch_bounds__(256) void k_cm_sharpen(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ out,
                                                    int H, int W) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= W) return;
  int acc0 = 0, acc1 = 0, acc2 = 0;
#pragma unroll
  for (int k = -4; k <= 4; ++k) {
    const int yy = cm_reflect101(y + k, H);
    const uint8_t* q = bgr + ((long long)yy * W + x) * 3;
    const int b = q[0], g = q[1], r = q[2];
    const int wgt = (k == 0) ? 9 : -1;
    acc0 += wgt * b;
    acc1 += wgt * g;
    acc2 += wgt * r;
  }
  uint8_t* o = out + ((long long)y * W + x) * 3;
  o[0] = (uint8_t)min(255, max(0, acc0));
  o[1] = (uint8_t)min(255, max(0, acc1));
  o[2] = (uint8_t)min(255, max(0, acc2));
}

__global__ __launch_bounds__(256) void k_cm_dt_init(const uint8_t* __restrict__ gray, int t,
                                                    unsigned* __restrict__ dt, long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride)
    dt[p] = ((int)gray[p] > t) ? CM_INIT : 0u;
}

// One relaxation sweep of the 5x5 chamfer mask, in place (Gauss-Seidel in whatever order the
// waves run: every value stays an upper bound that is a path length).  `changed` is set when any
// pixel decreased.  A pixel at <= 1 (HV) cannot decrease (the backward pass's own shortcut).
__global__ __launch_bounds__(256) void k_cm_dt_sweep(unsigned* dt, int H, int W, int* changed) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= W) return;
  const long long p = (long long)y * W + x;
  const unsigned cur = __hip_atomic_load(dt + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (cur <= CM_HV) return;
  unsigned t0 = cur;
  const int dy[16] = {-2, -2, -1, -1, -1, -1, -1, 0, 0, 1, 1, 1, 1, 1, 2, 2};
  const int dx[16] = {-1, 1, -2, -1, 0, 1, 2, -1, 1, -2, -1, 0, 1, 2, -1, 1};
  const unsigned wt[16] = {CM_LG, CM_LG, CM_LG, CM_DG, CM_HV, CM_DG, CM_LG, CM_HV,
                           CM_HV, CM_LG, CM_DG, CM_HV, CM_DG, CM_LG, CM_LG, CM_LG};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int yy = y + dy[k], xx = x + dx[k];
    if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
    const unsigned v = __hip_atomic_load(dt + (long long)yy * W + xx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + wt[k];
    t0 = min(t0, v);
  }
  if (t0 < cur) {
    __hip_atomic_store(dt + p, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *changed = 1;
  }
}

__global__ __launch_bounds__(256) void k_cm_minmax(const unsigned* __restrict__ dt, long long N,
                                                   unsigned* __restrict__ mm) {
  unsigned lo = 0xffffffffu, hi = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const unsigned v = dt[p];
    lo = min(lo, v);
    hi = max(hi, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (unsigned)__shfl_xor((int)lo, o));
    hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(mm, lo);
    atomicMax(mm + 1, hi);
  }
}

// normalize(0, 1, NORM_MINMAX) then threshold(0.4, 1, BINARY): float(t0) * 2^-16 * scale (+ shift
// when the minimum is not 0), compared with 0.4f -- the float operations of convertTo and
// thresh_32f, without contraction.
__global__ __launch_bounds__(256) void k_cm_peaks(const unsigned* __restrict__ dt, float scale, float shift,
                                                  int use_shift, uint8_t* __restrict__ thr, long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const float d = __fmul_rn((float)dt[p], 1.0f / 65536.0f);
    float v = __fmul_rn(d, scale);
    if (use_shift) v = __fadd_rn(v, shift);
    thr[p] = v > 0.4f ? 1 : 0;
  }
}

// dilate with a 3x3 kernel of ones (pixels outside the image do not take part)
__global__ __launch_bounds__(256) void k_cm_dilate3(const uint8_t* __restrict__ thr, uint8_t* __restrict__ pk,
                                                    int H, int W) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= W) return;
  uint8_t m = 0;
#pragma unroll
  for (int a = -1; a <= 1; ++a)
#pragma unroll
    for (int b = -1; b <= 1; ++b) {
      const int yy = y + a, xx = x + b;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) m |= thr[(long long)yy * W + xx];
    }
  pk[(long long)y * W + x] = m;
}

// Region lists: every component root with the background region left of its first pixel
// (-1 at the image's left edge), every hole root (background, not touching the frame) with the
// component left of its first pixel.  Roots are first pixels in raster order (CCL).
__global__ __launch_bounds__(256) void k_cm_regions(const uint8_t* __restrict__ pk, const int* __restrict__ L,
                                                    const int* __restrict__ L2, const uint8_t* __restrict__ frame,
                                                    int W, long long N, int2* comps, int2* holes, int* counts) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    if (pk[p]) {
      if (L[p] == (int)p) {
        const int e = (p % W) ? L2[p - 1] : -1;
        comps[atomicAdd(counts, 1)] = make_int2((int)p, e);
      }
    } else if (L2[p] == (int)p && !frame[p]) {
      holes[atomicAdd(counts + 1, 1)] = make_int2((int)p, L[p - 1]);
    }
  }
}

// Final marker image: components and holes take their region labels (R1 at the root), foreground
// pixels 4-adjacent to a hole also that hole's own label (R2) if higher, the frame-touching
// background 0; then the circle((5,5), 3) spans get 255.
__global__ __launch_bounds__(256) void k_cm_paint(const uint8_t* __restrict__ pk, const int* __restrict__ L,
                                                  const int* __restrict__ L2, const uint8_t* __restrict__ frame,
                                                  const int* __restrict__ R1, const int* __restrict__ R2,
                                                  int32_t* __restrict__ out, int H, int W, int4 c0, int4 c1) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= W) return;
  const long long p = (long long)y * W + x;
  int lab;
  if (pk[p]) {
    lab = R1[L[p]];
    const int dy[4] = {0, 0, -1, 1}, dx[4] = {-1, 1, 0, 0};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int yy = y + dy[d], xx = x + dx[d];
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      const long long q = (long long)yy * W + xx;
      if (pk[q]) continue;
      const int r = L2[q];
      if (!frame[r]) lab = max(lab, R2[r]);
    }
  } else {
    const int r = L2[p];
    lab = frame[r] ? 0 : R1[r];
  }
  // circle spans: rows 2..8 around (5, 5); c0 = x-from for rows 2..5, c1 = x-to for rows 2..5,
  // mirrored below (the walk is symmetric)
  const int dyc = y - 5;
  if (dyc >= -3 && dyc <= 3) {
    const int a = dyc < 0 ? -dyc : dyc;  // 0..3
    const int half = (a == 0) ? c0.x : (a == 1) ? c0.y : (a == 2) ? c0.z : c0.w;
    if (half >= 0 && x >= 5 - half && x <= 5 + half) lab = 255;
  }
  (void)c1;
  out[p] = lab;
}

__global__ __launch_bounds__(256) void k_cm_scatter(const int* __restrict__ tri, int n, int* __restrict__ R1,
                                                    int* __restrict__ R2) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const int r = tri[k];
  R1[r] = tri[n + k];
  R2[r] = tri[2 * n + k];
}

}  // namespace msg
