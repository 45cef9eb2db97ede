// shape_kernels.hip -- gfx950 kernels of the SHAPE_METHOD marker stage, the caller that builds
// the flood's seeds in PictureService.shapeAutoMarkerWatershed (PictureService.java:395-466):
//
//   srcGray = cvtColor(src, BGR2GRAY); medianBlur(srcGray, k)        :404-408   k_gray, k_median
//   Canny(brdGray, 5, 50)                                             :415-416   k_canny_nms + CCL
//   markerMask = dilate5(dilate3(edges)) - dilate3(edges); median 3  :426-435   k_ring_median3
//   connectedComponents(markerMask, markers, 8, CV_32S)               :441       CCL + numbering
//   depth = findContours(markerMask, RETR_CCOMP).size()               :447-452   CCL of the holes
//
// Stencils (gray, Sobel/NMS, ring/median3) stage tiles in LDS and stream; the median keeps a
// per-thread 256-bin histogram in LDS that slides down a column (Huang), so a k x k median costs
// 2k histogram updates per pixel instead of k^2 samples.  Connected components are a lock-free
// union-find over a parent array (hook the larger root under the smaller with atomicMin; roots
// end as the smallest pixel index of their component), used three times: Canny's hysteresis
// (candidates, 8-connected), the markers (8-connected), the holes (background, 4-connected).
// OpenCV's label order (first 2x2 block in block-raster order, see oracle/shape_oracle.py) comes
// from a per-root atomicMin of the block key, a flag per first block and an exclusive scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msg {

// ---- gray (OpenCV fixed point, same formula as k_gray_hist) ---------------------------------
__global__ __launch_bounds__(256) void k_gray(const uint8_t* __restrict__ bgr, long long N,
                                              uint8_t* __restrict__ g) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const uint8_t* q = bgr + 3 * p;
    g[p] = (uint8_t)((1868u * q[0] + 9617u * q[1] + 4899u * q[2] + 8192u) >> 14);
  }
}

// ---- k x k median, BORDER_REPLICATE (medianBlur) ---------------------------------------------
// Thread = one column x, rows [r0, r0 + MED_ROWS).  Its window histogram lives in LDS as 16-bit
// counts, two threads' bins per dword (lane pair), updated with no-return ds_add (a decrement is
// the add of 0xFFFF / 0xFFFF0000: the bin holds the removed sample, so no borrow crosses halves).
// The median m is tracked with lt = #samples < m: each update adjusts lt, then m moves until
// lt <= half < lt + hist[m].
constexpr int MED_BS = 64;
constexpr int MED_ROWS = 128;

__device__ __forceinline__ int med_bin(const unsigned* h, int v, int lane) {
  const unsigned w = h[v * (MED_BS / 2) + (lane >> 1)];
  return (int)((lane & 1) ? (w >> 16) : (w & 0xffffu));
}

__global__ __launch_bounds__(MED_BS) void k_median(const uint8_t* __restrict__ src,
                                                   uint8_t* __restrict__ dst, int H, int W, int k) {
  __shared__ unsigned hist[256 * (MED_BS / 2)];
  const int lane = threadIdx.x;
  const int x = blockIdx.x * MED_BS + lane;
  const int r0 = blockIdx.y * MED_ROWS;
  const int r1 = min(H, r0 + MED_ROWS);
  for (int i = lane; i < 256 * (MED_BS / 2); i += MED_BS) hist[i] = 0;
  __syncthreads();
  const bool on = x < W;
  const int h = k >> 1, half = (k * k) >> 1;
  const unsigned one = (lane & 1) ? 0x10000u : 1u;
  const unsigned minus = (lane & 1) ? 0xffff0000u : 0xffffffffu;
  unsigned* const hcol = hist + (lane >> 1);
  auto add_row = [&](int r, unsigned inc) {  // the k samples of row r (clamped) in this window
    const uint8_t* row = src + (long long)min(max(r, 0), H - 1) * W;
    for (int j = -h; j <= h; ++j) {
      const int v = row[min(max(x + j, 0), W - 1)];
      atomicAdd(&hcol[v * (MED_BS / 2)], inc);
    }
  };
  int m = 0, lt = 0;
  if (on) {
    for (int r = r0 - h; r <= r0 + h; ++r) add_row(r, one);
    // first median: scan up from 0
    int acc = 0;
    for (;;) {
      const int c = med_bin(hist, m, lane);
      if (acc + c > half) break;
      acc += c;
      ++m;
    }
    lt = acc;
  }
  for (int r = r0; r < r1; ++r) {
    if (on) {
      if (r > r0) {
        const uint8_t* out_row = src + (long long)min(max(r - 1 - h, 0), H - 1) * W;
        const uint8_t* in_row = src + (long long)min(r + h, H - 1) * W;
        for (int j = -h; j <= h; ++j) {
          const int xc = min(max(x + j, 0), W - 1);
          const int vo = out_row[xc], vi = in_row[xc];
          atomicAdd(&hcol[vo * (MED_BS / 2)], minus);
          atomicAdd(&hcol[vi * (MED_BS / 2)], one);
          lt += (vi < m) - (vo < m);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the adds land before the reads below
        while (lt > half) {
          --m;
          lt -= med_bin(hist, m, lane);
        }
        for (;;) {
          const int c = med_bin(hist, m, lane);
          if (lt + c > half) break;
          lt += c;
          ++m;
        }
      }
      dst[(long long)r * W + x] = (uint8_t)m;
    }
  }
}

// ---- Canny: 3x3 Sobel (replicate), L1 magnitude, non-maximum suppression ------------------
// Output class per pixel: 0 not a candidate, 1 candidate (m > low after NMS), 2 candidate with
// m > high.  Tile 64 x 16 outputs; gray staged with a 2-pixel halo, magnitudes with 1 (zero
// outside the frame, like OpenCV's zeroed magnitude border).
constexpr int CN_TX = 64, CN_TY = 16;
constexpr int CANNY_SHIFT = 15;
constexpr int CANNY_TG22 = 13573;  // (int)(tan(22.5 deg) * 2^15 + 0.5)

__global__ __launch_bounds__(256) void k_canny_nms(const uint8_t* __restrict__ g,
                                                   uint8_t* __restrict__ cls, int H, int W,
                                                   int low, int high) {
  __shared__ int sg[CN_TY + 4][CN_TX + 4];
  __shared__ int smag[CN_TY + 2][CN_TX + 2];
  __shared__ short sdx[CN_TY][CN_TX], sdy[CN_TY][CN_TX];
  const int tid = threadIdx.x;
  const int bx = blockIdx.x * CN_TX, by = blockIdx.y * CN_TY;
  for (int i = tid; i < (CN_TY + 4) * (CN_TX + 4); i += 256) {
    const int yy = i / (CN_TX + 4), xx = i % (CN_TX + 4);
    const int r = min(max(by + yy - 2, 0), H - 1), c = min(max(bx + xx - 2, 0), W - 1);
    sg[yy][xx] = g[(long long)r * W + c];
  }
  __syncthreads();
  for (int i = tid; i < (CN_TY + 2) * (CN_TX + 2); i += 256) {
    const int yy = i / (CN_TX + 2), xx = i % (CN_TX + 2);
    const int r = by + yy - 1, c = bx + xx - 1;
    int mg = 0;
    if (r >= 0 && r < H && c >= 0 && c < W) {
      const int y0 = yy + 1, x0 = xx + 1;  // centre in sg
      const int dx = (sg[y0 - 1][x0 + 1] - sg[y0 - 1][x0 - 1]) + 2 * (sg[y0][x0 + 1] - sg[y0][x0 - 1]) +
                     (sg[y0 + 1][x0 + 1] - sg[y0 + 1][x0 - 1]);
      const int dy = (sg[y0 + 1][x0 - 1] - sg[y0 - 1][x0 - 1]) + 2 * (sg[y0 + 1][x0] - sg[y0 - 1][x0]) +
                     (sg[y0 + 1][x0 + 1] - sg[y0 - 1][x0 + 1]);
      mg = abs(dx) + abs(dy);
      if (yy >= 1 && yy <= CN_TY && xx >= 1 && xx <= CN_TX) {
        sdx[yy - 1][xx - 1] = (short)dx;
        sdy[yy - 1][xx - 1] = (short)dy;
      }
    }
    smag[yy][xx] = mg;
  }
  __syncthreads();
  for (int i = tid; i < CN_TY * CN_TX; i += 256) {
    const int yy = i / CN_TX, xx = i % CN_TX;
    const int r = by + yy, c = bx + xx;
    if (r >= H || c >= W) continue;
    const int y0 = yy + 1, x0 = xx + 1;
    const int m = smag[y0][x0];
    int out = 0;
    if (m > low) {
      const int dx = sdx[yy][xx], dy = sdy[yy][xx];
      const int xs = abs(dx), ys = abs(dy);
      const int tx = xs * CANNY_TG22, ty = ys << CANNY_SHIFT;
      bool keep;
      if (ty < tx) {
        keep = m > smag[y0][x0 - 1] && m >= smag[y0][x0 + 1];
      } else {
        const int tg67 = tx + (xs << (CANNY_SHIFT + 1));
        if (ty > tg67) {
          keep = m > smag[y0 - 1][x0] && m >= smag[y0 + 1][x0];
        } else {
          const int s = ((dx ^ dy) < 0) ? -1 : 1;
          keep = m > smag[y0 - 1][x0 - s] && m > smag[y0 + 1][x0 + s];
        }
      }
      if (keep) out = (m > high) ? 2 : 1;
    }
    cls[(long long)r * W + c] = (uint8_t)out;
  }
}

// ---- connected components: union-find over a parent array ---------------------------------
// mode 0: fg = cls > 0 (Canny candidates), 8-connected; mode 1: fg = mask != 0, 8-connected;
// mode 2: fg = mask == 0 (background), 4-connected.
__device__ __forceinline__ bool ccl_fg(const uint8_t* a, long long p, int mode) {
  return mode == 2 ? a[p] == 0 : a[p] != 0;
}

__device__ __forceinline__ int ccl_find(const int* L, int x) {
  int y = __hip_atomic_load(L + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (y != x) {
    x = y;
    y = __hip_atomic_load(L + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return x;
}

__device__ __forceinline__ void ccl_union(int* L, int a, int b) {
  a = ccl_find(L, a);
  b = ccl_find(L, b);
  while (a != b) {
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    // a > b: hook root a under b; if a stopped being a root meanwhile, continue from its parent
    const int old = atomicMin(L + a, b);
    if (old == a) return;
    a = ccl_find(L, old);
    b = ccl_find(L, b);
  }
}

__global__ __launch_bounds__(256) void k_ccl_init(const uint8_t* __restrict__ a, int* __restrict__ L,
                                                  long long N, int mode) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride)
    L[p] = ccl_fg(a, p, mode) ? (int)p : -1;
}

__global__ __launch_bounds__(256) void k_ccl_merge(const uint8_t* __restrict__ a, int* L, int H, int W,
                                                   int mode) {
  const long long N = (long long)H * W;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    if (!ccl_fg(a, p, mode)) continue;
    const int r = (int)(p / W), c = (int)(p - (long long)r * W);
    if (c > 0 && ccl_fg(a, p - 1, mode)) ccl_union(L, (int)p, (int)(p - 1));
    if (r > 0) {
      if (ccl_fg(a, p - W, mode)) ccl_union(L, (int)p, (int)(p - W));
      if (mode != 2) {
        if (c > 0 && ccl_fg(a, p - W - 1, mode)) ccl_union(L, (int)p, (int)(p - W - 1));
        if (c + 1 < W && ccl_fg(a, p - W + 1, mode)) ccl_union(L, (int)p, (int)(p - W + 1));
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_ccl_compress(int* L, long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const int l = L[p];
    if (l >= 0 && l != (int)p) L[p] = ccl_find(L, l);
  }
}

// ---- hysteresis from the candidate components ----------------------------------------------
__global__ __launch_bounds__(256) void k_hyst_mark(const uint8_t* __restrict__ cls, const int* __restrict__ L,
                                                   uint8_t* __restrict__ flag, long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride)
    if (cls[p] == 2) flag[L[p]] = 1;
}

__global__ __launch_bounds__(256) void k_hyst_edges(const uint8_t* __restrict__ cls, const int* __restrict__ L,
                                                    const uint8_t* __restrict__ flag,
                                                    uint8_t* __restrict__ edges, long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride)
    edges[p] = (cls[p] && flag[L[p]]) ? 255 : 0;
}

// ---- ring = dilate5(dilate3(e)) - dilate3(e) = [max7 > max3] (dilations ignore the outside),
// then the 3x3 median with BORDER_REPLICATE of that binary image = majority of 9 -------------
constexpr int RG_T = 32;  // output tile RG_T x RG_T, edges staged with a 4-pixel halo

__global__ __launch_bounds__(256) void k_ring_median3(const uint8_t* __restrict__ e,
                                                      uint8_t* __restrict__ mask, int H, int W) {
  constexpr int S = RG_T + 8, R = RG_T + 2;
  __shared__ uint8_t se[S][S];
  __shared__ uint8_t h3[S][S], h7[S][S];  // horizontal maxima
  __shared__ uint8_t ring[R][R];
  const int tid = threadIdx.x;
  const int bx = blockIdx.x * RG_T, by = blockIdx.y * RG_T;
  for (int i = tid; i < S * S; i += 256) {
    const int yy = i / S, xx = i % S;
    const int r = by + yy - 4, c = bx + xx - 4;
    se[yy][xx] = (r >= 0 && r < H && c >= 0 && c < W) ? e[(long long)r * W + c] : 0;
  }
  __syncthreads();
  for (int i = tid; i < S * S; i += 256) {
    const int yy = i / S, xx = i % S;
    uint8_t m3 = 0, m7 = 0;
    for (int d = -3; d <= 3; ++d) {
      const int x2 = xx + d;
      if (x2 < 0 || x2 >= S) continue;
      const uint8_t v = se[yy][x2];
      m7 = max(m7, v);
      if (d >= -1 && d <= 1) m3 = max(m3, v);
    }
    h3[yy][xx] = m3;
    h7[yy][xx] = m7;
  }
  __syncthreads();
  // ring at tile positions -1..RG_T (clamped into the frame for the replicated median border)
  for (int i = tid; i < R * R; i += 256) {
    const int yy = i / R, xx = i % R;
    const int r = min(max(by + yy - 1, 0), H - 1), c = min(max(bx + xx - 1, 0), W - 1);
    const int sy = r - by + 4, sx = c - bx + 4;  // inside the staged halo: |offset| <= 1
    uint8_t m3 = 0, m7 = 0;
    for (int d = -3; d <= 3; ++d) {
      const int y2 = sy + d;
      if (y2 < 0 || y2 >= S) continue;
      m7 = max(m7, h7[y2][sx]);
      if (d >= -1 && d <= 1) m3 = max(m3, h3[y2][sx]);
    }
    ring[yy][xx] = (uint8_t)(m7 > m3 ? (m7 - m3) : 0);
  }
  __syncthreads();
  for (int i = tid; i < RG_T * RG_T; i += 256) {
    const int yy = i / RG_T, xx = i % RG_T;
    const int r = by + yy, c = bx + xx;
    if (r >= H || c >= W) continue;
    // 3x3 median of a {0, v} image: v if at least 5 of the 9 samples are nonzero
    int cnt = 0;
    uint8_t v = 0;
    for (int dy = 0; dy < 3; ++dy)
      for (int dx = 0; dx < 3; ++dx) {
        const uint8_t s = ring[yy + dy][xx + dx];
        cnt += s != 0;
        v = max(v, s);
      }
    mask[(long long)r * W + c] = cnt >= 5 ? v : 0;
  }
}

// ---- marker numbering: first 2x2 block of each component, block-raster order ---------------
__device__ __forceinline__ int block_key(long long p, int W) {
  const int r = (int)(p / W), c = (int)(p - (long long)(p / W) * W);
  return (r >> 1) * ((W + 1) >> 1) + (c >> 1);
}

__global__ __launch_bounds__(256) void k_cc_minkey(const int* __restrict__ L, int* __restrict__ K,
                                                   long long N, int W) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const int l = L[p];
    if (l >= 0) atomicMin(K + l, block_key(p, W));
  }
}

__global__ __launch_bounds__(256) void k_cc_firstflag(const int* __restrict__ L, const int* __restrict__ K,
                                                      int* __restrict__ F, long long N, int W) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const int l = L[p];
    if (l >= 0 && (long long)l == p) F[K[l]] = 1;  // one root per component
  }
}

__global__ __launch_bounds__(256) void k_cc_label(const int* __restrict__ L, const int* __restrict__ K,
                                                  const int* __restrict__ P, int32_t* __restrict__ out,
                                                  long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
    const int l = L[p];
    out[p] = l >= 0 ? P[K[l]] + 1 : 0;
  }
}

// ---- holes: background components (4-connected) that do not touch the frame ----------------
__global__ __launch_bounds__(256) void k_hole_border(const int* __restrict__ L, uint8_t* __restrict__ flag,
                                                     int H, int W) {
  const long long nb = 2ll * W + 2ll * H;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride) {
    long long p;
    if (i < W) p = i;
    else if (i < 2ll * W) p = (long long)(H - 1) * W + (i - W);
    else if (i < 2ll * W + H) p = (i - 2ll * W) * W;
    else p = (i - 2ll * W - H) * W + (W - 1);
    const int l = L[p];
    if (l >= 0) flag[l] = 1;
  }
}

__global__ __launch_bounds__(256) void k_hole_count(const int* __restrict__ L, const uint8_t* __restrict__ flag,
                                                    int* __restrict__ count, long long N) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  int n = 0;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride)
    if (L[p] == (int)p && !flag[p]) ++n;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(count, n);
}

}  // namespace msg
