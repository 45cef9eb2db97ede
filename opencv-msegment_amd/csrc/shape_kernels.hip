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
// Block = one wave = 64 columns, rows [r0, r0 + MED_ROWS).  Each thread's window histogram lives
// in LDS as 16-bit counts, two threads' bins per dword (lane pair), updated with no-return ds_add
// (a decrement adds 0xFFFF / 0xFFFF0000: the bin holds the removed sample, so no borrow crosses
// halves).  The median m is tracked with lt = #samples < m: each update adjusts lt, then m moves
// until lt <= half < lt + hist[m].  The two rows a step needs (leaving, entering) are fetched
// for the whole wave's column span (64 + k - 1 bytes) one step AHEAD into registers, staged in
// LDS, and read from there: one global round trip per step, overlapped with the step before.
constexpr int MED_BS = 64;
constexpr int MED_ROWS = 128;
constexpr int MED_SPAN = MED_BS + 256;  // span bytes for k <= 255 (64 + k - 1 <= 318)
constexpr int MED_Q = (MED_SPAN + MED_BS - 1) / MED_BS;  // bytes fetched per lane per row

__device__ __forceinline__ int med_bin(const unsigned* h, int v, int lane) {
  const unsigned w = h[v * (MED_BS / 2) + (lane >> 1)];
  return (int)((lane & 1) ? (w >> 16) : (w & 0xffffu));
}

__global__ __launch_bounds__(MED_BS) void k_median(const uint8_t* __restrict__ src,
                                                   uint8_t* __restrict__ dst, int H, int W, int k) {
  __shared__ unsigned hist[256 * (MED_BS / 2)];
  __shared__ uint8_t rows[2][MED_SPAN];  // [leaving, entering] row of the current step
  const int lane = threadIdx.x;
  const int x = blockIdx.x * MED_BS + lane;
  const int r0 = blockIdx.y * MED_ROWS;
  const int r1 = min(H, r0 + MED_ROWS);
  for (int i = lane; i < 256 * (MED_BS / 2); i += MED_BS) hist[i] = 0;
  const bool on = x < W;
  const int h = k >> 1, half = (k * k) >> 1;
  const int xs = blockIdx.x * MED_BS - h, span = MED_BS + 2 * h;
  const unsigned one = (lane & 1) ? 0x10000u : 1u;
  const unsigned minus = (lane & 1) ? 0xffff0000u : 0xffffffffu;
  unsigned* const hcol = hist + (lane >> 1);
  auto fetch = [&](int r, uint8_t (&v)[MED_Q]) {  // span bytes of row r (clamped) into registers
    const uint8_t* row = src + (long long)min(max(r, 0), H - 1) * W;
#pragma unroll
    for (int q = 0; q < MED_Q; ++q) {
      const int j = lane + MED_BS * q;
      v[q] = (j < span) ? row[min(max(xs + j, 0), W - 1)] : 0;
    }
  };
  auto stage = [&](int slot, const uint8_t (&v)[MED_Q]) {
#pragma unroll
    for (int q = 0; q < MED_Q; ++q) {
      const int j = lane + MED_BS * q;
      if (j < span) rows[slot][j] = v[q];
    }
  };
  __syncthreads();
  // initial window: rows r0 - h .. r0 + h, each staged then added
  uint8_t a[MED_Q], b[MED_Q];
  fetch(r0 - h, a);
  for (int r = r0 - h; r <= r0 + h; ++r) {
    stage(0, a);
    if (r < r0 + h) fetch(r + 1, a);
    __syncthreads();
    if (on) {
#pragma unroll 8
      for (int j = 0; j < k; ++j) atomicAdd(&hcol[rows[0][lane + j] * (MED_BS / 2)], one);
    }
    __syncthreads();
  }
  int m = 0, lt = 0;
  if (on) {
    int acc = 0;
    for (;;) {
      const int c = med_bin(hist, m, lane);
      if (acc + c > half) break;
      acc += c;
      ++m;
    }
    lt = acc;
    dst[(long long)r0 * W + x] = (uint8_t)m;
  }
  if (r0 + 1 < r1) {
    fetch(r0 - h, a);
    fetch(r0 + 1 + h, b);
  }
  for (int r = r0 + 1; r < r1; ++r) {
    stage(0, a);
    stage(1, b);
    if (r + 1 < r1) {  // next step's rows, in flight while this step runs
      fetch(r - h, a);
      fetch(r + 1 + h, b);
    }
    __syncthreads();
    if (on) {
#pragma unroll 8
      for (int j = 0; j < k; ++j) {
        const int vo = rows[0][lane + j], vi = rows[1][lane + j];
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
      dst[(long long)r * W + x] = (uint8_t)m;
    }
    __syncthreads();
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

// Tiled labelling: k_ccl_local labels each 32 x 32 tile in LDS (same union-find, workgroup
// scope) and writes every pixel's tile-local root as its global parent (the local root is the
// smallest global index of that tile's part of the component); k_ccl_boundary then unions only
// the pairs that cross a tile border (pixels in a tile's top row, left or right column), and
// k_ccl_compress points every pixel at its final root.
constexpr int CT = 32;

__device__ __forceinline__ int lfind(int* lp, int x) {
  int y = __hip_atomic_load(lp + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (y != x) {
    x = y;
    y = __hip_atomic_load(lp + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  return x;
}

__device__ __forceinline__ void lunion(int* lp, int a, int b) {
  a = lfind(lp, a);
  b = lfind(lp, b);
  while (a != b) {
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    const int old = atomicMin(lp + a, b);
    if (old == a) return;
    a = lfind(lp, old);
    b = lfind(lp, b);
  }
}

__global__ __launch_bounds__(256) void k_ccl_local(const uint8_t* __restrict__ a, int* __restrict__ L,
                                                   int H, int W, int mode) {
  __shared__ int lp[CT * CT];
  __shared__ uint8_t fg[CT * CT];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * CT, y0 = blockIdx.y * CT;
  for (int i = tid; i < CT * CT; i += 256) {
    const int r = y0 + i / CT, c = x0 + i % CT;
    const bool on = r < H && c < W && ccl_fg(a, (long long)r * W + c, mode);
    fg[i] = on;
    lp[i] = on ? i : -1;
  }
  __syncthreads();
  for (int i = tid; i < CT * CT; i += 256) {
    if (!fg[i]) continue;
    const int r = i / CT, c = i % CT;
    if (c > 0 && fg[i - 1]) lunion(lp, i, i - 1);
    if (r > 0) {
      if (fg[i - CT]) lunion(lp, i, i - CT);
      if (mode != 2) {
        if (c > 0 && fg[i - CT - 1]) lunion(lp, i, i - CT - 1);
        if (c + 1 < CT && fg[i - CT + 1]) lunion(lp, i, i - CT + 1);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < CT * CT; i += 256) {
    const int r = y0 + i / CT, c = x0 + i % CT;
    if (r >= H || c >= W) continue;
    int v = -1;
    if (fg[i]) {
      const int root = lfind(lp, i);
      v = (y0 + root / CT) * W + x0 + root % CT;
    }
    L[(long long)r * W + c] = v;
  }
}

// One block per tile, one thread per border pixel that has a previous neighbour (left, up-left,
// up, up-right) in another tile: the 32 pixels of the top row, then the left and the right
// column below it.
__global__ __launch_bounds__(128) void k_ccl_boundary(const uint8_t* __restrict__ a, int* L, int H, int W,
                                                      int mode) {
  const int t = threadIdx.x;
  if (t >= 3 * CT - 2) return;
  const int x0 = blockIdx.x * CT, y0 = blockIdx.y * CT;
  int r, c;
  if (t < CT) {
    r = y0;
    c = x0 + t;
  } else if (t < 2 * CT - 1) {
    r = y0 + 1 + (t - CT);
    c = x0;
  } else {
    r = y0 + 1 + (t - (2 * CT - 1));
    c = x0 + CT - 1;
  }
  if (r >= H || c >= W) return;
  const long long p = (long long)r * W + c;
  if (!ccl_fg(a, p, mode)) return;
  const bool top = r == y0, left = c == x0, right = c == x0 + CT - 1;
  if (c > 0 && left && ccl_fg(a, p - 1, mode)) ccl_union(L, (int)p, (int)(p - 1));
  if (r > 0) {
    if (top && ccl_fg(a, p - W, mode)) ccl_union(L, (int)p, (int)(p - W));
    if (mode != 2) {
      if (c > 0 && (top || left) && ccl_fg(a, p - W - 1, mode)) ccl_union(L, (int)p, (int)(p - W - 1));
      if (c + 1 < W && (top || right) && ccl_fg(a, p - W + 1, mode)) ccl_union(L, (int)p, (int)(p - W + 1));
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
// 2-D grid: blockIdx.y = row, x over columns.  Only pixels with no 8-neighbour (of the same
// component, i.e. any foreground neighbour) in a block of smaller key contribute: the
// component's first block passes that test, and big components no longer pile every pixel's
// atomicMin onto their root's word.
__global__ __launch_bounds__(256) void k_cc_minkey(const int* __restrict__ L, int* __restrict__ K, int H,
                                                   int W) {
  const int r = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W) return;
  const int l = L[(long long)r * W + c];
  if (l < 0) return;
  const int bw = (W + 1) >> 1;
  const int key = (r >> 1) * bw + (c >> 1);
  for (int dr = -1; dr <= 1; ++dr) {
    const int rr = r + dr;
    if (rr < 0 || rr >= H) continue;
    for (int dc = -1; dc <= 1; ++dc) {
      const int cc = c + dc;
      if ((dr == 0 && dc == 0) || cc < 0 || cc >= W) continue;
      if ((rr >> 1) * bw + (cc >> 1) < key && L[(long long)rr * W + cc] >= 0) return;
    }
  }
  atomicMin(K + l, key);
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
