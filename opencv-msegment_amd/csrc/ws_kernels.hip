// ws_kernels.hip -- gfx950 kernels of the exact watershed flood.
//
// The reference hot path is OpenCV 3.4.2 cv::watershed (reached from
// PictureService.java:909) followed by PictureService.colorByIndexes (PictureService.java:913-936).
// cv::watershed is a serial 256-bucket FIFO priority flood.  This file re-derives
// it as a bucket-synchronous GENERATION engine that is exact by construction:
//
//   * a batch = the current contents of the lowest non-empty bucket L, in FIFO order (rank i);
//   * serially those pixels would be popped one after another, unless one of them pushes a
//     neighbour at a level < L ("interrupt"); the batch is therefore cut after the first item
//     that does so, and everything after the cut stays queued (exactly as in the serial run);
//   * inside a batch, item i sees (a) every already-labelled neighbour and (b) the labels of
//     earlier batch items adjacent to it; a 0-pixel is pushed by the earliest non-WSHED batch
//     item adjacent to it (first-push-wins), in (rank, direction L,R,T,B) order;
//   * the pushes of the committed prefix are appended to their buckets in (rank, dir) order by
//     an ordered multi-bucket append (per-chunk level histograms -> column scan -> stable
//     scatter), so every bucket stays in exact serial FIFO order.
//
// Data in HBM (N = rows*cols pixels; details in DESIGN.md section 4):
//   mk   i32[tiles*16] TILED pixel states, 4x4-pixel tiles in tile-row-major order, so one
//                  128-B line holds two horizontally adjacent tiles (8x4 pixels): state >0
//                  label, 0 unknown, -1 WSHED/frame, phase-1 marker, <= -3 queued at slot -3-s
//   w4   u32[tiles*16] the same tiling: the four L-inf BGR distances to the L,R,T,B neighbours
//                  (read only for a batch item itself, so the radius-2 state reads of
//                  k_resolve touch 32-pixel lines)
//   qbuf int32[..] 256 bucket FIFOs of tiled pixel indices, bucket L = qbuf[qbase[L] + head[L]
//                  .. qbase[L] + tail[L]), sized exactly by a per-level histogram of each
//                  pixel's distinct interior edge weights
//   tl   u64[N]    per-rank granule of the current batch: {epoch, label} or provisional
//   desc u64[N]    per-rank push descriptor: four 8-bit levels | mask << 32 | level | segment
//   ipx  int32[N]  per-rank pixel
// Per iteration: k_resolve (decide every item) -> k_scan (1 block: column scan, heads, next
// batch; small batches run here) -> k_scatter (commit labels, ordered append).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ws_shared.h"

namespace msg {

__device__ __forceinline__ int cdiff3(const uint8_t* a, const uint8_t* b) {
  int d0 = abs((int)a[0] - (int)b[0]);
  int d1 = abs((int)a[1] - (int)b[1]);
  int d2 = abs((int)a[2] - (int)b[2]);
  return max(max(d0, d1), d2);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}

// Wave-wide scans and reductions in DPP lane moves (row_shr 1/2/4/8 within each 16-lane row, then
// row_bcast 15/31 across rows): six VALU steps instead of six LDS-crossbar shuffles
// (ds_bpermute, ~50+ cycles each on a dependent chain).  The whole wave must be active.
__device__ __forceinline__ int wave_scan_add(int v) {  // inclusive
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ int wave_sum(int v) { return __builtin_amdgcn_readlane(wave_scan_add(v), 63); }
__device__ __forceinline__ int wave_min(int v) {
  constexpr int MAXI = 0x7fffffff;
  v = min(v, __builtin_amdgcn_update_dpp(MAXI, v, 0x111, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(MAXI, v, 0x112, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(MAXI, v, 0x114, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(MAXI, v, 0x118, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(MAXI, v, 0x142, 0xa, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(MAXI, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------
// Stand-alone colour-distance stencil (exposed as msg_edge_weights_dev; the same arithmetic is
// fused into k_prep): wr[p] = L-inf BGR distance to the right neighbour, wd[p] to the one below,
// 0 past the edge.  5 algorithmic bytes per pixel (3 in, 2 out).
//
// k_edge_weights16<R>: rows whose width is a multiple of 16 (and 16-B aligned buffers): one
// thread = a 16-pixel column segment of R rows: R + 1 rows of three 16-B loads (the extra row is
// the next strip's first), one dword per row for the right neighbour of pixel 15, one 16-B store
// per output row.  Blocks are renumbered XCD-aware (blocks b, b + 8, ... run on one XCD under
// round-robin placement and get consecutive strips), so the extra row is mostly the one that
// XCD's L2 just fetched for its neighbour strip.  The kernel is VALU-heavy for its bytes (6
// channel differences and 2 maxima per pixel), so every channel byte is extracted once per row
// and each |a - b| is one v_sad_u16 (operands < 2^16): 16.5 -> ~10 VALU ops per pixel, which
// took the 4096^2 launch from 18.1 to 14.7 us (R = 1; scripts/exp/stream_variants.hip).  Frames
// are < 2^29 pixels (check_size), so 32-bit offsets suffice (3N < 2^31).
// k_edge_weights: any shape, 4 pixels per thread.
__device__ __forceinline__ uint32_t absdiff(uint32_t x, uint32_t y) { return __builtin_amdgcn_sad_u16(x, y, 0u); }
__device__ __forceinline__ uint32_t linf_ch(const uint32_t* p, const uint32_t* q) {
  return max(max(absdiff(p[0], q[0]), absdiff(p[1], q[1])), absdiff(p[2], q[2]));
}
// the 17 pixels (16 + the right neighbour) of a row segment as channel values
__device__ __forceinline__ void unpack17(const uint32_t* w, uint32_t px[17][3]) {
#pragma unroll
  for (int k = 0; k < 17; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) px[k][c] = (w[(3 * k + c) >> 2] >> (8 * ((3 * k + c) & 3))) & 255u;
}

__device__ __forceinline__ void ld48(const uint8_t* p, uint32_t* w) {
  const uint4* a = reinterpret_cast<const uint4*>(p);
  const uint4 x0 = a[0], x1 = a[1], x2 = a[2];
  w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w;
  w[4] = x1.x; w[5] = x1.y; w[6] = x1.z; w[7] = x1.w;
  w[8] = x2.x; w[9] = x2.y; w[10] = x2.z; w[11] = x2.w;
}

template <int EW_ROWS>
__global__ __launch_bounds__(256) void k_edge_weights16(const uint8_t* __restrict__ img,
                                                        uint8_t* __restrict__ wr,
                                                        uint8_t* __restrict__ wd, int H, int W) {
  const unsigned segs = (unsigned)W >> 4;
  unsigned b = blockIdx.x;
  const unsigned per_xcd = gridDim.x / 8;
  if (b < per_xcd * 8) b = (b % 8) * per_xcd + b / 8;  // a bijection on the first 8*per_xcd blocks
  const unsigned t = b * blockDim.x + threadIdx.x;
  const unsigned strips = ((unsigned)H + EW_ROWS - 1) / EW_ROWS;
  if (t >= strips * segs) return;
  const unsigned st = t / segs, sx = t - st * segs;
  const int r0 = (int)st * EW_ROWS;
  const bool has_r = sx + 1 < segs;
  // every load of the strip first: EW_ROWS + 1 rows of 48 B, the right neighbours' first dwords
  uint32_t rows[EW_ROWS + 1][13];
#pragma unroll
  for (int i = 0; i <= EW_ROWS; ++i) {
    const int r = r0 + i;
    const unsigned p0 = (unsigned)r * (unsigned)W + 16u * sx;
#pragma unroll
    for (int k = 0; k < 13; ++k) rows[i][k] = 0;
    if (r < H) {
      ld48(img + 3u * p0, rows[i]);
      if (has_r && i < EW_ROWS) rows[i][12] = *reinterpret_cast<const uint32_t*>(img + 3u * (p0 + 16u));
    }
  }
  uint32_t cur[17][3], nxt[17][3];
  unpack17(rows[0], cur);
#pragma unroll
  for (int i = 0; i < EW_ROWS; ++i) {
    const int r = r0 + i;
    if (r >= H) break;
    const bool has_d = r + 1 < H;
    unpack17(rows[i + 1], nxt);
    uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t vr = (k < 15 || has_r) ? linf_ch(cur[k], cur[k + 1]) : 0u;
      const uint32_t vd = has_d ? linf_ch(cur[k], nxt[k]) : 0u;
      orr[k >> 2] |= vr << (8 * (k & 3));
      odd[k >> 2] |= vd << (8 * (k & 3));
    }
    const unsigned p0 = (unsigned)r * (unsigned)W + 16u * sx;
    *reinterpret_cast<uint4*>(wr + p0) = make_uint4(orr[0], orr[1], orr[2], orr[3]);
    *reinterpret_cast<uint4*>(wd + p0) = make_uint4(odd[0], odd[1], odd[2], odd[3]);
#pragma unroll
    for (int k = 0; k < 17; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) cur[k][c] = nxt[k][c];
  }
}

__global__ __launch_bounds__(256) void k_edge_weights(const uint8_t* __restrict__ img,
                                                      uint8_t* __restrict__ wr,
                                                      uint8_t* __restrict__ wd, int H, int W) {
  const long long N = (long long)H * W;
  const long long q = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (q >= N) return;
  for (int k = 0; k < 4; ++k) {
    const long long p = q + k;
    if (p >= N) break;
    const int r = (int)(p / W), c = (int)(p - (long long)r * W);
    const uint8_t* ip = img + p * 3;
    wr[p] = (c + 1 < W) ? (uint8_t)cdiff3(ip, ip + 3) : (uint8_t)0;
    wd[p] = (r + 1 < H) ? (uint8_t)cdiff3(ip, ip + 3 * (long long)W) : (uint8_t)0;
  }
}

// ---------------------------------------------------------------------------------------------
// Phase 0 + phase 1 of cv::watershed (border, sanitise, initial queue levels) fused with the
// colour-distance stencil and the bucket-capacity histogram.  One thread = one 4x4 tile (its
// states and weights written with 16-B stores into mk and w4), one block = a 4-row x RSEG-column
// strip, i.e. 4 raster chunks, whose phase-1 counts feed the raster-order compaction.
__device__ __forceinline__ uint32_t ld_bgr(const uint8_t* img, int r, int c, int H, int W) {
  if (r < 0 || r >= H || c < 0 || c >= W) return 0;
  const uint8_t* q = img + ((long long)r * W + c) * 3;
  return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
}

__device__ __forceinline__ int cdiffp(uint32_t a, uint32_t b) {  // L-inf BGR distance, packed
  const int d0 = abs((int)(a & 255u) - (int)(b & 255u));
  const int d1 = abs((int)((a >> 8) & 255u) - (int)((b >> 8) & 255u));
  const int d2 = abs((int)((a >> 16) & 255u) - (int)((b >> 16) & 255u));
  return max(max(d0, d1), d2);
}

constexpr int PREP_COLS = RSEG + 2;                  // strip columns incl. the 1-pixel halo
constexpr int PREP_LDW = RSEG + 5;                   // LDS row stride (words): conflict-free stencil
constexpr int PREP_RAW = (3 * PREP_COLS + 8) / 4 + 1;  // dwords of one BGR row segment

// thread = one tile row (4 pixels): tile tid >> 2, row tid & 3, so 4 consecutive lanes write one
// whole 128-B tile line; frames are < 2^29 pixels, so 32-bit offsets (3N < 2^31) suffice.
// The flood's zeroed state, written by the phase-0 kernel instead of two host memsets ahead of
// it (≈5 µs and a dependent launch each): the control block (block 0) and the per-chunk level
// histograms (a slice per block).  Neither is read before the next kernel.
__device__ __forceinline__ void prep_zero(const Ws& ws) {
  const int G = gridDim.x, b = blockIdx.x, T = blockDim.x, t = threadIdx.x;
  if (b == 0) {
    int* p = reinterpret_cast<int*>(ws.ctl);
    for (int k = t; k < (int)(sizeof(Ctl) / 4); k += T) p[k] = 0;
  }
  const long long ncnt = ((ws.N + CH - 1) / CH) * NQ;
  const long long per = (ncnt + G - 1) / G;
  const long long e = min((long long)(b + 1) * per, ncnt);
  for (long long k = (long long)b * per + t; k < e; k += T) ws.cnt[k] = 0;
}

__global__ __launch_bounds__(RSEG) void k_prep(Ws ws, const int32_t* __restrict__ mk_in) {
  static_assert(RSEG >= NQ && RSEG % 64 == 0 && PREP_RAW <= RSEG, "strip = RSEG/4 tiles x 4 rows = RSEG threads");
  __shared__ unsigned caph[NQ];
  __shared__ uint32_t s_raw[6][PREP_RAW];
  __shared__ uint32_t s_px[6][PREP_LDW];
  __shared__ int32_t s_m[6][PREP_LDW];
  __shared__ unsigned long long s_wsum[RSEG / 64];
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int H = ws.H, W = ws.W, Wt = ws.Wt;
  const int tr = blockIdx.x / ws.nseg, cs = blockIdx.x % ws.nseg;
  const int r0 = tr * 4, x0 = cs * RSEG;
  const int ncol = min(RSEG, W - x0) + 2;  // strip column j <-> image column x0 - 1 + j
  const int nbytes = 3 * H * W;
  prep_zero(ws);
  if (tid < NQ) caph[tid] = 0;
  // ---- stage rows r0-1..r0+4: all loads issued before the first LDS store ----
  const bool aligned = (((uintptr_t)ws.img) & 3) == 0;
  int a0[6];
  int mreg[6][2];
  uint32_t ireg[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int r = r0 - 1 + i;
    const bool rin = r >= 0 && r < H;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int j = tid + RSEG * it, c = x0 - 1 + j;
      mreg[i][it] = (rin && j < ncol && c >= 0 && c < W) ? mk_in[r * W + c] : 0;
    }
    const int ca = max(x0 - 1, 0), cb = min(x0 + ncol - 1, W);
    a0[i] = (3 * (r * W + ca)) & ~3;
    const int e = rin ? 3 * (r * W + cb) : a0[i];
    const int ad = a0[i] + 4 * tid;
    uint32_t w = 0;
    if (tid < PREP_RAW && ad < e) {
      if (aligned && ad + 4 <= nbytes) {
        w = *reinterpret_cast<const uint32_t*>(ws.img + ad);
      } else {
        for (int k = 0; k < 4; ++k)
          if (ad + k < nbytes) w |= (uint32_t)ws.img[ad + k] << (8 * k);
      }
    }
    ireg[i] = w;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int j = tid + RSEG * it;
      if (j < ncol) s_m[i][j] = mreg[i][it];
    }
    if (tid < PREP_RAW) s_raw[i][tid] = ireg[i];
  }
  __syncthreads();
  const uint8_t* rawb = reinterpret_cast<const uint8_t*>(&s_raw[0][0]);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int r = r0 - 1 + i;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int j = tid + RSEG * it;
      if (j >= ncol) continue;
      const int c = x0 - 1 + j;
      uint32_t v = 0;
      if (r >= 0 && r < H && c >= 0 && c < W) {
        const int o = 3 * (r * W + c) - a0[i] + i * PREP_RAW * 4;
        v = (uint32_t)rawb[o] | ((uint32_t)rawb[o + 1] << 8) | ((uint32_t)rawb[o + 2] << 16);
      }
      s_px[i][j] = v;
    }
  }
  __syncthreads();
  // ---- one tile row per thread ----
  const int tl = tid >> 2, ry = tid & 3;
  const int tc = cs * (RSEG / 4) + tl;
  const int r = r0 + ry, i = ry + 1;
  unsigned p1mask = 0;  // bit rx: phase-1 pixel
  int run_w = -1;
  unsigned run_n = 0;
  auto cap_add = [&](int w) {
    if (w != run_w) {
      if (run_n) atomicAdd(&caph[run_w], run_n);
      run_w = w;
      run_n = 0;
    }
    ++run_n;
  };
  if (tc < Wt) {
    const int c0 = tc * 4, jb = 4 * tl;  // strip column of c0 - 1
    int sv[4];
    unsigned wv4[4];
    // every channel byte extracted once (this row's 6 pixels, the 4 above and below), each
    // |a - b| one v_sad_u16, the horizontal distances shared by neighbouring pixels (k_prep was
    // VALU-bound at ~190 lane-ops per pixel with 4 packed distances per pixel)
    uint32_t cm[6][3], cu[4][3], cd[4][3];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint32_t px = s_px[i][jb + k];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) cm[k][ch] = (px >> (8 * ch)) & 255u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t pu = s_px[i - 1][jb + 1 + k], pd = s_px[i + 1][jb + 1 + k];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        cu[k][ch] = (pu >> (8 * ch)) & 255u;
        cd[k][ch] = (pd >> (8 * ch)) & 255u;
      }
    }
    int hd[5];  // distance between strip columns jb + k and jb + k + 1
#pragma unroll
    for (int k = 0; k < 5; ++k) hd[k] = (int)linf_ch(cm[k], cm[k + 1]);
#pragma unroll
    for (int rx = 0; rx < 4; ++rx) {
      const int c = c0 + rx, j = jb + rx + 1;
      int state = WSHED;
      unsigned w4 = 0;
      if (r < H && c < W) {
        const int wl = (c >= 1) ? hd[rx] : 0;
        const int wr = (c + 1 < W) ? hd[rx + 1] : 0;
        const int wu = (r >= 1) ? (int)linf_ch(cm[rx + 1], cu[rx]) : 0;
        const int wd = (r + 1 < H) ? (int)linf_ch(cm[rx + 1], cd[rx]) : 0;
        w4 = (unsigned)wl | ((unsigned)wr << 8) | ((unsigned)wu << 16) | ((unsigned)wd << 24);
        if (!(r == 0 || r == H - 1 || c == 0 || c == W - 1)) {
          const int m = s_m[i][j];
          if (m > 0) {
            state = m;
          } else {
            // interior neighbours (the frame is WSHED in the serial code and never counts)
            const int wleft = (c >= 2) ? wl : -1;
            const int wup = (r >= 2) ? wu : -1;
            const int wr_i = (c <= W - 3) ? wr : -1;
            const int wd_i = (r <= H - 3) ? wd : -1;
            int lvl = 256;
            if (wleft >= 0 && s_m[i][j - 1] > 0) lvl = min(lvl, wleft);
            if (wr_i >= 0 && s_m[i][j + 1] > 0) lvl = min(lvl, wr_i);
            if (wup >= 0 && s_m[i - 1][j] > 0) lvl = min(lvl, wup);
            if (wd_i >= 0 && s_m[i + 1][j] > 0) lvl = min(lvl, wd_i);
            if (lvl < 256) {
              state = p1_state(lvl);
              p1mask |= 1u << rx;
            } else {
              state = 0;
            }
            // this pixel may be queued once, at one of its distinct interior edge weights
            if (wleft >= 0) cap_add(wleft);
            if (wr_i >= 0 && wr_i != wleft) cap_add(wr_i);
            if (wup >= 0 && wup != wleft && wup != wr_i) cap_add(wup);
            if (wd_i >= 0 && wd_i != wleft && wd_i != wr_i && wd_i != wup) cap_add(wd_i);
          }
        }
      }
      sv[rx] = state;
      wv4[rx] = w4;
    }
    const long long to = ((long long)(tr * Wt + tc) << 4) + 4 * ry;
    *reinterpret_cast<int4*>(ws.mk + to) = make_int4(sv[0], sv[1], sv[2], sv[3]);
    *reinterpret_cast<int4*>(ws.w4 + to) = make_int4((int)wv4[0], (int)wv4[1], (int)wv4[2], (int)wv4[3]);
  }
  if (run_n) atomicAdd(&caph[run_w], run_n);
  // ---- phase-1 pixels of each of the 4 raster chunks (rows), in raster order, into scratch at
  // the chunk's raster offset in qbuf (read by k_compact; qbuf is filled only after it):
  // segmented exclusive scan, row ry's count in bits 16*ry of a 64-bit word ----
  const unsigned long long mine = (unsigned long long)__popc(p1mask) << (16 * ry);
  // the four 16-bit row counts never carry into each other (at most 4 per lane, 64 lanes), so the
  // 64-bit scan is two 32-bit DPP scans
  const unsigned long long x =
      (unsigned long long)(uint32_t)wave_scan_add((int)(uint32_t)mine) |
      ((unsigned long long)(uint32_t)wave_scan_add((int)(uint32_t)(mine >> 32)) << 32);
  if (lane == 63) s_wsum[wv] = x;
  __syncthreads();
  unsigned long long excl = x - mine, total = 0;
  for (int k = 0; k < RSEG / 64; ++k) {
    if (k < wv) excl += s_wsum[k];
    total += s_wsum[k];
  }
  if (p1mask) {
    int q = r * W + x0 + (int)((excl >> (16 * ry)) & 0xffff);
    const int t0 = ((tr * Wt + tc) << 4) + 4 * ry;
#pragma unroll
    for (int rx = 0; rx < 4; ++rx)
      if ((p1mask >> rx) & 1u) ws.qbuf[q++] = t0 + rx;
  }
  if (tid < NQ && caph[tid]) atomicAdd(&ws.capp[(blockIdx.x % CAP_SLOTS) * NQ + tid], caph[tid]);
  if (tid < 4 && r0 + tid < H) ws.tot[(r0 + tid) * ws.nseg + cs] = (int)((total >> (16 * tid)) & 0xffff);
}

// k_prep4: the same phase 0/1 + stencil + histogram for rows whose width is a multiple of 4 (and
// 4-B aligned BGR, 16-B aligned markers), one thread per 4x4 tile instead of per tile row.  Each
// thread loads its own 12-B pixel quads and 16-B marker quads of the 6 rows r0-1..r0+4 straight
// from global memory (lane-contiguous), shares only its first and last column through LDS (the
// neighbours' halo), extracts every channel once and computes the 20 horizontal and 20 vertical
// distances of its tile once each (a tile-row thread recomputed the vertical ones of 3 rows and
// rebuilt packed pixels in LDS): about half of k_prep's VALU instructions per pixel.  Same
// outputs, same raster chunks (a block is still a 4-row x RSEG-column strip), same capacity
// histogram.  Halving the VALU work alone moved 118 -> 110 us at 4096^2 (PMC: 51% of wave
// cycles waiting on memory, 9% VALU-active); what bounded it was the write pattern -- a tile per
// thread stored 16 B per lane at a 64-B stride doubled the HBM writes (283 MB against 128) --
// so the tiles now go out lane-contiguously through the halo's LDS: 89 us, 138 MB written.
constexpr int PREP4_T = RSEG / 4;  // threads per block = tiles per strip

struct alignas(4) Quad3 { uint32_t x, y, z; };

// the halo columns while the tiles are computed, then the strip's tiles for the coalesced stores
union Prep4Lds {
  struct {
    uint32_t pf[6][PREP4_T + 2], pb[6][PREP4_T + 2];  // each tile's first / last pixel
    int32_t mf[6][PREP4_T + 2], mb[6][PREP4_T + 2];   // and their markers
  } h;
  int4 tile[4 * PREP4_T];
};

// One row of a thread's tile column as loaded: 4 BGR pixels (12 B), 4 markers, and for the two
// halo threads the strip's outside column (x0 - 1 or x0 + RSEG).
struct Prep4Row {
  Quad3 q;
  int4 m;
  uint32_t hv;
  int hm;
};

__device__ __forceinline__ Prep4Row prep4_load(const Ws& ws, const int32_t* __restrict__ mk_in, int r, int c0,
                                               bool tin, bool halo, int hc) {
  const int H = ws.H, W = ws.W;
  Prep4Row x;
  x.q = Quad3{0, 0, 0};
  x.m = make_int4(0, 0, 0, 0);
  x.hv = 0;
  x.hm = 0;
  if (r < 0 || r >= H) return x;
  if (tin) {
    const unsigned o = (unsigned)r * (unsigned)W + (unsigned)c0;
    x.q = *reinterpret_cast<const Quad3*>(ws.img + 3u * o);
    x.m = *reinterpret_cast<const int4*>(mk_in + o);
  }
  if (halo && hc >= 0 && hc < W) {
    const unsigned o = (unsigned)r * (unsigned)W + (unsigned)hc;
    x.hv = (uint32_t)ws.img[3u * o] | ((uint32_t)ws.img[3u * o + 1] << 8) | ((uint32_t)ws.img[3u * o + 2] << 16);
    x.hm = mk_in[o];
  }
  return x;
}

__global__ __launch_bounds__(PREP4_T) void k_prep4(Ws ws, const int32_t* __restrict__ mk_in) {
  __shared__ unsigned caph[NQ];
  __shared__ Prep4Lds u;
  __shared__ unsigned long long s_wsum[PREP4_T / 64];
  auto& s_pf = u.h.pf;
  auto& s_pb = u.h.pb;
  auto& s_mf = u.h.mf;
  auto& s_mb = u.h.mb;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int H = ws.H, W = ws.W, Wt = ws.Wt;
  const int tr = blockIdx.x / ws.nseg, cs = blockIdx.x % ws.nseg;
  const int r0 = tr * 4, x0 = cs * RSEG;
  const int tc = cs * PREP4_T + tid, c0 = tc * 4;
  const bool tin = c0 < W;  // W % 4 == 0: a tile is wholly inside or wholly outside
  const bool halo = (tid == 0 || tid == PREP4_T - 1);  // the strip's halo columns x0 - 1 and x0 + RSEG
  const int hc = (tid == 0) ? x0 - 1 : x0 + RSEG;
  for (int k = tid; k < NQ; k += PREP4_T) caph[k] = 0;
  // every load of the strip -- its rows and the two halo threads' outside columns -- issued before
  // the first use: one round trip (the halo columns in a branch after the rows' LDS stores were a
  // second one: 81-84 -> 72-75 us at 4096^2, profiles/r03n_ab_prep_commit.log "tr1")
  Prep4Row rw[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) rw[i] = prep4_load(ws, mk_in, r0 - 1 + i, c0, tin, halo, hc);
  prep_zero(ws);  // (stores issued while the loads are in flight)
  uint32_t px[6][4];
  int mm[6][4];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const Quad3 q = rw[i].q;
    const int4 m4 = rw[i].m;
    px[i][0] = q.x & 0xffffffu;
    px[i][1] = (q.x >> 24) | ((q.y & 0xffffu) << 8);
    px[i][2] = (q.y >> 16) | ((q.z & 0xffu) << 16);
    px[i][3] = q.z >> 8;
    mm[i][0] = m4.x; mm[i][1] = m4.y; mm[i][2] = m4.z; mm[i][3] = m4.w;
    s_pf[i][tid + 1] = px[i][0];
    s_pb[i][tid + 1] = px[i][3];
    s_mf[i][tid + 1] = m4.x;
    s_mb[i][tid + 1] = m4.w;
  }
  if (halo) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      if (tid == 0) {
        s_pb[i][0] = rw[i].hv;
        s_mb[i][0] = rw[i].hm;
      } else {
        s_pf[i][PREP4_T + 1] = rw[i].hv;
        s_mf[i][PREP4_T + 1] = rw[i].hm;
      }
    }
  }
  __syncthreads();
  // distances from packed pixels, channels extracted per use (registers, not VALU, bound the
  // occupancy of this latency-bound kernel)
  auto dist = [](uint32_t a, uint32_t b) -> int {
    const uint32_t pa[3] = {a & 255u, (a >> 8) & 255u, (a >> 16) & 255u};
    const uint32_t pb[3] = {b & 255u, (b >> 8) & 255u, (b >> 16) & 255u};
    return (int)linf_ch(pa, pb);
  };
  int run_w = -1;
  unsigned run_n = 0;
  auto cap_add = [&](int w) {
    if (w != run_w) {
      if (run_n) atomicAdd(&caph[run_w], run_n);
      run_w = w;
      run_n = 0;
    }
    ++run_n;
  };
  unsigned p1m[4] = {0, 0, 0, 0};
  int sv[4][4];
  unsigned wq[4][4];
  if (tin) {
    int vdn[5][4];  // distance between rows i and i + 1 at pixel k
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) vdn[i][k] = dist(px[i][k], px[i + 1][k]);
#pragma unroll
    for (int ry = 0; ry < 4; ++ry) {
      const int r = r0 + ry, i = ry + 1;
      int hd[5];
      hd[0] = dist(s_pb[i][tid], px[i][0]);
#pragma unroll
      for (int k = 1; k < 4; ++k) hd[k] = dist(px[i][k - 1], px[i][k]);
      hd[4] = dist(px[i][3], s_pf[i][tid + 2]);
      const int mlh = s_mb[i][tid], mrh = s_mf[i][tid + 2];
#pragma unroll
      for (int rx = 0; rx < 4; ++rx) {
        const int c = c0 + rx;
        int state = WSHED;
        unsigned w4 = 0;
        if (r < H) {
          const int wl = (c >= 1) ? hd[rx] : 0;
          const int wr = (c + 1 < W) ? hd[rx + 1] : 0;
          const int wu = (r >= 1) ? vdn[ry][rx] : 0;
          const int wd = (r + 1 < H) ? vdn[ry + 1][rx] : 0;
          w4 = (unsigned)wl | ((unsigned)wr << 8) | ((unsigned)wu << 16) | ((unsigned)wd << 24);
          if (!(r == 0 || r == H - 1 || c == 0 || c == W - 1)) {
            const int m = mm[i][rx];
            if (m > 0) {
              state = m;
            } else {
              const int wleft = (c >= 2) ? wl : -1;
              const int wup = (r >= 2) ? wu : -1;
              const int wr_i = (c <= W - 3) ? wr : -1;
              const int wd_i = (r <= H - 3) ? wd : -1;
              const int ml = (rx > 0) ? mm[i][rx - 1] : mlh;
              const int mr = (rx < 3) ? mm[i][rx + 1] : mrh;
              int lvl = 256;
              if (wleft >= 0 && ml > 0) lvl = min(lvl, wleft);
              if (wr_i >= 0 && mr > 0) lvl = min(lvl, wr_i);
              if (wup >= 0 && mm[i - 1][rx] > 0) lvl = min(lvl, wup);
              if (wd_i >= 0 && mm[i + 1][rx] > 0) lvl = min(lvl, wd_i);
              if (lvl < 256) {
                state = p1_state(lvl);
                p1m[ry] |= 1u << rx;
              } else {
                state = 0;
              }
              if (wleft >= 0) cap_add(wleft);
              if (wr_i >= 0 && wr_i != wleft) cap_add(wr_i);
              if (wup >= 0 && wup != wleft && wup != wr_i) cap_add(wup);
              if (wd_i >= 0 && wd_i != wleft && wd_i != wr_i && wd_i != wup) cap_add(wd_i);
            }
          }
        }
        sv[ry][rx] = state;
        wq[ry][rx] = w4;
      }
    }
  }
  if (run_n) atomicAdd(&caph[run_w], run_n);
  // phase-1 pixels of the strip's 4 raster chunks in raster order (as k_prep): row ry's count
  // in bits 16 * ry of a 64-bit word, scanned over the tiles
  unsigned long long mine = 0;
#pragma unroll
  for (int ry = 0; ry < 4; ++ry) mine |= (unsigned long long)__popc(p1m[ry]) << (16 * ry);
  // the four 16-bit row counts never carry into each other (at most 4 per lane, 64 lanes), so the
  // 64-bit scan is two 32-bit DPP scans
  const unsigned long long x =
      (unsigned long long)(uint32_t)wave_scan_add((int)(uint32_t)mine) |
      ((unsigned long long)(uint32_t)wave_scan_add((int)(uint32_t)(mine >> 32)) << 32);
  if (lane == 63) s_wsum[wv] = x;
  __syncthreads();
  unsigned long long excl = x - mine, total = 0;
#pragma unroll
  for (int k = 0; k < PREP4_T / 64; ++k) {
    if (k < wv) excl += s_wsum[k];
    total += s_wsum[k];
  }
#pragma unroll
  for (int ry = 0; ry < 4; ++ry) {
    if (!p1m[ry]) continue;
    const int r = r0 + ry;
    int q = r * W + x0 + (int)((excl >> (16 * ry)) & 0xffff);
    const int t0 = ((tr * Wt + tc) << 4) + 4 * ry;
#pragma unroll
    for (int rx = 0; rx < 4; ++rx)
      if ((p1m[ry] >> rx) & 1u) ws.qbuf[q++] = t0 + rx;
  }
  for (int k = tid; k < NQ; k += PREP4_T)
    if (caph[k]) atomicAdd(&ws.capp[(blockIdx.x % CAP_SLOTS) * NQ + k], caph[k]);
  if (tid < 4 && r0 + tid < H) ws.tot[(r0 + tid) * ws.nseg + cs] = (int)((total >> (16 * tid)) & 0xffff);
  // the strip's tiles are contiguous in mk / w4 (tile-row-major): stored lane-contiguously through
  // LDS (a tile per thread stored 16 B per lane at a 64-B stride, and the partial lines were
  // written back separately: 283 MB of HBM writes per 4096^2 frame against 128 MB)
  const int ntile = min(PREP4_T, Wt - cs * PREP4_T);  // tiles of this strip inside the frame
  const unsigned base = (unsigned)(tr * Wt + cs * PREP4_T) << 4;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    __syncthreads();  // the halo columns (a = 0) / the previous array's chunks (a = 1) are consumed
    if (tin) {
#pragma unroll
      for (int ry = 0; ry < 4; ++ry)
        u.tile[4 * tid + ry] = a == 0 ? make_int4(sv[ry][0], sv[ry][1], sv[ry][2], sv[ry][3])
                                      : make_int4((int)wq[ry][0], (int)wq[ry][1], (int)wq[ry][2], (int)wq[ry][3]);
    }
    __syncthreads();
    int32_t* const dst = a == 0 ? ws.mk : ws.w4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = k * PREP4_T + tid;  // 16-B chunk: tile q / 4, tile row q % 4
      if (q < 4 * ntile) *reinterpret_cast<int4*>(dst + base + 4u * q) = u.tile[q];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Column scan: coff[c][lv] = tail[lv] + sum_{c' < c} cnt[c'][lv]   (c < nch), tail += totals.
// `partial` (LDS, may be null) replaces the counts of the last chunk.  1024 threads.
__device__ void column_scan(const int* cnt, int* coff, int nch, const int* partial, int* tail) {
  __shared__ int gs[4][NQ];
  constexpr int MAXR = 32;  // per-thread chunk values kept in registers (nch <= 128)
  const int tid = threadIdx.x;
  const int lv = tid & (NQ - 1), g = tid >> 8;
  const int per = (nch + 3) >> 2;
  const int a = min(nch, g * per), b = min(nch, a + per);
  if (per <= MAXR) {
    int v[MAXR];
#pragma unroll
    for (int k = 0; k < MAXR; ++k) {  // all loads issued back to back
      const int c = a + k;
      v[k] = (c < b) ? ((partial && c == nch - 1) ? partial[lv] : cnt[(long long)c * NQ + lv]) : 0;
    }
    int sum = 0;
#pragma unroll
    for (int k = 0; k < MAXR; ++k) sum += v[k];
    gs[g][lv] = sum;
    __syncthreads();
    int base = tail[lv];
    for (int k = 0; k < g; ++k) base += gs[k][lv];
#pragma unroll
    for (int k = 0; k < MAXR; ++k) {
      if (a + k < b) coff[(long long)(a + k) * NQ + lv] = base;
      base += v[k];
    }
  } else {
    int sum = 0;
    for (int c = a; c < b; ++c) sum += (partial && c == nch - 1) ? partial[lv] : cnt[(long long)c * NQ + lv];
    gs[g][lv] = sum;
    __syncthreads();
    int base = tail[lv];
    for (int k = 0; k < g; ++k) base += gs[k][lv];
    for (int c = a; c < b; ++c) {
      coff[(long long)c * NQ + lv] = base;
      base += (partial && c == nch - 1) ? partial[lv] : cnt[(long long)c * NQ + lv];
    }
  }
  __syncthreads();
  if (g == 0) tail[lv] += gs[0][lv] + gs[1][lv] + gs[2][lv] + gs[3][lv];
  __syncthreads();
}

__device__ int block_sum(int v) {  // every thread of the block calls; result to all
  __shared__ int part[32];
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane_id() == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = 0;
  for (int k = 0; k < nw; ++k) r += part[k];
  __syncthreads();
  return r;
}

// Next batch from the queue state (global or LDS arrays).  Block-wide, >= 64 threads, wave 0
// does the work; result in segs[0..*nseg) and *ntot (LDS), visible after the caller's barrier.
// The batch is the lowest non-empty bucket, extended by the following non-empty buckets (in level
// order, total <= MERGE_CAP) when `minpush` -- the lowest level the previous batch pushed -- is
// above that lowest level: a batch that did not feed its own or a lower level is unlikely to
// start a generation, so later segments are unlikely to be cut (the cut rules keep it exact).
__device__ void form_batch(const int* qbase, const int* head, const int* tail, int minpush,
                           int wcap, Seg* segs, int* nseg_out, int* n_out) {
  const int capn = (wcap > 0 && wcap < MERGE_CAP) ? wcap : MERGE_CAP;
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  int cnt[4];
  int ne = 0, sum = 0, lo = NQ;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int l = lane * 4 + k;
    cnt[k] = tail[l] - head[l];
    if (cnt[k] > 0) {
      ++ne;
      sum += cnt[k];
      lo = min(lo, l);
    }
  }
  const int xe = wave_scan_add(ne), xs = wave_scan_add(sum);
  lo = wave_min(lo);
  const bool merge = minpush > lo;
  int segi = xe - ne, cum = xs - sum, inc_n = 0, inc_items = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (cnt[k] <= 0) continue;
    const int l = lane * 4 + k;
    const bool inc = (segi == 0) || (merge && cum + cnt[k] <= capn);
    if (inc) {
      Seg s;
      s.L = l;
      s.bstart = qbase[l] + head[l];
      s.rank = cum;
      s.n = (segi == 0) ? min(cnt[k], capn) : cnt[k];  // the window truncates the first segment
      segs[segi] = s;
      ++inc_n;
      inc_items += s.n;
    }
    cum += cnt[k];
    ++segi;
  }
  inc_n = wave_sum(inc_n);
  inc_items = wave_sum(inc_items);
  if (lane == 0) {
    *nseg_out = inc_n;
    *n_out = inc_items;
  }
}

// A batch the two-launch iterations (k_resolve -> k_commit_fast) suit: a flood batch too large
// for k_scan's one-workgroup loop, and within k_commit_fast's chunk limit: 1 within FAST_CH chunks
// (k_commit_fast), 2 within FAST_PASS * FAST_CH (k_commit_fast_mp), 0 otherwise.  A batch the
// commit declined (hold) is k_scan's: 0, so that the host goes back to three-launch iterations.
__device__ __forceinline__ int fast_batch(const Batch& b, const Ctl* ctl) {
  if (b.mode != 0 || b.n <= SMALL_MAX || ctl->hold == b.epoch) return 0;
  return b.n <= FAST_CH * CH ? 1 : b.n <= FAST_PASS * FAST_CH * CH ? 2 : 0;
}

// rank -> segment (segments sorted by rank); slot -> batch rank or -1 (sorted by bstart too:
// bucket regions are laid out in level order).
__device__ __forceinline__ int seg_of_rank(const Seg* s, int nseg, int r) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s[mid].rank <= r) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
__device__ __forceinline__ int rank_of_slot(const Seg* s, int nseg, int slot) {
  if (nseg == 1) {
    const int r = slot - s[0].bstart;
    return (r >= 0 && r < s[0].n) ? r : -1;
  }
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s[mid].bstart <= slot) lo = mid;
    else hi = mid - 1;
  }
  const int off = slot - s[lo].bstart;
  return (off >= 0 && off < s[lo].n) ? s[lo].rank + off : -1;
}
// First segment after `sg` whose level is above t (NONE if none): the batch must end before it
// when an item of segment sg pushes at level t (those pushes are popped before that bucket).
__device__ __forceinline__ int seg_cut_for(const Seg* s, int nseg, int sg, int t) {
  int lo = sg + 1, hi = nseg;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid].L > t) hi = mid;
    else lo = mid + 1;
  }
  return lo < nseg ? lo : NONE;
}

__device__ __forceinline__ void load_segs(const Ctl* ctl, const Batch& B, Seg* s) {
  for (int k = threadIdx.x; k < B.nseg; k += blockDim.x) s[k] = ctl->seg[k];
}

// Turn the next batch into a speculative generation (k_spec_round): the whole lowest bucket L
// (navail items from bstart, at most SPEC_WIN), round tags continuing from the last round.
// One thread; nb.epoch is already set.
__device__ void spec_begin(Ctl* ctl, Batch& nb, int L, int bstart, int navail) {
  SpecCtl& s = ctl->spec;
  nb.mode = 3;
  nb.nseg = 1;
  nb.L = L;
  nb.bstart = bstart;
  nb.n = min(navail, SPEC_WIN);
  nb.ncommit = 0;
  nb.nchunk = 0;
  nb.rrun = 0;
  s.G = s.T + 1;
  s.T = s.G;
  s.L = L;
  s.n = nb.n;
  s.bstart = bstart;
  s.P = 0;
  s.Pold = 0;
  s.Pprom = 0;
  s.rounds = 1;
  s.state = 1;
  ctl->sfc.v = NONE;
  ctl->sovf.v = NONE;
  ctl->sdeal.v = 0;
  s.ticket = 0;
  ctl->slogtop.v = 0;
  ctl->sxtop.v = 0;
  s.fallback = 0;
  s.ftile = 0;
  s.tgen = (long long)__builtin_amdgcn_s_memrealtime();
  s.gxlong0 = s.xlong;
}

// ---------------------------------------------------------------------------------------------
// Init scan (1 block x 1024): bucket bases from the capacity histogram; exclusive scan of the
// per-chunk phase-1 counts (compaction offsets); sets up the phase-1 pseudo-batch.
__global__ __launch_bounds__(1024) void k_init_scan(Ws ws, int npxchunk, unsigned epoch0, unsigned stag0) {
  Ctl* ctl = ws.ctl;
  const int tid = threadIdx.x;
  __shared__ long long wsum[16];
  __shared__ long long capw[4];
  __shared__ long long total_items;
  // bucket regions: exclusive scan of the level capacities (waves 0-3)
  __shared__ unsigned long long capq[4][NQ];
  {  // sum the CAP_SLOTS partial histograms: 4 groups of 16 slots, then the groups
    const int g = tid >> 8, lv = tid & (NQ - 1);
    unsigned long long sum = 0;
#pragma unroll
    for (int k = 0; k < CAP_SLOTS / 4; ++k) sum += ws.capp[(g * (CAP_SLOTS / 4) + k) * NQ + lv];
    capq[g][lv] = sum;
    // zeroed for the context's next flood once read (the host clears them itself when a flood
    // stopped between the phase-0 kernel and this one: msg_ctx::capp_clean)
#pragma unroll
    for (int k = 0; k < CAP_SLOTS / 4; ++k) ws.capp[(g * (CAP_SLOTS / 4) + k) * NQ + lv] = 0;
  }
  __syncthreads();
  long long cv = 0, cx = 0;
  if (tid < NQ) {
    cv = (long long)(capq[0][tid] + capq[1][tid] + capq[2][tid] + capq[3][tid]);
    cx = cv;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long y = __shfl_up(cx, o);
      if ((tid & 63) >= o) cx += y;
    }
    if ((tid & 63) == 63) capw[tid >> 6] = cx;
  }
  // raster-chunk offsets: exclusive scan of the per-chunk phase-1 counts, 16 K chunks per pass
  // (16 per thread, int4 loads/stores, in-register prefix, wave + block prefix, running carry)
  const int lane = tid & 63, wv = tid >> 6;
  long long carry = 0;
  for (int c0 = 0; c0 < npxchunk; c0 += 1024 * 16) {
    const int c = c0 + tid * 16;
    int v[16];
    if (c + 16 <= npxchunk) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int4 t = *reinterpret_cast<const int4*>(ws.tot + c + 4 * q);
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = (c + q < npxchunk) ? ws.tot[c + q] : 0;
    }
    long long s = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += v[q];
    long long x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    long long off = carry + x - s;
    long long tot = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < wv) off += wsum[k];
      tot += wsum[k];
    }
    int o16[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      o16[q] = (int)off;
      off += v[q];
    }
    if (c + 16 <= npxchunk) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<int4*>(ws.choff + c + 4 * q) = make_int4(o16[4 * q], o16[4 * q + 1], o16[4 * q + 2], o16[4 * q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (c + q < npxchunk) ws.choff[c + q] = o16[q];
    }
    carry += tot;
    __syncthreads();  // wsum reused by the next pass
  }
  if (tid == 0) total_items = carry;
  __syncthreads();
  if (tid < NQ) {  // bucket region bases (capw is visible after the barriers above)
    long long base = cx - cv;
    for (int k = 0; k < (tid >> 6); ++k) base += capw[k];
    ctl->qbase[tid] = (int)base;
    if (tid == NQ - 1) {
      const long long acc = base + cv;
      ctl->qbase[NQ] = (int)min(acc, (long long)0x7fffffff);
      if (acc > ws.qcap) ctl->error = ERR_CAPACITY;
    }
  }
  const long long M = total_items;
  if (tid == 0) {
    Batch pb;
    pb.mode = 1;
    pb.rrun = 0;
    pb.L = -1;
    pb.bstart = 0;
    pb.n = (int)M;
    pb.nseg = 0;
    pb.epoch = epoch0;
    pb.ncommit = (int)M;
    pb.nchunk = (int)((M + CH - 1) / CH);
    ctl->bat = pb;
    ctl->cut = NONE;
    ctl->segcut = NONE;
    ctl->minpush = 0;  // the first flood batch is never merged
    ctl->spec.T = stag0;  // speculative round tags continue from the context's last one
    if (M == 0) ctl->done = 1;
  }
}

// Ordered compaction of the phase-1 pixels in raster order into ilist/desc + level histograms:
// a wave owns CPW raster chunks and copies each non-empty chunk's list (k_prep's scratch in
// qbuf) 64 entries per step -- dense seeds do not serialise a long list on one lane (one lane
// per chunk: 430 us for the shape stage's ring seeds at 4096^2), sparse seeds keep the grid
// small (one wave per chunk: 29 us for the mosaic's, 32 K mostly idle waves).
__device__ __forceinline__ int ld_state(const Ws& ws, long long t);

constexpr int CPW = 4;  // raster chunks per k_compact wave

__global__ __launch_bounds__(256) void k_compact(Ws ws, int nrc) {
  if (ws.ctl->bat.n == 0 || ws.ctl->bat.mode != 1) return;
  const int lane = lane_id();
  const int ch0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * CPW;  // this wave's raster chunks
  if (ch0 >= nrc) return;
  const int myc = ch0 + lane;
  const int myn = (lane < CPW && myc < nrc) ? ws.tot[myc] : 0;
  long long mrs = 0, mk0 = 0;
  if (myn > 0) {
    const int r = myc / ws.nseg, cs = myc % ws.nseg;
    mrs = (long long)r * ws.W + (long long)cs * RSEG;
    mk0 = ws.choff[myc];
  }
  unsigned long long todo = __ballot(myn > 0);
  while (todo) {  // wave-uniform
    const int src = __ffsll((long long)todo) - 1;
    todo &= todo - 1;
    const int n = __shfl(myn, src);
    const long long rs = __shfl(mrs, src), k0 = __shfl(mk0, src);
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int j = j0 + lane;
      const bool on = j < n;
      const long long k = k0 + j;
      long long bin = -1;
      if (on) {
        const int t = ws.qbuf[rs + j];
        const int lv = ld_state(ws, t) & 255;
        ws.ilist[k] = t;
        ws.desc[k] = make_desc((unsigned)lv, 1u, 0, 0);
        bin = (k / CH) * NQ + lv;
      }
      // plateau seeds share a level: one atomic per distinct histogram bin of the wave
      unsigned long long rem = __ballot(on);
      while (rem) {
        const int leader = __ffsll((long long)rem) - 1;
        const long long lb = __shfl(bin, leader);
        const unsigned long long same = __ballot(on && bin == lb);
        if (lane == leader) atomicAdd(&ws.cnt[lb], (int)__popcll(same));
        rem &= ~same;
      }
    }
  }
}

__device__ __forceinline__ int ld_state(const Ws& ws, long long t) { return ws.mk[t]; }

// 32-bit form of nb_of for indices taken from the margin start (a multiple of 16: tile-aligned)
__device__ __forceinline__ int nbi(int t, int d, int Wt) {
  const int row = Wt << 4;
  switch (d) {
    case 0: return (t & 3) ? t - 1 : t - 13;
    case 1: return ((t & 3) != 3) ? t + 1 : t + 13;
    case 2: return (t & 12) ? t - 4 : t - row + 12;
    default: return ((t & 12) != 12) ? t + 4 : t + row - 12;
  }
}
__device__ __forceinline__ void st_state(const Ws& ws, long long t, int v) { ws.mk[t] = v; }
__device__ __forceinline__ unsigned ld_w4(const Ws& ws, long long t) {
  return (unsigned)ws.w4[t];
}

__device__ __forceinline__ int fold_lab(int lab, int v) {
  return (lab == 0) ? v : (lab == v ? v : WSHED);
}


struct Item {
  int p;             // tiled pixel index (< 2^31 - 512: check_size)
  int base_lab;      // fold of the settled (>0) neighbours: 0, a label, or WSHED
  unsigned zero_mask;
  unsigned wts;      // 4 packed 8-bit edge weights, directions L,R,T,B
  int dep[16];       // 0..3 label deps, 4+3d+k push deps (earlier items adjacent to the d-target)
};

// LEAN (k_resolve): the competitors of 0-neighbours only, in a second round of loads.  Otherwise
// (the one-workgroup small-batch loops, where each batch is a chain of dependent round trips) the
// whole radius-2 diamond in one round, the values of non-0 neighbours' competitors discarded.
template <bool LEAN>
__device__ __forceinline__ void gather_item(const Ws& ws, const Seg* segs, int nseg, int i, int slot,
                                            Item& it) {
  const int Wt = ws.Wt;
  const int p = ws.qbuf[slot];
  it.p = p;
  it.base_lab = 0;
  it.zero_mask = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) it.dep[k] = -1;
  it.wts = ld_w4(ws, p);
  // the 4 neighbours and their 3 other neighbours (push competitors, needed only for a 0-pixel
  // neighbour: LEAN loads them after the neighbours, for 0-pixels only, since k_resolve is bound
  // by the new lines it fetches per item -- DESIGN.md section 6).  Offsets are taken from the
  // margin's start (the buffer has a one-tile-row margin either side), so they are non-negative
  // and fit 32 bits.
  const int32_t* const mkb = ws.mk - ws.marg;
  const int pb = p + ws.marg;  // tiled index relative to the margin start
  int v[4], nn[4], vo[4][3];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    nn[d] = nbi(pb, d, Wt);
    v[d] = mkb[(unsigned)nn[d]];
    if (!LEAN) {
      const int e0 = (d == 1) ? 1 : 0;  // directions ascending, skipping the way back to p
      const int e1 = (d <= 1) ? 2 : 1;
      const int e2 = (d == 2) ? 2 : 3;
      vo[d][0] = mkb[(unsigned)nbi(nn[d], e0, Wt)];
      vo[d][1] = mkb[(unsigned)nbi(nn[d], e1, Wt)];
      vo[d][2] = mkb[(unsigned)nbi(nn[d], e2, Wt)];
    }
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (v[d] > 0) {
      it.base_lab = fold_lab(it.base_lab, v[d]);
    } else if (v[d] <= -3) {
      const int r = rank_of_slot(segs, nseg, state_slot(v[d]));
      if (r >= 0 && r < i) it.dep[d] = r;
    } else if (v[d] == 0) {
      it.zero_mask |= 1u << d;
    }
  }
  if (it.base_lab == WSHED) return;  // WSHED absorbs: no label or push dependency matters
  if (LEAN) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int e0 = (d == 1) ? 1 : 0;
      const int e1 = (d <= 1) ? 2 : 1;
      const int e2 = (d == 2) ? 2 : 3;
      const bool z = (it.zero_mask >> d) & 1u;
      vo[d][0] = z ? mkb[(unsigned)nbi(nn[d], e0, Wt)] : 0;
      vo[d][1] = z ? mkb[(unsigned)nbi(nn[d], e1, Wt)] : 0;
      vo[d][2] = z ? mkb[(unsigned)nbi(nn[d], e2, Wt)] : 0;
    }
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (!((it.zero_mask >> d) & 1u)) continue;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (vo[d][k] <= -3) {
        const int r = rank_of_slot(segs, nseg, state_slot(vo[d][k]));
        if (r >= 0 && r < i) it.dep[4 + 3 * d + k] = r;
      }
    }
  }
}

// Try to decide the item.  fetch(rank) -> resolved label of an earlier item, 0 = not yet.
template <class F>
__device__ __forceinline__ bool attempt_item(const Item& it, F fetch, int& lab_out, unsigned& mask_out) {
  int lab = it.base_lab;
  bool unknown = false;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int r = it.dep[d];
    if (r >= 0) {
      const int v = fetch(r);
      if (v == 0) unknown = true;
      else if (v > 0) lab = fold_lab(lab, v);
    }
  }
  if (lab == WSHED) {
    lab_out = WSHED;
    mask_out = 0;
    return true;
  }
  if (unknown) return false;
  unsigned m = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (!((it.zero_mask >> d) & 1u)) continue;
    bool lose = false, undecided = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int r = it.dep[4 + 3 * d + k];
      if (r >= 0) {
        const int v = fetch(r);
        if (v > 0) lose = true;
        else if (v == 0) undecided = true;
      }
    }
    if (!lose) {
      if (undecided) return false;
      m |= 1u << d;
    }
  }
  lab_out = lab;
  mask_out = m;
  return true;
}

// ---------------------------------------------------------------------------------------------
// Large batches: one kernel decides every item, k_scatter commits.
//
// k_resolve: label of an item = fold of its settled neighbours and of the labels of EARLIER batch
// items adjacent to it; it pushes a 0-neighbour z unless an earlier batch item adjacent to z has
// a non-WSHED label (serially that item pushed z first).  Both only wait on LOWER ranks.  Ranks
// are dealt round-robin over the grid (block-round r covers ranks [r*G*RBS, (r+1)*G*RBS)), so a
// lower rank is in the same round or an earlier one.  Progress does not rest on the grid being
// co-resident: a block claims each chunk as it starts it, and a wait that has lasted YIELD_TICKS
// on a chunk nobody has claimed (its block is not resident, and the slots it needs may be held
// by waiters) makes the waiting block give its chunk up and exit.  Everything a chunk writes
// before it completes is idempotent (final and provisional granules, descriptors, cut words),
// its histogram is added only on completion, and k_scan re-runs the batch (same epoch) until
// every chunk has completed; a re-run skips completed chunks, so the lowest unfinished chunk
// always completes.  In-wave dependencies go through register shuffles, others through
// 8-byte granules {epoch, label} (final) or {epoch | bit 63, base fold} (provisional: a pending
// dep whose settled neighbours fold to b can only end as b or WSHED).  Items then add their
// pushes to the per-chunk level histograms and the cut words, which k_scan consumes.
__device__ Batch scan_body(const Ws& ws);
__device__ void scatter_chunks(const Ws& ws, const Batch& B, int first, int stride);
__device__ __forceinline__ void small_loop(const Ws& ws, int ser_next);

// Cold path of k_resolve's long waits (out of line, so its registers stay off the hot loop): is
// some chunk below `chunk` neither claimed in this run nor completed?
__device__ __attribute__((noinline)) bool orphan_below(const unsigned long long* cflag, int chunk,
                                                       unsigned long long ctag, unsigned epoch) {
  bool orphan = false;
  for (int c2 = lane_id(); c2 < chunk; c2 += 64)
    if (__hip_atomic_load(&cflag[2 * c2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ctag &&
        __hip_atomic_load(&cflag[2 * c2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch)
      orphan = true;
  return orphan;
}

// 6 waves per SIMD: 80 VGPRs, so three 512-thread blocks per CU and a block-round of 768 x 512
// items: the batches of 262 145-393 216 items, which at the 96-VGPR build's two blocks per CU took
// a second block-round of the whole round-trip chain, take one (k_resolve 22.7 -> 21.6 us,
// headline 5088 -> 5180 Mpx/s, batch 9204 -> 9366; 8 waves: 64 VGPRs, 4970:
// profiles/r05zy_ab_resolve_waves.log).  Without scratch (see the chunk loop's end): 5283, batch
// 9620 (profiles/r05zz_ab_resolve_nospill.log)
template <bool INJECT>
__global__ __launch_bounds__(RBS) __attribute__((amdgpu_waves_per_eu(6))) void k_resolve(Ws ws) {
  Ctl* ctl = ws.ctl;
  __shared__ Seg segs[NQ];
  __shared__ int hist[NQ];
  __shared__ int s_minpush;
  // the first segments are loaded together with the batch header (most batches have one), the
  // rest -- of a multi-segment batch -- once its size is known
  if (threadIdx.x < 4) segs[threadIdx.x] = ctl->seg[threadIdx.x];
  const Batch B = ctl->bat;
  // hold: k_commit_fast declined this decided batch (too many chunks); k_scan commits it
  const bool work = !(B.n == 0 || B.mode != 0 || ctl->error || ctl->hold == B.epoch);
  if (work)
    for (int k = 4 + threadIdx.x; k < B.nseg; k += blockDim.x) segs[k] = ctl->seg[k];
  if (threadIdx.x == 0) s_minpush = NQ;
  const int tid = threadIdx.x, lane = lane_id();
  const unsigned long long etag = (unsigned long long)B.epoch << 32;  // final label granule
  const unsigned long long ptag = etag | (1ull << 63);                // provisional base fold
  unsigned long long* const dg = ws.diag;
  // s_skip is double-buffered by chunk parity: a wave that skips a chunk reads its flag after
  // the chunk's barrier, and thread 0 may already be writing the next chunk's flag by then (the
  // skip path has no second barrier); one buffer let a late wave read the next chunk's flag and
  // process a completed chunk out of step with the block (re-runs under concurrent floods)
  __shared__ int s_skip[2], s_yield;
  __shared__ unsigned long long s_ctag;  // this run's chunk claims: {epoch, re-run}
  __shared__ unsigned long long s_tl[RBS];  // the chunk's granules, for dependencies inside the block
  if (tid == 0) s_ctag = etag | (unsigned)B.rrun;
  if (work && blockIdx.x == 0 && tid == 0) {
    ctl->rsv = B.epoch;  // k_scan commits only decided batches
    ctl->ritems += B.n;  // one writer per launch (block 0); re-runs count again: they redo the work
  }
  if (tid == 0) s_yield = 0;
  for (int base = blockIdx.x * RBS; work && base < B.n; base += gridDim.x * RBS) {
    const int chunk = base / RBS;
    const int par = (base / (gridDim.x * RBS)) & 1;
    if (tid == 0) {  // claim the chunk, or skip it when an earlier run of this batch completed it
      const int sk = B.rrun > 0 &&
                     __hip_atomic_load(&ws.cflag[2 * chunk + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == B.epoch;
      s_skip[par] = sk;
      if (!sk) __hip_atomic_store(&ws.cflag[2 * chunk], s_ctag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < NQ) hist[tid] = 0;
    s_tl[tid] = 0;
    __syncthreads();
    if (s_skip[par]) continue;
    const int wbase = base + (tid & ~63);
    const int i = wbase + lane;
    const bool valid = i < B.n;
    // a dependency on another wave of the block reads its granule from LDS (every wave of the
    // block is resident, so such a wait cannot outlast its writer); the global granule serves the
    // other blocks.  Measured: k_resolve 23.85 -> 23.37 us at 4096^2, the headline flat
    // (profiles/r05o_ab_resolve.log; merging the push phase's granule loads into the label
    // phase's round trip, or 1024-thread blocks, measured slower)
    auto gld = [&](int r) -> unsigned long long {
      return ((unsigned)(r - base) < (unsigned)RBS)
                 ? __hip_atomic_load(&s_tl[r - base], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                 : ld_granule(&ws.tl[r]);
    };
    auto gst = [&](unsigned long long v) {
      __hip_atomic_store(&s_tl[tid], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      st_granule(&ws.tl[i], v);
    };
    const unsigned long long t_a = dg ? __builtin_amdgcn_s_memtime() : 0;
    Item it;
    int sg = 0;
    if (valid) {
      sg = (B.nseg == 1) ? 0 : seg_of_rank(segs, B.nseg, i);
      gather_item<true>(ws, segs, B.nseg, i, segs[sg].bstart + (i - segs[sg].rank), it);
      ws.ipx[i] = (int32_t)it.p;
    } else {
      it.p = 0;
      it.base_lab = WSHED;
      it.zero_mask = 0;
      it.wts = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) it.dep[k] = -1;
    }
    if (INJECT && (blockIdx.x & 1) && base < (int)(gridDim.x * RBS) && B.rrun == 0) {
      if (tid == 0) s_yield = 1;  // fault injection: exercise the give-up / re-run path
      __syncthreads();
      if (tid == 0) {
        __hip_atomic_store(&ws.cflag[2 * chunk], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctl->rgive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
    unsigned inw = 0;  // wave-uniform: dependency slots that point inside this wave
    bool anydep = false;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (__any((unsigned)(it.dep[k] - wbase) < 64u)) inw |= 1u << k;
      anydep |= it.dep[k] >= 0;
    }
    anydep = __any(anydep);
    bool lab_done = !valid, push_done = !valid, published = false;
    int mylab = 0;
    long long t0 = 0, iters = 0;
    int spins = 0;
    const unsigned long long t_b = dg ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
      // label phase: in-wave snapshots of the 4 label deps (label + base fold)
      int snap[4] = {0, 0, 0, 0}, sbase[4] = {0, 0, 0, 0};
      if (anydep) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((inw >> k) & 1u) {
            const int r = it.dep[k];
            const int src = ((unsigned)(r - wbase) < 64u) ? r - wbase : lane;
            snap[k] = __shfl(mylab, src);
            sbase[k] = __shfl(it.base_lab, src);
          }
      }
      if (!lab_done) {
        // fold the settled labels and the final labels of resolved deps; a pending dep whose
        // base fold is WSHED or already in the fold is redundant
        int lab = it.base_lab;
        int prov[4] = {0, 0, 0, 0};
        unsigned pm = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int r = it.dep[d];
          if (r < 0) continue;
          int v, pb;
          if ((unsigned)(r - wbase) < 64u) {
            v = snap[d];
            pb = sbase[d];
          } else {
            const unsigned long long g = gld(r);
            const unsigned long long hi = g & 0xffffffff00000000ull;
            v = (hi == etag) ? (int)(uint32_t)g : 0;
            pb = (hi == ptag) ? (int)(uint32_t)g : 0;
          }
          if (v > 0) lab = fold_lab(lab, v);
          else if (v == 0) {
            prov[d] = pb;
            pm |= 1u << d;
          }
          // a final dependency is folded in for good and dropped: later passes neither reload nor
          // wait for it (its label joins the base fold: the item still ends as it or WSHED).
          // Measured: 128 -> 96 VGPRs, k_resolve 23.3 -> 22.7 us, headline 4963 -> 5103 Mpx/s
          // (profiles/r05w_ab_resolve_drop.log)
          if (v != 0) {
            if (v > 0) it.base_lab = fold_lab(it.base_lab, v);
            it.dep[d] = -1;
          }
        }
        bool unknown = false;
#pragma unroll
        for (int d = 0; d < 4; ++d)
          if (((pm >> d) & 1u) && prov[d] != WSHED && !(prov[d] > 0 && prov[d] == lab)) unknown = true;
        if (unknown && lab != WSHED) {
          if (!published && it.base_lab != 0) {  // let later items see this one's base fold
            gst(ptag | (uint32_t)it.base_lab);
            published = true;
          }
        } else {
          if (lab == 0) {  // impossible for an exact queue: flag, label as WSHED
            atomicOr(&ctl->error, ERR_STATE);
            lab = WSHED;
          }
          mylab = lab;
          gst(etag | (uint32_t)lab);
          lab_done = true;
        }
      }
      // push phase: in-wave snapshots of the 12 push-competitor labels (after this round's labels)
      int psnap[12];
#pragma unroll
      for (int k = 0; k < 12; ++k) psnap[k] = 0;
      if (anydep) {
#pragma unroll
        for (int k = 0; k < 12; ++k)
          if ((inw >> (4 + k)) & 1u) {
            const int r = it.dep[4 + k];
            psnap[k] = __shfl(mylab, ((unsigned)(r - wbase) < 64u) ? r - wbase : lane);
          }
      }
      if (lab_done && !push_done) {
        // push to 0-neighbour z unless an earlier batch item adjacent to z is non-WSHED
        unsigned m = 0;
        bool undecided = false;
        if (mylab != WSHED) {
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            if (!((it.zero_mask >> d) & 1u)) continue;
            bool lose = false, und = false;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const int r = it.dep[4 + 3 * d + k];
              if (r < 0) continue;
              int v;
              if ((unsigned)(r - wbase) < 64u) {
                v = psnap[3 * d + k];
              } else {
                const unsigned long long g = gld(r);
                v = ((g & 0xffffffff00000000ull) == etag) ? (int)(uint32_t)g : 0;
              }
              if (v > 0) lose = true;
              else if (v == 0) und = true;
              else it.dep[4 + 3 * d + k] = -1;  // a WSHED competitor never pushes: dropped
            }
            if (lose) it.zero_mask &= ~(1u << d);  // lost for good: no more loads for z
            if (!lose) {
              if (und) undecided = true;
              else m |= 1u << d;
            }
          }
        }
        if (!undecided) {
          push_done = true;
          const int lvi = segs[sg].L;
          ws.desc[i] = make_desc(it.wts, m, lvi, sg);
          bool lower = false;
          int tmin = NQ;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            if (!((m >> d) & 1u)) continue;
            const int lv = (it.wts >> (8 * d)) & 255;
            atomicAdd(&hist[lv], 1);
            if (lv < lvi) lower = true;
            else tmin = min(tmin, lv);
          }
          if (lower) {
            atomicMin(&ctl->cut, i);
            atomicMin(&s_minpush, 0);
          }
          if (tmin < NQ) {
            atomicMin(&s_minpush, tmin);
            if (B.nseg > 1) {
              const int mc = seg_cut_for(segs, B.nseg, sg, tmin);
              if (mc != NONE) atomicMin(&ctl->segcut, mc);
            }
          }
        }
      }
      ++iters;
      if (!__any(!push_done)) break;
      if (++spins > 16) {
        __builtin_amdgcn_s_sleep(1);
        // {error, rgive}: stop on an error; give the chunk up when some block gave one up
        const unsigned long long ew = __hip_atomic_load((unsigned long long*)&ctl->error, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        if (ew) {
          if (!(uint32_t)ew && lane == 0) s_yield = 1;
          break;
        }
        const long long now = (long long)__builtin_amdgcn_s_memrealtime();
        if (t0 == 0) t0 = now;
        else if (now - t0 > SPIN_LIMIT_TICKS) {
          if (!push_done) atomicOr(&ctl->error, ERR_TIMEOUT);
          break;
        } else if ((spins & 255) == 0 && now - t0 > YIELD_TICKS) {
          // a long wait: is every lower chunk claimed by a running block (or completed)?
          const bool orphan = orphan_below(ws.cflag, chunk, *(volatile unsigned long long*)&s_ctag, B.epoch);
          if (__any(orphan)) {
            if (lane == 0) {
              s_yield = 1;
              __hip_atomic_store(&ctl->rgive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
          }
        }
      }
    }
    if (dg && lane == 0) {  // diagnostics path only (msg_set_diag)
      const unsigned long long t_c = __builtin_amdgcn_s_memtime();
      atomicAdd(&dg[0], t_b - t_a);
      atomicAdd(&dg[1], t_c - t_b);
      atomicAdd(&dg[2], (unsigned long long)iters);
      atomicMax(&dg[3], t_c - t_b);
      atomicAdd(&dg[4], 1ull);
    }
    __syncthreads();
    if (s_yield) {  // chunk given up: no histogram, no completion; k_scan re-runs the batch
      if (tid == 0) {
        __hip_atomic_store(&ws.cflag[2 * chunk], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctl->rgive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
    // the row address and the epoch are formed here: hoisted out of the chunk loop they were two
    // 64-bit values live across the whole kernel, which the 80-VGPR budget spilled to scratch
    // (16 B written per thread per launch)
    int t = tid;
    unsigned ep = B.epoch;
    asm volatile("" : "+v"(t), "+s"(ep));
    if (t < NQ && hist[t]) atomicAdd(&ws.cnt[(long long)(base / CH) * NQ + t], hist[t]);
    if (t == 0) __hip_atomic_store(&ws.cflag[2 * chunk + 1], (unsigned long long)ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  }
  __syncthreads();
  if (tid == 0 && s_minpush < NQ) atomicMin(&ctl->minpush, s_minpush);
}

// Scan (1 block x 1024) of the batch k_resolve decided; a committed batch of at most SMALL_MAX
// items is scattered here too, and then, with nothing left for k_scatter, this block runs the
// following small batches itself (small_loop).
__global__ __launch_bounds__(1024) void k_scan(Ws ws, int ser_next) {
  Ctl* ctl = ws.ctl;
  const Batch cb = scan_body(ws);
  if (cb.mode == 2) return;  // k_resolve gave chunks up: the batch runs again, nothing committed
  if (cb.nchunk > 0 && cb.n <= SMALL_MAX && !ctl->error) {
    scatter_chunks(ws, cb, 0, 1);
    __syncthreads();
    if (threadIdx.x == 0) ctl->cbat.nchunk = 0;
  } else if (cb.nchunk > 0) {
    return;  // k_scatter commits it
  }
  if (!ws.multi) small_loop(ws, ser_next);  // a many-floods batch pops in k_serial_multi instead
}

// ---------------------------------------------------------------------------------------------
// Scan (1 block x 1024): committed prefix (interrupt cut, segment cut), recount of the cut chunk,
// column scan -> per-chunk bucket offsets, head/tail update, hand the committed batch to k_scatter
// (cbat), form the next batch.
__device__ Batch scan_body(const Ws& ws) {
  Ctl* ctl = ws.ctl;
  const Batch B = ctl->bat;
  const int tid = threadIdx.x;
  Batch none = B;
  none.n = 0;
  none.nchunk = 0;
  if (B.n == 0 || ctl->error) {  // nothing committed this iteration (finished, or stopped)
    __syncthreads();
    if (tid == 0) {
      ctl->cbat.n = 0;
      ctl->cbat.nchunk = 0;
      if (ctl->error) {
        ctl->bat.n = 0;
        ctl->done = 1;
      }
    }
    return none;
  }
  if (B.mode == 3 || (B.mode == 0 && ctl->rsv != B.epoch)) {
    // not decided yet: speculative rounds still running, or an iteration without k_resolve
    // (the host queued the other iteration kind): nothing to commit here
    __syncthreads();
    if (tid == 0) {
      ctl->cbat.n = 0;
      ctl->cbat.nchunk = 0;
    }
    return none;
  }
  // the queue state lives in LDS for the whole kernel: one parallel load, one write-back
  __shared__ int partial[NQ];
  __shared__ int s_head[NQ], s_tail[NQ], s_base[NQ];
  __shared__ Seg s_seg[NQ];
  __shared__ Seg nsegs[NQ];
  __shared__ int s_nseg, s_n;
  __shared__ Batch s_cb;
  if (tid < NQ) {
    s_head[tid] = ctl->qhead[tid];
    s_tail[tid] = ctl->qtail[tid];
    s_base[tid] = ctl->qbase[tid];
    partial[tid] = 0;
  }
  if (B.mode == 0 && tid < B.nseg) s_seg[tid] = ctl->seg[tid];
  const int cut = ctl->cut, segcut = ctl->segcut, minpush = ctl->minpush;
  const int give = ctl->rgive;
  __syncthreads();
  if (give && B.mode == 0) {  // a k_resolve block gave its chunk up: run the same batch again
    if (tid == 0) {
      ctl->rgive = 0;
      ctl->cbat.n = 0;
      ctl->cbat.nchunk = 0;
      ctl->bat.rrun = B.rrun + 1;
    }
    none.mode = 2;
    return none;
  }
  int ncommit = B.n;
  if (B.mode == 0) {
    if (cut != NONE) ncommit = min(ncommit, cut + 1);
    if (segcut != NONE) ncommit = min(ncommit, s_seg[segcut].rank);
  }
  const int nch = (ncommit + CH - 1) / CH;
  const bool haspartial = (ncommit % CH) != 0 && ncommit != B.n;
  if (haspartial) {  // the cut chunk's histogram covers items past the cut: recount its prefix
    for (int i = (nch - 1) * CH + tid; i < ncommit; i += blockDim.x) {
      const unsigned long long d = ws.desc[i];
      const unsigned m = (unsigned)(d >> 32) & 15u;
      for (int k = 0; k < 4; ++k)
        if ((m >> k) & 1u) atomicAdd(&partial[(d >> (8 * k)) & 255], 1);
    }
    __syncthreads();
  }
  const int oldt = (tid < NQ) ? s_tail[tid] : 0;
  column_scan(ws.cnt, ws.coff, nch, haspartial ? partial : nullptr, s_tail);
  if (tid < NQ) {  // pushes appended: one atomic per wave of levels (no block barrier)
    int dp = s_tail[tid] - oldt;
    dp = wave_sum(dp);
    if ((tid & 63) == 0 && dp) {
      atomicAdd((unsigned long long*)&ctl->pushes, (unsigned long long)dp);
      atomicAdd((unsigned long long*)&ctl->spushes, (unsigned long long)dp);
    }
  }
  if (B.mode == 0 && tid < B.nseg) {  // advance every segment's bucket head by what it committed
    const Seg s = s_seg[tid];
    s_head[s.L] += max(0, min(ncommit - s.rank, s.n));
  }
  if (tid == 0) {
    if (B.mode == 0) {
      ctl->pops += ncommit;
      ctl->items += B.n;
      ctl->s0pops += ncommit;
    }
    ctl->spops += ncommit;
    Batch cb = B;
    cb.ncommit = ncommit;
    cb.nchunk = nch;
    ctl->cbat = cb;
    s_cb = cb;
  }
  // the histogram rows this batch accumulated are zeroed by k_scatter (cbat.n covers them all)
  __syncthreads();
  const int wcap = (B.mode == 0) ? next_wcap(ctl->wcap, B.n, ncommit, cut != NONE && ncommit == cut + 1)
                                 : ctl->wcap;
  form_batch(s_base, s_head, s_tail, B.mode == 0 ? minpush : 0, wcap, nsegs, &s_nseg, &s_n);
  __syncthreads();
  const int ns = s_nseg;
  for (int k = tid; k < ns; k += blockDim.x) ctl->seg[k] = nsegs[k];
  if (tid < NQ) {
    ctl->qhead[tid] = s_head[tid];
    ctl->qtail[tid] = s_tail[tid];
  }
  if (tid == 0) {
    Batch nb;
    nb.mode = 0;
    nb.epoch = B.epoch + 1;
    nb.ncommit = 0;
    nb.nchunk = 0;
    nb.rrun = 0;
    nb.nseg = ns;
    nb.n = (ns > 0) ? s_n : 0;
    nb.L = (ns > 0) ? nsegs[0].L : -1;
    nb.bstart = (ns > 0) ? nsegs[0].bstart : 0;
    if (ns > 0 && ctl->spec.on)
      spec_begin(ctl, nb, nsegs[0].L, nsegs[0].bstart, s_tail[nsegs[0].L] - s_head[nsegs[0].L]);
    ctl->bat = nb;
    ctl->wcap = wcap;
    ctl->cut = NONE;
    ctl->segcut = NONE;
    ctl->minpush = NQ;
    if (ns > 0) ctl->batches += 1;
    else ctl->done = 1;
  }
  if (tid < 64) {  // queued items left (host polling hint): wave 0 alone
    int q = 0;
#pragma unroll
    for (int k = 0; k < NQ / 64; ++k) q += s_tail[tid + 64 * k] - s_head[tid + 64 * k];
    q = wave_sum(q);
    if (tid == 0) ctl->remaining = q;
  }
  __syncthreads();
  return s_cb;  // visible after the barrier above
}

// Stable rank of this lane's pushes among the wave's pushes of the same level, in (lane, dir)
// order.  Writes the per-level wave totals to wrow[level].  Wave-uniform loop over the distinct
// levels present in the wave.
__device__ __forceinline__ void wave_rank(unsigned mask, unsigned lvls, int pos[4], int* wrow) {
  const int lane = lane_id();
  unsigned rem = mask;
  for (;;) {
    const unsigned long long act = __ballot(rem != 0);
    if (act == 0) break;
    const int leader = __ffsll((long long)act) - 1;
    const int myl = rem ? (int)((lvls >> (8 * (__ffs(rem) - 1))) & 255u) : -1;
    const int lsel = __builtin_amdgcn_readlane(myl, leader);  // uniform lane: no LDS crossbar
    unsigned sel = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if (((rem >> d) & 1u) && (int)((lvls >> (8 * d)) & 255u) == lsel) sel |= 1u << d;
    // exclusive prefix of the per-lane counts (0..4) from three ballots of their bits and
    // mbcnt (lanes below this one), instead of a six-step shuffle scan: no LDS-crossbar round
    // trips on the ordered append's critical path
    const int cnt = __popc(sel);
    const unsigned long long b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2), b2 = __ballot(cnt & 4);
    const int total = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    int k = lanes_below(b0) + 2 * lanes_below(b1) + 4 * lanes_below(b2);
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if ((sel >> d) & 1u) pos[d] = k++;
    if (lane == 0) wrow[lsel] = total;
    rem &= ~sel;
  }
}

// Ordered scatter: commit labels of the committed prefix and append its pushes to the buckets in
// exact (rank, dir) order.  mode 1 (phase-1 pseudo-batch): item i is pixel ilist[i] itself.
// One 1024-thread block per 1024-item sub-round, four per 4096-item chunk, all independent: a
// sub-round's in-chunk offset is the chunk offset (k_scan) plus the per-level push counts of the
// chunk's earlier sub-rounds, recounted here from their (L2-resident) descriptors.  The blocks
// also zero the histogram rows the batch accumulated (consumed by k_scan).
__device__ void scatter_chunks(const Ws& ws, const Batch& B, int first, int stride) {
  Ctl* ctl = ws.ctl;
  constexpr int NW = 16, SUBS = CH / 1024;
  __shared__ int run[NQ];
  __shared__ int wcnt[NW][NQ];
  __shared__ int qb[NQ];
  const int tid = threadIdx.x, wv = tid >> 6;
  const int Wt = ws.Wt;
  {
    const long long rows = (long long)((B.n + CH - 1) / CH) * NQ;
    for (long long k = (long long)first * 1024 + tid; k < rows; k += (long long)stride * 1024)
      ws.cnt[k] = 0;
  }
  if (tid < NQ) qb[tid] = ctl->qbase[tid];
  for (int vb = first; vb < B.nchunk * SUBS; vb += stride) {
    const int ch = vb / SUBS, i0 = ch * CH + (vb % SUBS) * 1024;
    if (i0 >= B.ncommit) continue;  // block-uniform
    if (tid < NQ) {
      run[tid] = ws.coff[(long long)ch * NQ + tid];
#pragma unroll
      for (int k = 0; k < NW; ++k) wcnt[k][tid] = 0;
    }
    __syncthreads();
    for (int j = ch * CH + tid; j < i0; j += 1024) {  // earlier sub-rounds of this chunk
      const unsigned long long d = ws.desc[j];
      const unsigned m = (unsigned)(d >> 32) & 15u;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((m >> k) & 1u) atomicAdd(&run[(d >> (8 * k)) & 255], 1);
    }
    const int i = i0 + tid;
    const bool valid = i < B.ncommit;
    unsigned mask = 0, lvls = 0;
    long long p = 0;
    if (valid) {
      const unsigned long long d = ws.desc[i];
      mask = (unsigned)(d >> 32) & 15u;
      lvls = (unsigned)d;
      if (B.mode == 0) {
        p = ws.ipx[i];
        st_state(ws, p, (int32_t)(uint32_t)ws.tl[i]);
      } else {
        p = ws.ilist[i];
      }
    }
    int pos[4] = {0, 0, 0, 0};
    wave_rank(mask, lvls, pos, wcnt[wv]);
    __syncthreads();
    if (tid < NQ) {  // exclusive prefix over the waves, per level, on top of the sub-round offset
      int acc = run[tid];
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        const int t = wcnt[k][tid];
        wcnt[k][tid] = acc;
        acc += t;
      }
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (!((mask >> d) & 1u)) continue;
      const int lv = (lvls >> (8 * d)) & 255;
      const int dest = qb[lv] + wcnt[wv][lv] + pos[d];
      if (dest < 0 || (long long)dest >= ws.qcap) {
        atomicOr(&ctl->error, ERR_CAPACITY);
        continue;
      }
      const long long n = (B.mode == 0) ? nb_of(p, d, Wt) : p;
      st_state(ws, n, queued_state(dest));
      ws.qbuf[dest] = (int32_t)n;
    }
    __syncthreads();  // before the next sub-round reuses run/wcnt
  }
}

// End of a flood: the control block into its host-mapped copy, then `seq` released into the
// progress mirror's word 7, on which the host spins instead of synchronising the stream (the wake
// of a stream synchronisation is a device signal; a mapped word is seen on its first read).
__global__ __launch_bounds__(256) void k_tail(const Ctl* __restrict__ ctl, Ctl* htail, int* hmir, int seq) {
  const int* s = reinterpret_cast<const int*>(ctl);
  int* d = reinterpret_cast<int*>(htail);
  for (int k = threadIdx.x; k < (int)(sizeof(Ctl) / 4); k += blockDim.x)
    __hip_atomic_store(d + k, s[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(hmir + 7, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void k_scatter(Ws ws, int iter) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && ws.hmir) {
    // progress mirror for the host loop: k_scan of this iteration has finished, so its control
    // words are final.  System-scope stores into pinned host memory; the iteration number is
    // released last, so a host that sees it also sees the three words before it.
    __hip_atomic_store(ws.hmir + 1, ws.ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 2, ws.ctl->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 3, ws.ctl->remaining, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 4, ws.ctl->spec.on, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 5, ws.ctl->spec_want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 6, fast_batch(ws.ctl->bat, ws.ctl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 8, ws.ctl->ser_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir, iter, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const Batch B = ws.ctl->cbat;
  if (B.nchunk == 0 || ws.ctl->error) return;
  scatter_chunks(ws, B, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------------------------
// Two-launch iterations for large batches (k_resolve -> k_commit_fast): the commit of k_scan and
// k_scatter in one grid.  Blocks 0 .. FAST_CH*SUBS-1 each take one 1024-item sub-round and compute
// its bucket offsets themselves -- the old tails plus the histogram rows of the earlier chunks (at
// most FAST_CH rows, L2-resident) plus the chunk's earlier sub-rounds, recounted from their
// descriptors -- so no column scan has to finish first.  The last block is the FINALIZER: it forms
// the next batch from the same control words and rows (all its reads overlap the scatter), then
// waits until every sub-round block has ARRIVED -- reported after that block's last read of the
// control block and of the rows, on one of 8 counters by blockIdx % 8 (a single counter costs
// ~12 ns per arrival) -- and only then rewrites the queue state and zeroes the rows.  The grid
// (FAST_SUBS + 1 = 481 blocks of 1024 threads, two per CU) is resident at once.  No fence is
// needed: the finalizer reads only what k_resolve wrote, and the arrivals only order reads before
// writes.  Batches it cannot commit are left alone: not decided yet (a speculative generation, or
// the host queued this iteration kind on stale information) -- nothing happens; decided but over
// FAST_CH chunks -- `hold` stops k_resolve from deciding it again and k_scan commits it.  k_scan's
// one-workgroup loop for runs of small batches is not here: the host goes back to three-launch
// iterations when the progress mirror reports a batch that is not fast_batch.
constexpr int FAST_SUBS = FAST_CH * (CH / 1024);  // sub-round blocks; the grid is FAST_SUBS + 1

// sum of cnt[c][lv] over the rows c < nrows with c % 4 == g (nrows <= FAST_CH): all loads first
__device__ __forceinline__ int rows_sum(const int* cnt, int g, int nrows, int lv) {
  int v[FAST_CH / 4];
#pragma unroll
  for (int k = 0; k < FAST_CH / 4; ++k) {
    const int c = g + 4 * k;
    v[k] = (c < nrows) ? cnt[(long long)c * NQ + lv] : 0;
  }
  int sum = 0;
#pragma unroll
  for (int k = 0; k < FAST_CH / 4; ++k) sum += v[k];
  return sum;
}
// the same over any number of rows, FAST_CH rows (one round trip) at a time
__device__ __forceinline__ int rows_sum_any(const int* cnt, int g, int nrows, int lv) {
  int sum = 0;
#pragma unroll 1
  for (int c0 = 0; c0 < nrows; c0 += FAST_CH)
    sum += rows_sum(cnt + (long long)c0 * NQ, g, min(FAST_CH, nrows - c0), lv);
  return sum;
}

// What the commit of the current batch is: 1 commit ncommit items, 2 re-run (a k_resolve block
// gave its chunk up), 4 decided but too large (k_scan commits it), 0 nothing to do.
template <bool MP>
__device__ __forceinline__ int fast_flags(const Ctl* ctl, const Batch& B, int& ncommit, int G) {
  const unsigned rsv = ctl->rsv, hold = ctl->hold;
  const int err = ctl->error, give = ctl->rgive, cut = ctl->cut, segcut = ctl->segcut;
  ncommit = 0;
  const bool decided = B.mode == 0 && B.n > 0 && rsv == B.epoch && !err && hold != B.epoch;
  if (!decided) return 0;
  if (give) return 2;
  if (B.n > (MP ? FAST_PASS : 1) * G * 1024) return 4;  // G sub-round blocks of 1024 items
  ncommit = B.n;
  if (cut != NONE) ncommit = min(ncommit, cut + 1);
  if (segcut != NONE) ncommit = min(ncommit, ctl->seg[segcut].rank);
  return 1;
}

template <bool MP>
__device__ __forceinline__ void commit_fast_body(Ws ws, int iter) {
  constexpr int NPASS = MP ? FAST_PASS : 1;
  Ctl* ctl = ws.ctl;
  constexpr int NW = 16, SUBS = CH / 1024;
  __shared__ int run[NQ], qb[NQ], gpart[4][NQ], s_run[NPASS][NQ];
  __shared__ int wcnt[NW][NQ];
  __shared__ Batch s_B;
  __shared__ int s_ncommit, s_flags;
  const int tid = threadIdx.x, wv = tid >> 6;
  const int Wt = ws.Wt;
  // G sub-round blocks (the grid is G + 1; G a multiple of SUBS, at most FAST_SUBS): the whole
  // chip for one flood, a share of it per flood when the batch entry points keep several in flight
  const int G = MP ? (int)gridDim.x - 1 : FAST_SUBS;  // (compile-time on the single-flood path)
  // the bucket bases are loaded into registers before the header: a global -> LDS copy after
  // thread 0's header branch would cost wave 0 a second round trip before the barrier
#ifdef MSEG_CF_PROF
  // diagnostic build (make cfprof, scripts/cf_phases.py): s_memrealtime phase split, diag[8..15]
  const long long cf_t0 = (long long)__builtin_amdgcn_s_memrealtime();
  unsigned long long* const cfd = ws.diag ? ws.diag + 8 : nullptr;
  long long cf_t[6] = {0, 0, 0, 0, 0, 0};
#define CF_STAMP(k) do { if (cfd && tid == 0) cf_t[k] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define CF_STAMP(k) do { } while (0)
#endif
  const int r_qb = (tid < NQ) ? ctl->qbase[tid] : 0;
  if (tid == 0) {
    const Batch B = ctl->bat;
    int ncommit;
    s_flags = fast_flags<MP>(ctl, B, ncommit, G);
    s_ncommit = ncommit;
    s_B = B;
  }
  if (tid < NQ) qb[tid] = r_qb;
  __syncthreads();
  CF_STAMP(0);
  const Batch B = s_B;
  const int ncommit = s_ncommit, flags = s_flags;
  Ctl::Arrive* const arrive = ctl->farrive;
  const int vb = (int)blockIdx.x;
  if (vb < G) {
    // ---- a sub-round block ----
    const int ch = vb / SUBS, i0 = ch * CH + (vb % SUBS) * 1024;
    if (!(flags & 1) || i0 >= ncommit) {  // block-uniform: nothing to scatter, done reading
      if (tid == 0) atomicAdd(&arrive[vb & 7].v, 1u);
      return;
    }
    // Sub-rounds vb, vb + G, ... (up to FAST_PASS of them: batches of up to FAST_PASS * G / SUBS
    // chunks).  First, for each of them, everything the finalizer will rewrite -- the old
    // tails and the earlier chunks' histogram rows -- is read and reduced to the sub-round's
    // starting offsets per level (s_run); then the block arrives, and the scatters follow (their
    // descriptors, items and granules are the batch's, which only the next k_resolve rewrites).
    // pass j's chunk is G / SUBS (<= FAST_CH) chunks after pass j - 1's: its row prefix adds one
    // window of G / SUBS rows (one round trip) to the previous one
    int acc = (tid < NQ) ? ctl->qtail[tid] : 0;
    int npass = 0;
#pragma unroll 1
    for (int j = 0; j < NPASS; ++j) {
      const int vs = vb + j * G, chj = vs / SUBS;
      if (chj * CH + (vs % SUBS) * 1024 >= ncommit) break;  // block-uniform
      const int c0 = (j == 0) ? 0 : chj - G / SUBS;
      gpart[tid >> 8][tid & (NQ - 1)] = rows_sum(ws.cnt + (long long)c0 * NQ, tid >> 8, chj - c0, tid & (NQ - 1));
      __syncthreads();
      if (tid < NQ) {
        acc += gpart[0][tid] + gpart[1][tid] + gpart[2][tid] + gpart[3][tid];
        s_run[j][tid] = acc;
      }
      __syncthreads();
      ++npass;
    }
    // this block's reads of the control block and of the rows are complete
    if (tid == 0) atomicAdd(&arrive[vb & 7].v, 1u);
#ifdef MSEG_CF_PROF
    if (cfd && tid == 0 && vb == 0) atomicAdd(&cfd[6], (unsigned long long)((long long)__builtin_amdgcn_s_memrealtime() - cf_t0));
#endif
#pragma unroll 1
    for (int j = 0; j < npass; ++j) {
      const int vs = vb + j * G, chj = vs / SUBS, sub = vs % SUBS;
      const int i0j = chj * CH + sub * 1024;
      // the earlier sub-rounds' descriptors of its chunk and its own items: one round trip
      unsigned long long dj[SUBS - 1];
#pragma unroll
      for (int k = 0; k < SUBS - 1; ++k) dj[k] = (k < sub) ? ws.desc[chj * CH + k * 1024 + tid] : 0ull;
      const int i = i0j + tid;
      const bool valid = i < ncommit;
      unsigned long long dself = 0;
      int pself = 0, lself = 0;
      if (valid) {
        dself = ws.desc[i];
        pself = ws.ipx[i];
        lself = (int)(uint32_t)ws.tl[i];
      }
      if (tid < NQ) {
        run[tid] = s_run[j][tid];
#pragma unroll
        for (int k = 0; k < NW; ++k) wcnt[k][tid] = 0;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < SUBS - 1; ++k) {  // pushes of the earlier sub-rounds of this chunk
        const unsigned m = (unsigned)(dj[k] >> 32) & 15u;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if ((m >> e) & 1u) atomicAdd(&run[(dj[k] >> (8 * e)) & 255], 1);
      }
      const unsigned mask = (unsigned)(dself >> 32) & 15u;
      const unsigned lvls = (unsigned)dself;
      const long long p = pself;
      if (valid) st_state(ws, p, lself);
      int pos[4] = {0, 0, 0, 0};
      wave_rank(mask, lvls, pos, wcnt[wv]);
      __syncthreads();
      if (tid < NQ) {
        int acc = run[tid];
#pragma unroll
        for (int k = 0; k < NW; ++k) {
          const int t = wcnt[k][tid];
          wcnt[k][tid] = acc;
          acc += t;
        }
      }
      __syncthreads();
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if (!((mask >> d) & 1u)) continue;
        const int lv = (lvls >> (8 * d)) & 255;
        const int dest = qb[lv] + wcnt[wv][lv] + pos[d];
        if (dest < 0 || (long long)dest >= ws.qcap) {
          atomicOr(&ctl->error, ERR_CAPACITY);
          continue;
        }
        const long long n = nb_of(p, d, Wt);
        st_state(ws, n, queued_state(dest));
        ws.qbuf[dest] = (int32_t)n;
      }
      __syncthreads();  // wcnt / run are reused by the next pass
    }
    return;
  }
  // ---- the finalizer ----
  __shared__ int s_head[NQ], s_tail[NQ], partial[NQ];
  __shared__ Seg nsegs[NQ];
  __shared__ int s_nseg, s_n, s_wcap, s_minpush;
  if (flags & 1) {
    const int nch = (ncommit + CH - 1) / CH;
    const bool haspartial = (ncommit % CH) != 0 && ncommit != B.n;
    // the queue state, the window words and the batch's segments in one round trip (registers
    // first, then LDS)
    const int r_wcap = ctl->wcap, r_minpush = ctl->minpush, r_cut = ctl->cut;
    int r_h = 0, r_t = 0;
    if (tid < NQ) {
      r_h = ctl->qhead[tid];
      r_t = ctl->qtail[tid];
    }
    Seg r_sg{0, 0, 0, 0};
    if (tid < B.nseg) r_sg = ctl->seg[tid];
    if (tid < NQ) {
      s_head[tid] = r_h;
      s_tail[tid] = r_t;
      partial[tid] = 0;
    }
    if (tid == 0) {
      s_wcap = next_wcap(r_wcap, B.n, ncommit, r_cut != NONE && ncommit == r_cut + 1);
      s_minpush = r_minpush;
    }
    __syncthreads();
    CF_STAMP(1);
    if (haspartial) {  // the cut chunk's row counts items past the cut: recount its prefix
      for (int i = (nch - 1) * CH + tid; i < ncommit; i += 1024) {
        const unsigned long long d = ws.desc[i];
        const unsigned m = (unsigned)(d >> 32) & 15u;
        for (int k = 0; k < 4; ++k)
          if ((m >> k) & 1u) atomicAdd(&partial[(d >> (8 * k)) & 255], 1);
      }
    }
    const int nrows = haspartial ? nch - 1 : nch;
    gpart[tid >> 8][tid & (NQ - 1)] = MP ? rows_sum_any(ws.cnt, tid >> 8, nrows, tid & (NQ - 1))
                                         : rows_sum(ws.cnt, tid >> 8, nrows, tid & (NQ - 1));
    __syncthreads();
    CF_STAMP(5);
    int dp = 0;
    if (tid < NQ) {
      dp = gpart[0][tid] + gpart[1][tid] + gpart[2][tid] + gpart[3][tid] + partial[tid];
      s_tail[tid] += dp;
    }
    if (tid < B.nseg)  // advance every segment's bucket head by what it committed
      atomicAdd(&s_head[r_sg.L], max(0, min(ncommit - r_sg.rank, r_sg.n)));
    if (tid < NQ) {
      dp = wave_sum(dp);
      if ((tid & 63) == 0 && dp) atomicAdd((unsigned long long*)&ctl->pushes, (unsigned long long)dp);
    }
    __syncthreads();
    form_batch(qb, s_head, s_tail, s_minpush, s_wcap, nsegs, &s_nseg, &s_n);
    CF_STAMP(2);
  }
  // wait for every sub-round block's arrival -- each arrives once it has read the control block,
  // whether or not it has a sub-round to scatter (a block starting after the finalizer wrote would
  // read the next batch's words).  The grid fits the device at once (FAST_SUBS + 1 blocks of 1024
  // threads, two per CU), and sub-round blocks never wait, so they all get to run.
  if (tid < 64) {
    const int expect = G;
    long long t0 = 0;
    for (;;) {
      unsigned v = (tid < 8) ? __hip_atomic_load(&arrive[tid].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) v += __shfl_xor(v, o);
      v = __builtin_amdgcn_readlane(v, 0);
      if ((int)v >= expect) break;
      __builtin_amdgcn_s_sleep(1);
      const long long now = (long long)__builtin_amdgcn_s_memrealtime();
      if (t0 == 0) t0 = now;
      else if (now - t0 > SPIN_LIMIT_TICKS) {
        if (tid == 0) atomicOr(&ctl->error, ERR_TIMEOUT);
        break;
      }
    }
    if (tid < 8) arrive[tid].v = 0u;  // every arrival is in: reset for the next launch
    CF_STAMP(3);
  }
  __syncthreads();
  if (flags & 1) {
    // the rows k_resolve accumulated are consumed: zero them for the next batch
    const long long rows = (long long)((B.n + CH - 1) / CH) * NQ;
    for (long long k = tid; k < rows; k += 1024) ws.cnt[k] = 0;
    const int ns = s_nseg;
    for (int k = tid; k < ns; k += 1024) ctl->seg[k] = nsegs[k];
    if (tid < NQ) {
      ctl->qhead[tid] = s_head[tid];
      ctl->qtail[tid] = s_tail[tid];
    }
    if (tid < 64) {  // queued items left (host polling hint)
      int q = 0;
#pragma unroll
      for (int k = 0; k < NQ / 64; ++k) q += s_tail[tid + 64 * k] - s_head[tid + 64 * k];
      q = wave_sum(q);
      if (tid == 0) ctl->remaining = q;
    }
    if (tid == 0) {
      ctl->pops += ncommit;
      ctl->items += B.n;
      Batch nb;
      nb.mode = 0;
      nb.epoch = B.epoch + 1;
      nb.ncommit = 0;
      nb.nchunk = 0;
      nb.rrun = 0;
      nb.nseg = ns;
      nb.n = (ns > 0) ? s_n : 0;
      nb.L = (ns > 0) ? nsegs[0].L : -1;
      nb.bstart = (ns > 0) ? nsegs[0].bstart : 0;
      if (ns > 0 && ctl->spec.on)
        spec_begin(ctl, nb, nsegs[0].L, nsegs[0].bstart, s_tail[nsegs[0].L] - s_head[nsegs[0].L]);
      ctl->bat = nb;
      ctl->cbat.n = 0;
      ctl->cbat.nchunk = 0;
      ctl->wcap = s_wcap;
      ctl->cut = NONE;
      ctl->segcut = NONE;
      ctl->minpush = NQ;
      if (ns > 0) ctl->batches += 1;
      else ctl->done = 1;
    }
#ifdef MSEG_CF_PROF
    CF_STAMP(4);
    if (cfd && tid == 0) {  // header, queue-state loads, rows + segments + next batch, arrivals, writes
      atomicAdd(&cfd[0], (unsigned long long)(cf_t[0] - cf_t0));
      atomicAdd(&cfd[1], (unsigned long long)(cf_t[1] - cf_t[0]));
      atomicAdd(&cfd[2], (unsigned long long)(cf_t[5] - cf_t[1]));  // rows (+ a cut chunk's recount)
      atomicAdd(&cfd[3], (unsigned long long)(cf_t[2] - cf_t[5]));  // segments, next batch
      atomicAdd(&cfd[4], (unsigned long long)(cf_t[3] - cf_t[2]));
      atomicAdd(&cfd[5], (unsigned long long)(cf_t[4] - cf_t[3]));
      atomicAdd(&cfd[7], 1ull);
    }
#endif
  } else if (tid == 0) {
    if (flags & 2) {
      ctl->rgive = 0;
      ctl->bat.rrun = B.rrun + 1;
    } else if (flags & 4) {
      ctl->hold = B.epoch;
    }
  }
  __syncthreads();
  if (tid == 0 && ws.hmir) {
    const Batch nb = ctl->bat;
    __hip_atomic_store(ws.hmir + 1, ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 2, ctl->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 3, ctl->remaining, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 4, ctl->spec.on, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 5, ctl->spec_want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir + 6, fast_batch(nb, ctl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.hmir, iter, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// batches of up to FAST_CH chunks (the common case: 46-54 VGPRs, two blocks per CU)
__global__ __launch_bounds__(1024) void k_commit_fast(Ws ws, int iter) { commit_fast_body<false>(ws, iter); }
// up to FAST_PASS * FAST_CH chunks (large frames' generations: 16384^2 peaks at ~700 K items),
// each sub-round block taking several sub-rounds; held to 64 VGPRs so that two blocks per CU keep
// the whole grid resident (it spills some: only launched when the last report was such a batch)
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void k_commit_fast_mp(Ws ws, int iter) {
  commit_fast_body<true>(ws, iter);
}

// ---------------------------------------------------------------------------------------------
// Small batches, one workgroup (16 waves), many batches per launch.  Runs of small batches
// (interrupt cascades, generation tails) dominate the batch count; here each one costs a few
// workgroup barriers instead of three kernel boundaries.  Labels of the batch live in LDS and
// push decisions are pulled (an earlier non-WSHED batch item adjacent to the target pushes it
// first).  Exits, writing the queue state back, when the next batch is larger than SMALL_MAX,
// the flood is done, or on error.
// attempt_item with the dependencies' labels given per dependency slot (v[k] for it.dep[k]).
__device__ __forceinline__ bool attempt_item_slots(const Item& it, const int (&v)[16], int& lab_out,
                                                   unsigned& mask_out) {
  int lab = it.base_lab;
  bool unknown = false;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (it.dep[d] < 0) continue;
    if (v[d] == 0) unknown = true;
    else if (v[d] > 0) lab = fold_lab(lab, v[d]);
  }
  if (lab == WSHED) {
    lab_out = WSHED;
    mask_out = 0;
    return true;
  }
  if (unknown) return false;
  unsigned m = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (!((it.zero_mask >> d) & 1u)) continue;
    bool lose = false, undecided = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (it.dep[4 + 3 * d + k] < 0) continue;
      const int x = v[4 + 3 * d + k];
      if (x > 0) lose = true;
      else if (x == 0) undecided = true;
    }
    if (!lose) {
      if (undecided) return false;
      m |= 1u << d;
    }
  }
  lab_out = lab;
  mask_out = m;
  return true;
}

// Tiny batches (<= 64 items), wave 0 only, no block barriers: item i on lane i, labels and push
// decisions through register shuffles, the cut words through ballots, the ordered append through
// wave_rank on the queue state the small loop keeps in LDS (in-order LDS within one wave).
// Returns when the next batch has more than 64 items, the flood is done, or on error.
constexpr int TINY_MAX = 64;
constexpr int SERIAL_RUN = 4096;    // serial pops: clean pops after which batches pay again
constexpr int SERIAL_SWITCH = 16;   // a tiny batch cut before this many items -> serial pops
// k_serial_one's (a single flood's serial phases after its first): 4096 -> 16384 took the NC
// pipeline at 4096^2 1.97 -> 2.18 Mpx/s and album.jpg 969 -> 930 ms, the colour pipeline 3.34 -> 3.24
// (profiles/r06sp_ab_serial_run.log)
constexpr int SERIAL_RUN_ONE = 16384;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ void tiny_loop(const Ws& ws, Batch* s_B, Seg* s_seg, const int* s_qbase, int* s_head, int* s_tail,
                          int* wrow, int* s_wcap, int* s_err, int* s_nseg, int* s_n, int* s_ser, long long* cnt) {
  const int lane = lane_id();
  const int Wt = ws.Wt;
  for (;;) {
    wave_sync();
    const Batch B = *s_B;
    if (B.n == 0 || B.mode != 0 || B.n > TINY_MAX || *s_err) return;
    const int i = lane;
    const bool valid = i < B.n;
    Item it;
    int sg = 0;
    if (valid) {
      sg = (B.nseg == 1) ? 0 : seg_of_rank(s_seg, B.nseg, i);
      gather_item<false>(ws, s_seg, B.nseg, i, s_seg[sg].bstart + (i - s_seg[sg].rank), it);
    } else {
      it.p = 0;
      it.base_lab = WSHED;
      it.zero_mask = 0;
      it.wts = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) it.dep[k] = -1;
    }
    int mylab = 0;
    unsigned mymask = 0;
    bool done = !valid;
    for (int round = 0; round <= TINY_MAX && __any(!done); ++round) {  // deps point to lower lanes
      int snap[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) snap[k] = __shfl(mylab, it.dep[k] >= 0 ? it.dep[k] : lane);
      if (!done) {
        int lab;
        unsigned m;
        if (attempt_item_slots(it, snap, lab, m)) {
          if (lab == 0) {  // impossible for an exact queue
            *s_err = ERR_STATE;
            lab = WSHED;
          }
          mylab = lab;
          mymask = (lab == WSHED) ? 0u : m;
          done = true;
        }
      }
    }
    if (__any(!done)) {
      *s_err = ERR_STATE;
      return;
    }
    // cut words: interrupt (push below the item's level) and segment cut, lowest level pushed
    const int lvi = valid ? s_seg[sg].L : 0;
    bool lower = false;
    int tmin = NQ, mseg = NONE;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (!((mymask >> d) & 1u)) continue;
      const int t = (int)((it.wts >> (8 * d)) & 255u);
      if (t < lvi) lower = true;
      else tmin = min(tmin, t);
    }
    if (tmin < NQ && B.nseg > 1) mseg = seg_cut_for(s_seg, B.nseg, sg, tmin);
    const unsigned long long lowmask = __ballot(lower);
    const int cut = lowmask ? (__ffsll((long long)lowmask) - 1) : NONE;
    int minpush = lower ? 0 : tmin, segcut = mseg;
    minpush = wave_min(minpush);
    segcut = wave_min(segcut);
    int ncommit = B.n;
    if (cut != NONE) ncommit = min(ncommit, cut + 1);
    if (segcut != NONE) ncommit = min(ncommit, s_seg[segcut].rank);
    // commit labels, ordered append of the committed pushes
    const bool com = i < ncommit;
    if (com) st_state(ws, it.p, mylab);
    const unsigned mask = com ? mymask : 0u;
    int pos[4] = {0, 0, 0, 0};
    wave_rank(mask, it.wts, pos, wrow);  // wrow[level] = the wave's pushes at that level
    wave_sync();
    int pushed = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (!((mask >> d) & 1u)) continue;
      const int lv = (it.wts >> (8 * d)) & 255;
      const int dest = s_qbase[lv] + s_tail[lv] + pos[d];
      if (dest < 0 || (long long)dest >= ws.qcap) {
        *s_err = ERR_CAPACITY;
        continue;
      }
      const long long n = nb_of(it.p, d, Wt);
      st_state(ws, n, queued_state(dest));
      ws.qbuf[dest] = (int32_t)n;
      ++pushed;
    }
    wave_sync();
    // tails += the wave's per-level totals (one lane per distinct level), rows back to zero
    unsigned rem = mask;
    for (;;) {
      const unsigned long long act = __ballot(rem != 0);
      if (act == 0) break;
      const int leader = __ffsll((long long)act) - 1;
      const int myl = rem ? (int)((it.wts >> (8 * (__ffs(rem) - 1))) & 255u) : -1;
      const int lsel = __builtin_amdgcn_readlane(myl, leader);  // uniform lane: no LDS crossbar
      if (lane == leader) {
        s_tail[lsel] += wrow[lsel];
        wrow[lsel] = 0;
      }
#pragma unroll
      for (int d = 0; d < 4; ++d)
        if ((int)((it.wts >> (8 * d)) & 255u) == lsel) rem &= ~(1u << d);
      wave_sync();
    }
    pushed = wave_sum(pushed);
    if (lane < B.nseg) {
      const Seg s = s_seg[lane];
      s_head[s.L] += max(0, min(ncommit - s.rank, s.n));
    }
    wave_sync();
    const int wcap = next_wcap(*s_wcap, B.n, ncommit, cut != NONE && ncommit == cut + 1);
    if (lane == 0) {
      *s_wcap = wcap;
      cnt[0] += ncommit;
      cnt[1] += B.n;
      cnt[2] += pushed;
    }
    wave_sync();
    form_batch(s_qbase, s_head, s_tail, minpush, wcap, s_seg, s_nseg, s_n);
    wave_sync();
    if (lane == 0) {
      Batch nb;
      nb.mode = 0;
      nb.epoch = B.epoch + 1;
      nb.ncommit = 0;
      nb.nchunk = 0;
      nb.rrun = 0;
      nb.nseg = *s_nseg;
      nb.n = (*s_nseg > 0) ? *s_n : 0;
      nb.L = (*s_nseg > 0) ? s_seg[0].L : -1;
      nb.bstart = (*s_nseg > 0) ? s_seg[0].bstart : 0;
      *s_B = nb;
      if (*s_nseg > 0) cnt[3] += 1;
      if (cut != NONE && ncommit < SERIAL_SWITCH) *s_ser = 1;  // interrupt-dense: pop serially
    }
    wave_sync();
    if (*s_ser) return;
  }
}

// Serial pops: cv::watershed's own phase-2 loop (pop the oldest item of the lowest non-empty
// bucket, fold its labelled neighbours, push its unknown ones in L,R,T,B order) on the engine's own
// queue and state, for the interrupt-dense regime where batches commit a few items each: run by
// k_scan's wave 0 when a tiny batch commits fewer than SERIAL_SWITCH items before an interrupt, and
// by k_serial_multi's waves on many floods at once (serial_loop_lanes below).  Returns once a run
// of SERIAL_RUN pops pushed nothing below the popped level (batches pay again), or when the queue
// is empty, forming the next batch.

// Wait for every vector memory operation of the wave (s_waitcnt vmcnt(0); expcnt and lgkmcnt left
// alone), where the code knows a wait is due, so that the compiler need not place one where it
// cannot tell (a register written by a load in a branch, read after the join: its own wait there
// is vmcnt(0), behind every store issued since).
// The immediate is the gfx9 encoding (vmcnt[3:0] = 0, expcnt and lgkmcnt at their maxima, vmcnt[5:4]
// = 0); gfx10+ lay the fields out differently, so any other target is refused at compile time.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "vm_drain: s_waitcnt 0x0F70 is vmcnt(0) only in the gfx9 encoding (build for gfx950)"
#endif
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ int ld_qbuf_v(const Ws& ws, int slot) {
  return __hip_atomic_load(ws.qbuf + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// lowest non-empty bucket at or above `from` (NQ if none); wave-uniform
__device__ __forceinline__ int lowest_bucket(const int* head, const int* tail, int from) {
  const int lane = lane_id();
  int lo = NQ;
#pragma unroll
  for (int k = 0; k < NQ / 64; ++k) {
    const int l = lane * (NQ / 64) + k;
    if (l >= from && tail[l] > head[l]) lo = min(lo, l);
  }
  return wave_min(lo);
}

// serial_loop_lanes: the serial pops of one wave, with the pop's memory work spread over lanes:
// lane d < 4 loads the state of neighbour d and the other lanes the pixel's weights, in ONE load
// instruction; a pop's pushes are one store of queue slots and one of states (the popped pixel's
// label in the same instruction, lanes >= 4), their slots ranked among the pushing lanes in
// direction order (cv::watershed's push order).  The head of the popped bucket stays in a register
// while the loop stays on it; its next 64 slots sit in a register ring, so a pop only looks at the
// bucket's tail when the ring runs out.  Round 6 replaced a form whose every lane ran the same
// scalar program (~180 instructions a pop of scalar address arithmetic and an LDS round trip per
// push, issued one at a time by a lone wave): 92 notConnectedMarkers floods of one 1024^2 image
// 134 -> 170 Mpx/s (profiles/r06k_ab_serial_lanes.log), one such flood in k_scan 900 -> 810 ms
// (profiles/r06o_ab_serial_lanes_kscan.log).  The loads stay vector atomics: off the scalar cache,
// which does not see vector stores.
// Values the loop branches on are read from LDS through readfirstlane (and no store sits in a
// lane-divergent branch of its own): otherwise the compiler keeps them in vector registers and
// turns every branch of the loop into exec-mask code.
template <bool RELANE>
__device__ void serial_loop_lanes(const Ws& ws, Batch* s_B, Seg* s_seg, const int* s_qbase, int* s_head,
                                  int* s_tail, int* s_wcap, int* s_err, int* s_nseg, int* s_n, int* s_ser,
                                  long long* cnt, int spec_block, int* spec_cool, int run_limit = SERIAL_RUN) {
  const int lane = lane_id();
  const int marg = ws.marg;
  const int row = ws.Wt << 4;
  const Batch B0 = *s_B;
  const unsigned qcap32 = (unsigned)min(ws.qcap, (long long)0x7fffffff);
  int pops = 0, pushes = 0, run = 0;
  const int cool_lim = (spec_cool && *spec_cool > 0) ? *spec_cool : 0x7fffffff;
  int lo = __builtin_amdgcn_readfirstlane(lowest_bucket(s_head, s_tail, 0));
  int cl = -1, ch = 0, cb = 0;  // the bucket being popped: level, head (in a register), queue base
  int ring = 0, ring_h0 = 0, ring_end = 0;
#ifdef MSEG_SER_PROF
  unsigned long long ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, tprev = 0;  // load, fold, push, between, pushes, switches, refills, refill cycles, scan cycles
#endif
  while (lo < NQ) {
    if (lo != cl) {  // switch buckets (every lane stores the same value: no divergent branch)
      if (cl >= 0) s_head[cl] = ch;
      wave_sync();
#ifdef MSEG_SER_PROF
      ph[5] += 1;
#endif
      cl = lo;
      ch = __builtin_amdgcn_readfirstlane(s_head[lo]);
      cb = __builtin_amdgcn_readfirstlane(s_qbase[lo]);
      ring_end = ch;  // the ring is refilled before the first pop
    }
    if (ch >= ring_end) {  // the ring ran out: the bucket's tail decides
      const int ct = __builtin_amdgcn_readfirstlane(s_tail[cl]);
      if (ch >= ct) {  // empty: the next one up (LDS is current but for cl's head)
#ifdef MSEG_SER_PROF
        const unsigned long long E0 = __builtin_amdgcn_s_memtime();
#endif
        s_head[cl] = ch;
        wave_sync();
        cl = -1;
        lo = __builtin_amdgcn_readfirstlane(lowest_bucket(s_head, s_tail, lo + 1));
#ifdef MSEG_SER_PROF
        ph[8] += __builtin_amdgcn_s_memtime() - E0 + (unsigned)(lo & 0);
#endif
        continue;
      }
#ifdef MSEG_SER_PROF
      ph[6] += 1;
      const unsigned long long R0 = __builtin_amdgcn_s_memtime();
#endif
      ring_h0 = ch;  // its next 64 slots, one load per lane
      ring_end = ch + min(ct - ch, 64);
      ring = (ch + lane < ring_end) ? ld_qbuf_v(ws, cb + ch + lane) : 0;
      vm_drain();
#ifdef MSEG_SER_PROF
      ph[7] += __builtin_amdgcn_s_memtime() - R0 + (unsigned)(__builtin_amdgcn_readfirstlane(ring) & 0);
#endif
    }
    if (run >= run_limit) break;
    if (spec_block > 0 && lo >= spec_block) break;  // the cascade that stopped the speculative engine is done
    if (pops >= cool_lim) break;  // its cooldown is over
    // the speculative engine is being allocated (first entry into this regime): return soon, so
    // that the launches that carry it take the regime over
    if (ws.spec_lazy && pops >= 4096) break;
#ifdef MSEG_SER_PROF
    const unsigned long long T0 = __builtin_amdgcn_s_memtime();
    if (tprev) ph[3] += T0 - tprev;
#endif
    const int p = __builtin_amdgcn_readlane(ring, ch - ring_h0);
    // lane d < 4: neighbour d of tiled pixel pb is pb + (((pb & msk) != val) ? dn : dw) (nbi).
    // RELANE (k_scan, whose long-lived registers leave none for these): recomputed on every pop
    // from a lane id the compiler cannot hoist, instead of reloaded from scratch
    int lid = lane;
    if (RELANE) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0" : "=v"(lid));
    const bool nbl = lid < 4;
    const unsigned d8 = (unsigned)(lid & 3) << 3;  // the lane's byte of the packed per-direction constants
    const int msk = (int)__builtin_amdgcn_ubfe(0x0C0C0303u, d8, 8);
    const int val = (int)__builtin_amdgcn_ubfe(0x0C000300u, d8, 8);
    const int dn = __builtin_amdgcn_sbfe(0x04FC01FF, d8, 8);
    const int dw = (d8 < 16) ? __builtin_amdgcn_sbfe(0x00000DF3, d8, 8) : ((d8 == 16) ? 12 - row : row - 12);
    const int* ldbase = nbl ? ws.mk : ws.w4;
    const int pb = p + marg;
    const int idx = nbl ? pb + (((pb & msk) != val) ? dn : dw) - marg : p;
    const int v = __hip_atomic_load(ldbase + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const unsigned w4 = (unsigned)__builtin_amdgcn_readlane(v, 4);
#ifdef MSEG_SER_PROF
    const unsigned long long T1 = __builtin_amdgcn_s_memtime() + (w4 & 0u);
    ph[0] += T1 - T0;
#endif
    // the fold of the settled neighbours (fold_lab in direction order): 0 if none, their label if
    // they agree, WSHED otherwise -- i.e. from their largest and smallest label
    const bool pos = nbl && v > 0;
    int mx = pos ? v : 0, mn = pos ? v : 0x7fffffff;
    mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
    mn = min(mn, __builtin_amdgcn_update_dpp(0x7fffffff, mn, 0xB1, 0xF, 0xF, false));
    mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    mn = min(mn, __builtin_amdgcn_update_dpp(0x7fffffff, mn, 0x4E, 0xF, 0xF, false));
    const int smx = __builtin_amdgcn_readfirstlane(mx), smn = __builtin_amdgcn_readfirstlane(mn);
    int lab = (smx == 0) ? 0 : (smx == smn ? smx : WSHED);
    const bool bad = lab == 0;  // impossible for an exact queue
    if (bad) {
      *s_err = ERR_STATE;
      lab = WSHED;
    }
#ifdef MSEG_SER_PROF
    const unsigned long long T2 = __builtin_amdgcn_s_memtime() + (unsigned)(lab & 0);
    ph[1] += T2 - T1;
#endif
    ++ch;
    ++pops;
    // pushing lanes: neighbours in state 0 of a labelled pixel
    const bool push = nbl && v == 0 && lab != WSHED;
    const unsigned pm = (unsigned)__ballot(push);
    int sv = lab;  // lanes >= 4: the popped pixel's label (idx == p)
    int newlo = lo;
    bool ok = !nbl;  // lanes that store a state
    if (pm) {
      const int t = (int)__builtin_amdgcn_ubfe(w4, d8, 8);
      const int qb = s_qbase[t], qt = s_tail[t];
      int rank = 0;  // earlier pushing lanes of the same bucket (direction order)
      if (pm & (pm - 1)) {
#pragma unroll
        for (int e = 0; e < 3; ++e)
          rank += (((pm >> e) & 1u) && e < lane && (int)((w4 >> (8 * e)) & 255u) == t) ? 1 : 0;
      }
      const int dest = qb + qt + rank;
      if (__ballot(push && (unsigned)dest >= qcap32)) {
        *s_err = ERR_CAPACITY;
        break;
      }
      atomicAdd(&s_tail[t], push ? 1 : 0);  // (adds commute; lanes of the same bucket each add 1)
      pushes += __builtin_popcount(pm);
      int tm = push ? t : NQ;
      tm = min(tm, __builtin_amdgcn_update_dpp(NQ, tm, 0xB1, 0xF, 0xF, false));
      tm = min(tm, __builtin_amdgcn_update_dpp(NQ, tm, 0x4E, 0xF, 0xF, false));
      newlo = min(lo, __builtin_amdgcn_readfirstlane(tm));
      sv = push ? queued_state(dest) : lab;
      ok = ok || push;
      if (push) ws.qbuf[dest] = idx;
    }
    // the popped pixel's label and the pushed neighbours' queue states: one store
    if (ok) ws.mk[idx] = sv;
#ifdef MSEG_SER_PROF
    tprev = __builtin_amdgcn_s_memtime() + (unsigned)(newlo & 0);
    ph[2] += tprev - T2;
    ph[4] += __builtin_popcount(pm);
#endif
    run = (newlo < lo) ? 0 : run + 1;
    lo = newlo;
    if (bad) break;
  }
  if (cl >= 0) s_head[cl] = ch;
  wave_sync();
#ifdef MSEG_SER_PROF
  if (ws.diag && lane == 0) {
    for (int k = 0; k < 5; ++k) atomicAdd(&ws.diag[24 + k], ph[k]);
    atomicAdd(&ws.diag[29], (unsigned long long)pops);
    atomicAdd(&ws.diag[30], ph[7]);
    atomicAdd(&ws.diag[31], ph[8]);
  }
#endif
  if (lane == 0) {
    cnt[0] += pops;
    cnt[1] += pops;
    cnt[2] += pushes;
    *s_wcap = 0;  // the next batch: a whole generation
    if (spec_cool && *spec_cool > 0) *spec_cool = max(0, *spec_cool - pops);
  }
  wave_sync();
  form_batch(s_qbase, s_head, s_tail, 0, 0, s_seg, s_nseg, s_n);
  wave_sync();
  if (lane == 0) {
    Batch nb;
    nb.mode = 0;
    nb.epoch = B0.epoch + 1;
    nb.ncommit = 0;
    nb.nchunk = 0;
    nb.rrun = 0;
    nb.nseg = *s_nseg;
    nb.n = (*s_nseg > 0) ? *s_n : 0;
    nb.L = (*s_nseg > 0) ? s_seg[0].L : -1;
    nb.bstart = (*s_nseg > 0) ? s_seg[0].bstart : 0;
    *s_B = nb;
    *s_ser = 0;
    cnt[3] += pops;
  }
  wave_sync();
}

__device__ __forceinline__ void small_loop(const Ws& ws, int ser_next) {
  constexpr int NW = 16;
  Ctl* ctl = ws.ctl;
  __shared__ int s_lab[SMALL_MAX];
  __shared__ unsigned long long s_desc[SMALL_MAX];
  __shared__ int s_qbase[NQ], s_head[NQ], s_tail[NQ], s_tot[NQ];
  __shared__ int s_wcnt[NW][NQ];
  __shared__ Seg s_seg[NQ];
  __shared__ int s_cut, s_segcut, s_minpush, s_err, s_nseg, s_n, s_wcap;
  __shared__ int s_ser;  // 1: the interrupt-dense regime, tiny batches popped serially
  __shared__ int s_specgo, s_specblk;  // hand the regime to the speculative engine; its resume level
  __shared__ int s_specool;            // regime entries to skip first (SpecCtl.cool)
  __shared__ int s_lazyx;              // leave the launch: the speculative engine is being allocated
  __shared__ int s_sergo;              // leave the launch: k_serial_one (queued next) pops serially
  __shared__ Batch s_B;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const int Wt = ws.Wt;
  if (tid == 0) {
    s_B = ctl->bat;
    s_err = ctl->error;
    s_wcap = ctl->wcap;
    s_ser = 0;
    s_specgo = 0;
    s_lazyx = 0;
    s_sergo = 0;
    s_specblk = ws.spx ? ctl->spec.block : -1;  // -1: engine off
    s_specool = ctl->spec.cool;
  }
  if (tid < NQ) {
    s_qbase[tid] = ctl->qbase[tid];
    s_head[tid] = ctl->qhead[tid];
    s_tail[tid] = ctl->qtail[tid];
#pragma unroll
    for (int k = 0; k < NW; ++k) s_wcnt[k][tid] = 0;
    s_seg[tid] = ctl->seg[tid];
  }
  __syncthreads();
  long long nb_batches = 0, nb_pops = 0, nb_items = 0, nb_push = 0, iters = 0;
  bool worked = false;
  for (;;) {
    const Batch B = s_B;
    if (B.n == 0 || B.mode != 0 || B.n > SMALL_MAX || s_err) break;
    worked = true;
    if (B.n <= TINY_MAX) {  // runs of tiny batches: wave 0 alone, the other waves wait here
      if (wv == 0) {
        long long c4[4] = {0, 0, 0, 0};
        if (s_ser && s_specblk >= 0 && s_specool <= 0 && lowest_bucket(s_head, s_tail, 0) >= s_specblk) {
          if (lane == 0) s_specgo = 1;  // interrupt-dense: speculative generations from here on
        } else if (s_ser && ser_next) {
          // k_serial_one, queued right after this launch, pops them with its own register budget
          // (here the 1024-thread block's 128 VGPRs spill the loop's SGPRs into vector lanes)
          if (lane == 0) {
            s_sergo = 1;
            ctl->ser_seen = 1;
          }
        } else if (s_ser) {
          if (lane == 0) ctl->ser_seen = 1;  // the host queues k_serial_one from now on
          if (ws.spec_lazy && lane == 0) ctl->spec_want = 1;  // the host allocates the engine
          const unsigned long long t0 = ws.diag ? __builtin_amdgcn_s_memrealtime() : 0;
          serial_loop_lanes<true>(ws, &s_B, s_seg, s_qbase, s_head, s_tail, &s_wcap, &s_err, &s_nseg, &s_n, &s_ser, c4,
                            s_specblk > 0 ? s_specblk : 0, s_specblk >= 0 ? &s_specool : nullptr);
          if (ws.spec_lazy && lane == 0) s_lazyx = 1;
          if (ws.diag && lane == 0) {
            atomicAdd(&ws.diag[19], (unsigned long long)c4[0]);
            atomicAdd(&ws.diag[20], __builtin_amdgcn_s_memrealtime() - t0);
          }
          wave_sync();
          // the cascade that stopped the speculative engine is done, or its cooldown is over:
          // hand the regime back to it (not to a whole-bucket batch the next interrupt cuts again)
          if (s_specblk >= 0 && s_specool <= 0 && s_B.n > 0 && lowest_bucket(s_head, s_tail, 0) >= s_specblk &&
              lane == 0)
            s_specgo = 1;
        } else {
          const unsigned long long t0 = ws.diag ? __builtin_amdgcn_s_memrealtime() : 0;
          tiny_loop(ws, &s_B, s_seg, s_qbase, s_head, s_tail, s_wcnt[0], &s_wcap, &s_err, &s_nseg, &s_n, &s_ser, c4);
          if (ws.diag && lane == 0) {
            atomicAdd(&ws.diag[16], (unsigned long long)c4[3]);
            atomicAdd(&ws.diag[17], (unsigned long long)c4[0]);
            atomicAdd(&ws.diag[18], __builtin_amdgcn_s_memrealtime() - t0);
          }
        }
        if (tid == 0) {
          nb_pops += c4[0];
          nb_items += c4[1];
          nb_push += c4[2];
          nb_batches += c4[3];
        }
      }
      __syncthreads();
      if (s_specgo || s_lazyx || s_sergo) break;
      continue;
    }
    for (int k = tid; k < B.n; k += 1024) s_lab[k] = 0;
    if (tid == 0) {
      s_cut = NONE;
      s_segcut = NONE;
      s_minpush = NQ;
    }
    __syncthreads();
    // ---- resolve: item i on thread i % 1024, rounds in rank order, labels in LDS ----
    volatile int* vlab = s_lab;
    for (int base = 0; base < B.n; base += 1024) {
      const int i = base + tid;
      const bool valid = i < B.n;
      Item it;
      int sg = 0;
      if (valid) {
        sg = (B.nseg == 1) ? 0 : seg_of_rank(s_seg, B.nseg, i);
        gather_item<false>(ws, s_seg, B.nseg, i, s_seg[sg].bstart + (i - s_seg[sg].rank), it);
      }
      bool pending = valid;
      long long t0 = 0;
      int spins = 0;
      for (;;) {
        if (pending) {
          auto fetch = [&](int r) -> int { return vlab[r]; };
          int lab;
          unsigned m;
          if (attempt_item(it, fetch, lab, m)) {
            if (lab == 0) {
              s_err = ERR_STATE;
              lab = WSHED;
            }
            const unsigned mask = (lab == WSHED) ? 0u : m;
            const int lvi = s_seg[sg].L;
            s_desc[i] = make_desc(it.wts, mask, lvi, sg);
            vlab[i] = lab;
            pending = false;
            bool lower = false;
            int tmin = NQ;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              if (!((mask >> d) & 1u)) continue;
              const int t = (int)((it.wts >> (8 * d)) & 255u);
              if (t < lvi) lower = true;
              else tmin = min(tmin, t);
            }
            if (lower) {
              atomicMin(&s_cut, i);
              atomicMin(&s_minpush, 0);
            }
            if (tmin < NQ) {
              atomicMin(&s_minpush, tmin);
              if (B.nseg > 1) {
                const int mseg = seg_cut_for(s_seg, B.nseg, sg, tmin);
                if (mseg != NONE) atomicMin(&s_segcut, mseg);
              }
            }
          }
        }
        ++iters;
        if (!__any(pending)) break;
        if (++spins > 64) {
          __builtin_amdgcn_s_sleep(1);
          const long long now = (long long)__builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = now;
          else if (now - t0 > SPIN_LIMIT_TICKS) {
            if (pending) s_err = ERR_TIMEOUT;
            break;
          }
        }
      }
    }
    __syncthreads();
    if (s_err) break;
    int ncommit = B.n;
    if (s_cut != NONE) ncommit = min(ncommit, s_cut + 1);
    if (s_segcut != NONE) ncommit = min(ncommit, s_seg[s_segcut].rank);
    // ---- commit + ordered append, 1024 items per sub-round ----
    int pushed = 0;
    for (int i0 = 0; i0 < ncommit; i0 += 1024) {
      const int i = i0 + tid;
      const bool valid = i < ncommit;
      unsigned mask = 0, lvls = 0;
      long long p = 0;
      if (valid) {
        const unsigned long long d = s_desc[i];
        mask = (unsigned)(d >> 32) & 15u;
        lvls = (unsigned)d;
        const int sg = (int)((d >> 48) & 255);
        p = ws.qbuf[s_seg[sg].bstart + (i - s_seg[sg].rank)];
        st_state(ws, p, vlab[i]);
      }
      int pos[4] = {0, 0, 0, 0};
      wave_rank(mask, lvls, pos, s_wcnt[wv]);
      __syncthreads();
      if (tid < NQ) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
          const int t = s_wcnt[k][tid];
          s_wcnt[k][tid] = acc;
          acc += t;
        }
        s_tot[tid] = acc;
      }
      __syncthreads();
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if (!((mask >> d) & 1u)) continue;
        const int lv = (lvls >> (8 * d)) & 255;
        const int dest = s_qbase[lv] + s_tail[lv] + s_wcnt[wv][lv] + pos[d];
        if (dest < 0 || (long long)dest >= ws.qcap) {
          s_err = ERR_CAPACITY;
          continue;
        }
        const long long n = nb_of(p, d, Wt);
        st_state(ws, n, queued_state(dest));
        ws.qbuf[dest] = (int32_t)n;
        ++pushed;
      }
      __syncthreads();
      if (tid < NQ) {
        s_tail[tid] += s_tot[tid];
#pragma unroll
        for (int k = 0; k < NW; ++k) s_wcnt[k][tid] = 0;
      }
      __syncthreads();
    }
    const int npush = block_sum(pushed);
    if (tid < B.nseg) {
      const Seg s = s_seg[tid];
      s_head[s.L] += max(0, min(ncommit - s.rank, s.n));
    }
    if (tid == 0) {
      nb_pops += ncommit;
      nb_items += B.n;
      nb_push += npush;
      s_wcap = next_wcap(s_wcap, B.n, ncommit, s_cut != NONE && ncommit == s_cut + 1);
      if (ws.diag) atomicAdd(&ws.diag[23], (unsigned long long)ncommit);
    }
    __syncthreads();
    form_batch(s_qbase, s_head, s_tail, s_minpush, s_wcap, s_seg, &s_nseg, &s_n);
    __syncthreads();
    if (tid == 0) {
      Batch nb;
      nb.mode = 0;
      nb.epoch = B.epoch + 1;
      nb.ncommit = 0;
      nb.nchunk = 0;
      nb.rrun = 0;
      nb.nseg = s_nseg;
      nb.n = (s_nseg > 0) ? s_n : 0;
      nb.L = (s_nseg > 0) ? s_seg[0].L : -1;
      nb.bstart = (s_nseg > 0) ? s_seg[0].bstart : 0;
      s_B = nb;
      if (s_nseg > 0) ++nb_batches;
    }
    __syncthreads();
  }
  // write the queue state back for the multi-block kernels
  if (ws.diag && lane == 0 && iters) atomicAdd(&ws.diag[5], (unsigned long long)iters);
  if (!worked) {
    if (tid == 0 && s_err && !ctl->error) ctl->error = s_err;
    return;
  }
  if (ws.diag && tid == 0) atomicAdd(&ws.diag[6], (unsigned long long)nb_batches + 1);
  __syncthreads();
  if (tid < NQ) {
    ctl->qhead[tid] = s_head[tid];
    ctl->qtail[tid] = s_tail[tid];
  }
  const int q = block_sum(tid < NQ ? s_tail[tid] - s_head[tid] : 0);
  if (tid == 0) ctl->remaining = q;
  for (int k = tid; k < s_B.nseg; k += 1024) ctl->seg[k] = s_seg[k];
  if (tid == 0) {
    Batch nb = s_B;
    if (s_specgo) {
      spec_begin(ctl, nb, nb.L, s_qbase[nb.L] + s_head[nb.L], s_tail[nb.L] - s_head[nb.L]);
      if (ctl->spec.fresh || ctl->spec.tstart == 0) {  // flood start, or after a cooldown: judge anew
        ctl->spec.fresh = 0;
        ctl->spec.accg = 0;
        ctl->spec.tstart = (long long)__builtin_amdgcn_s_memrealtime();
        ctl->spec.tspec = ctl->spec.pspec = 0;
        ctl->spec.pstart = ctl->pops + nb_pops;  // nb_pops: this loop's, added below
      }
      ctl->spec.on = 1;
      ctl->spec.block = 0;
    }
    ctl->bat = nb;
    ctl->wcap = s_wcap;
    ctl->spec.cool = s_specool;
    if (s_sergo) ctl->ser_go = 1;
    ctl->cut = NONE;
    ctl->segcut = NONE;
    ctl->minpush = NQ;
    ctl->batches += nb_batches;
    ctl->pops += nb_pops;
    ctl->items += nb_items;
    ctl->pushes += nb_push;
    ctl->lpops += nb_pops;
    ctl->lpushes += nb_push;
    if (s_err) ctl->error |= s_err;
    if (s_B.n == 0 && !s_err) ctl->done = 1;
  }
}

// ---------------------------------------------------------------------------------------------
// k_serial_one: the serial pops of ONE flood of the full engine, queued after k_scan while the
// flood is in the serial regime (Ctl.ser_seen): when k_scan's small-batch loop reaches serial pops
// it stops (Ctl.ser_go) and this one-wave kernel pops them -- the same loop as k_serial_multi's,
// with the speculative engine's resume level and cooldown as k_scan's small-batch loop has them --
// then hands the regime back exactly as that loop would (the next batch, or a speculative
// generation).  A wave of its own pops at ≈0.6 µs against ≈0.8 inside k_scan, whose 1024-thread
// block leaves the loop 128 VGPRs and spills its SGPRs into vector lanes.
__global__ __launch_bounds__(64) void k_serial_one(Ws ws) {
  Ctl* ctl = ws.ctl;
  if (!ctl->ser_go) return;
  const int lane = lane_id();
  const Batch B0 = ctl->bat;
  if (ctl->done || ctl->error || B0.n == 0 || B0.mode != 0) {
    if (lane == 0) ctl->ser_go = 0;
    return;
  }
  __shared__ int s_qbase[NQ], s_head[NQ], s_tail[NQ];
  __shared__ Seg s_seg[NQ];
  __shared__ Batch s_B;
  __shared__ int s_wcap, s_err, s_nseg, s_n, s_ser, s_specool;
  const int specblk = ws.spx ? ctl->spec.block : -1;  // -1: engine off
#pragma unroll
  for (int k = 0; k < NQ / 64; ++k) {
    const int b = 64 * k + lane;
    s_qbase[b] = ctl->qbase[b];
    s_head[b] = ctl->qhead[b];
    s_tail[b] = ctl->qtail[b];
  }
  if (lane == 0) {
    s_B = B0;
    s_wcap = 0;
    s_err = 0;
    s_ser = 1;
    s_specool = ctl->spec.cool;
    if (ws.spec_lazy) ctl->spec_want = 1;  // the host allocates the engine
  }
  wave_sync();
  long long cnt[4] = {0, 0, 0, 0};
  const unsigned long long t0 = ws.diag ? __builtin_amdgcn_s_memrealtime() : 0;
  serial_loop_lanes<false>(ws, &s_B, s_seg, s_qbase, s_head, s_tail, &s_wcap, &s_err, &s_nseg, &s_n, &s_ser, cnt,
                           specblk > 0 ? specblk : 0, specblk >= 0 ? &s_specool : nullptr, SERIAL_RUN_ONE);
  wave_sync();
  // the cascade that stopped the speculative engine is done, or its cooldown is over: hand the
  // regime back to it (as k_scan's small-batch loop does)
  const bool specgo = specblk >= 0 && s_specool <= 0 && s_B.n > 0 &&
                      __builtin_amdgcn_readfirstlane(lowest_bucket(s_head, s_tail, 0)) >= specblk;
  for (int k = lane; k < NQ; k += 64) {
    ctl->qhead[k] = s_head[k];
    ctl->qtail[k] = s_tail[k];
  }
  const int ns = s_nseg;
  for (int k = lane; k < ns; k += 64) ctl->seg[k] = s_seg[k];
  int q = 0;
#pragma unroll
  for (int k = 0; k < NQ / 64; ++k) q += s_tail[lane + 64 * k] - s_head[lane + 64 * k];
  q = wave_sum(q);
  if (lane == 0) {
    Batch nb = s_B;
    if (specgo) {
      spec_begin(ctl, nb, nb.L, s_qbase[nb.L] + s_head[nb.L], s_tail[nb.L] - s_head[nb.L]);
      if (ctl->spec.fresh || ctl->spec.tstart == 0) {  // flood start, or after a cooldown: judge anew
        ctl->spec.fresh = 0;
        ctl->spec.accg = 0;
        ctl->spec.tstart = (long long)__builtin_amdgcn_s_memrealtime();
        ctl->spec.tspec = ctl->spec.pspec = 0;
        ctl->spec.pstart = ctl->pops + cnt[0];  // this launch's pops, added below
      }
      ctl->spec.on = 1;
      ctl->spec.block = 0;
    }
    ctl->bat = nb;
    ctl->wcap = 0;
    ctl->spec.cool = s_specool;
    ctl->cut = NONE;
    ctl->segcut = NONE;
    ctl->minpush = NQ;
    ctl->remaining = q;
    ctl->batches += cnt[3];
    ctl->pops += cnt[0];
    ctl->items += cnt[1];
    ctl->pushes += cnt[2];
    ctl->lpops += cnt[0];
    ctl->lpushes += cnt[2];
    ctl->ser_go = 0;
    if (s_err) ctl->error |= s_err;
    if (s_B.n == 0 && !s_err) ctl->done = 1;
    if (ws.diag) {
      atomicAdd(&ws.diag[19], (unsigned long long)cnt[0]);
      atomicAdd(&ws.diag[20], __builtin_amdgcn_s_memrealtime() - t0);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_serial_multi: the serial pops of MANY floods in one launch (the batch entry points' many-floods
// mode, msg_set_batch_floods): block f = one wave = flood f, each flood in its own workspace
// (wss[f]).  Photographs and scattered seeds put cv::watershed's exact order in its serial regime
// -- chains of dependent pops, a lone wave's memory latency per pop -- so a
// batch of such frames is bound by the number of floods in flight: here every flood of the call
// (hundreds), instead of the 4-8 streams over which the full engine's floods overlap.  Each wave
// runs the serial pops (serial_loop_lanes) on its flood from wherever it stands
// (after phase 1, or after a batch of the full engine) until its queue is empty, or until
// run_limit consecutive pops pushed nothing below their own level (batches pay again: the host
// finishes that flood with the full engine), then writes the queue state back and forms the next
// batch.  No wave waits for another: each block only touches its own flood.  A flood of zero
// pixels has no workspace (ctl == nullptr: flood_begin returns before binding it) and no work.
// (Round 4 measured a form with deferred stores and LDS rings, k_serial's: album.jpg 1362 against
// 1176 ms for this in-loop form; it was removed in round 5.)
__global__ __launch_bounds__(64) void k_serial_multi(const Ws* __restrict__ wss, int n, int run_limit) {
  const int f = blockIdx.x;
  if (f >= n) return;
  // loaded through the constant address space, the workspace's pointers are taken for global ones
  // (global_load / global_store; flat ones also count against the LDS counter, so that every LDS
  // wait of the pop loop also waited for the previous pop's stores)
#if defined(__HIP_DEVICE_COMPILE__)
  const Ws ws = ((const __attribute__((address_space(4))) Ws*)wss)[f];
#else
  const Ws ws = wss[f];  // the host pass of the single-source build: never runs
#endif
  Ctl* ctl = ws.ctl;
  if (ctl == nullptr || ws.N == 0) return;
  const int lane = lane_id();
  const Batch B0 = ctl->bat;
  if (ctl->done || ctl->error || B0.n == 0 || B0.mode != 0) return;
  __shared__ int s_qbase[NQ], s_head[NQ], s_tail[NQ];
  __shared__ Seg s_seg[NQ];
  __shared__ Batch s_B;
  __shared__ int s_wcap, s_err, s_nseg, s_n, s_ser;
#pragma unroll
  for (int k = 0; k < NQ / 64; ++k) {
    const int b = 64 * k + lane;
    s_qbase[b] = ctl->qbase[b];
    s_head[b] = ctl->qhead[b];
    s_tail[b] = ctl->qtail[b];
  }
  if (lane == 0) {
    s_B = B0;
    s_B.mode = 0;
    s_wcap = 0;
    s_err = 0;
    s_ser = 1;
  }
  wave_sync();
  long long cnt[4] = {0, 0, 0, 0};
  serial_loop_lanes<false>(ws, &s_B, s_seg, s_qbase, s_head, s_tail, &s_wcap, &s_err, &s_nseg, &s_n, &s_ser, cnt,
                           0, nullptr, run_limit);
  wave_sync();
  for (int k = lane; k < NQ; k += 64) {
    ctl->qhead[k] = s_head[k];
    ctl->qtail[k] = s_tail[k];
  }
  const int ns = s_nseg;
  for (int k = lane; k < ns; k += 64) ctl->seg[k] = s_seg[k];
  int q = 0;
#pragma unroll
  for (int k = 0; k < NQ / 64; ++k) q += s_tail[lane + 64 * k] - s_head[lane + 64 * k];
  q = wave_sum(q);
  if (lane == 0) {
    const Batch nb = s_B;
    ctl->bat = nb;
    ctl->wcap = 0;
    ctl->cut = NONE;
    ctl->segcut = NONE;
    ctl->minpush = NQ;
    ctl->remaining = q;
    ctl->batches += cnt[0];
    ctl->pops += cnt[0];
    ctl->items += cnt[1];
    ctl->pushes += cnt[2];
    ctl->lpops += cnt[0];
    ctl->lpushes += cnt[2];
    if (s_err) ctl->error |= s_err;
    if (nb.n == 0 && !s_err) ctl->done = 1;
  }
}

// ---------------------------------------------------------------------------------------------
// colorByIndexes (PictureService.java:913-936) + optional BGR2GRAY, 4 pixels per thread.
__global__ __launch_bounds__(256) void k_colorize(const int32_t* __restrict__ lab, long long N,
                                                  int depth, const uint8_t* __restrict__ pal,
                                                  uint8_t* __restrict__ dst,
                                                  uint8_t* __restrict__ gray) {
  extern __shared__ __attribute__((aligned(16))) uint32_t spal[];
  const bool lds_pal = pal != nullptr && depth <= PAL_LDS_MAX;
  if (lds_pal) {
    for (int k = threadIdx.x; k < depth; k += blockDim.x)
      spal[k] = (uint32_t)pal[3 * k] | ((uint32_t)pal[3 * k + 1] << 8) | ((uint32_t)pal[3 * k + 2] << 16);
    __syncthreads();
  }
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long q = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; q < N; q += stride) {
    uint32_t col[4];
    const int cnt = (int)min(4ll, N - q);
    int l[4];
    if (cnt == 4 && (q & 3) == 0) {
      const int4 v = *reinterpret_cast<const int4*>(lab + q);
      l[0] = v.x; l[1] = v.y; l[2] = v.z; l[3] = v.w;
    } else {
      for (int k = 0; k < 4; ++k) l[k] = (k < cnt) ? lab[q + k] : 0;
    }
    for (int k = 0; k < 4; ++k) {
      const int x = l[k];
      uint32_t c = 0;
      if (x > 0 && x <= depth) {
        if (pal == nullptr) c = 0xffffffu;
        else if (lds_pal) c = spal[x - 1];
        else c = (uint32_t)pal[3 * (x - 1)] | ((uint32_t)pal[3 * (x - 1) + 1] << 8) |
                 ((uint32_t)pal[3 * (x - 1) + 2] << 16);
      }
      col[k] = c;
    }
    if (cnt == 4) {
      // 12 output bytes: B0G0R0B1 G1R1B2G2 R2B3G3R3
      const uint32_t w0 = (col[0] & 0xffffffu) | (col[1] << 24);
      const uint32_t w1 = ((col[1] >> 8) & 0xffffu) | (col[2] << 16);
      const uint32_t w2 = ((col[2] >> 16) & 0xffu) | (col[3] << 8);
      uint8_t* o = dst + q * 3;
      if ((((uintptr_t)o) & 3) == 0) {
        reinterpret_cast<uint32_t*>(o)[0] = w0;
        reinterpret_cast<uint32_t*>(o)[1] = w1;
        reinterpret_cast<uint32_t*>(o)[2] = w2;
      } else {
        for (int k = 0; k < 4; ++k) {
          o[3 * k] = col[k] & 255; o[3 * k + 1] = (col[k] >> 8) & 255; o[3 * k + 2] = (col[k] >> 16) & 255;
        }
      }
    } else {
      for (int k = 0; k < cnt; ++k) {
        uint8_t* o = dst + (q + k) * 3;
        o[0] = col[k] & 255; o[1] = (col[k] >> 8) & 255; o[2] = (col[k] >> 16) & 255;
      }
    }
    if (gray) {
      uint32_t g4 = 0;
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = col[k] & 255, g = (col[k] >> 8) & 255, r = (col[k] >> 16) & 255;
        const uint32_t y = (1868u * b + 9617u * g + 4899u * r + 8192u) >> 14;
        g4 |= y << (8 * k);
      }
      if (cnt == 4 && (q & 3) == 0) *reinterpret_cast<uint32_t*>(gray + q) = g4;
      else for (int k = 0; k < cnt; ++k) gray[q + k] = (g4 >> (8 * k)) & 255;
    }
  }
}

// Diagnostics for ERR_LEFTOVER (msg_set_diag on): classify the queued states left after a flood.
// out[0] phase-1 states, out[1] queued states whose slot lies below its bucket's head (popped, so
// the label write was lost), out[2] queued states whose slot holds another pixel (the push was
// overwritten), out[3] all leftovers, out[4] / out[5] the last one's tiled index and slot.
__global__ __launch_bounds__(256) void k_leftover_diag(Ws ws, long long nt, unsigned long long* out) {
  const Ctl* ctl = ws.ctl;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (long long)gridDim.x * blockDim.x) {
    const int s = ws.mk[t];
    if (s > -3) continue;
    atomicAdd(out + 3, 1ull);
    if (is_p1(s)) {
      atomicAdd(out + 0, 1ull);
      continue;
    }
    const int slot = -3 - s;
    int lv = 0;
    while (lv + 1 < NQ && ctl->qbase[lv + 1] <= slot) ++lv;
    if (slot < ctl->qbase[lv] + ctl->qhead[lv]) atomicAdd(out + 1, 1ull);
    if ((long long)slot < ws.qcap && ws.qbuf[slot] != (int32_t)t) atomicAdd(out + 2, 1ull);
    out[4] = (unsigned long long)t;
    out[5] = (unsigned long long)slot;
  }
}

// ---------------------------------------------------------------------------------------------
// End of the flood: tiled states -> the caller's row-major label map (cv::watershed's in-place
// markers), fused with colorByIndexes (PictureService.java:913-936) + optional BGR2GRAY when dst
// is given.  One thread = one 4x4 tile: one 128-B line in, four 16-B label rows out.
__device__ __forceinline__ uint32_t label_colour(int x, int depth, const uint8_t* pal, bool lds_pal,
                                                 const uint32_t* spal) {
  if (x <= 0 || x > depth) return 0;
  if (pal == nullptr) return 0xffffffu;
  if (lds_pal) return spal[x - 1];
  return (uint32_t)pal[3 * (x - 1)] | ((uint32_t)pal[3 * (x - 1) + 1] << 8) |
         ((uint32_t)pal[3 * (x - 1) + 2] << 16);
}

__global__ __launch_bounds__(256) void k_untile(const int32_t* __restrict__ mk, int H, int W, int Wt,
                                                int32_t* __restrict__ lab, int depth,
                                                const uint8_t* __restrict__ pal,
                                                uint8_t* __restrict__ dst, uint8_t* __restrict__ gray,
                                                int* __restrict__ err) {
  // lane = one tile row (16 B of states = 4 pixels): loads are lane-contiguous (a wave reads 16
  // whole tiles), and the 16 lanes of one tile row of a wave store 256 B of labels, 192 B of
  // colours and 64 B of gray, each one 16-B / 12-B / 4-B store per lane (the 8-B unit layout it
  // replaces stored colours as three 2-B pieces: 33.5 -> 28.3 us at 4096^2 in
  // scripts/exp/stream_variants.hip).  Frames are < 2^29 pixels: 32-bit tile arithmetic.
  extern __shared__ __attribute__((aligned(16))) uint32_t spal[];
  const bool lds_pal = dst != nullptr && pal != nullptr && depth <= PAL_LDS_MAX;
  if (lds_pal) {
    for (int k = threadIdx.x; k < depth; k += blockDim.x)
      spal[k] = (uint32_t)pal[3 * k] | ((uint32_t)pal[3 * k + 1] << 8) | ((uint32_t)pal[3 * k + 2] << 16);
    __syncthreads();
  }
  const unsigned nrows = (unsigned)((H + 3) >> 2) * (unsigned)Wt * 4u;
  const bool w4 = (W & 3) == 0;
  const bool v4 = w4 && (((uintptr_t)lab) & 15) == 0;
  const bool v3 = w4 && dst != nullptr && (((uintptr_t)dst) & 3) == 0;
  const bool vg = w4 && gray != nullptr && (((uintptr_t)gray) & 3) == 0;
  for (unsigned u = blockIdx.x * blockDim.x + threadIdx.x; u < nrows; u += gridDim.x * blockDim.x) {
    const unsigned tt = u >> 2, ty = tt / (unsigned)Wt;
    const int r = (int)(ty * 4u + (u & 3u)), c = (int)((tt - ty * (unsigned)Wt) * 4u);
    if (r >= H) continue;
    const int4 s = reinterpret_cast<const int4*>(mk)[u];
    const int l[4] = {s.x, s.y, s.z, s.w};
    const unsigned q = (unsigned)r * (unsigned)W + (unsigned)c;
    const int cnt = min(4, W - c);
    // consistency: the flood pops everything it queues, so no queued or phase-1 state (<= -3) is
    // left (a lost push or label write would otherwise end as a silently wrong label)
    bool left = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) left |= j < cnt && l[j] <= -3;
    if (left) atomicOr(err, ERR_LEFTOVER);
    // the outputs are not read again here: nontemporal stores (35.3 -> 33.2 us in the bench step)
    typedef int i4nt __attribute__((ext_vector_type(4)));
    if (cnt == 4 && v4) __builtin_nontemporal_store((i4nt){s.x, s.y, s.z, s.w}, reinterpret_cast<i4nt*>(lab + q));
    else for (int j = 0; j < cnt; ++j) lab[q + j] = l[j];
    if (dst == nullptr) continue;
    uint32_t col[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = label_colour(l[j], depth, pal, lds_pal, spal);
    uint8_t* o = dst + 3u * q;
    if (cnt == 4 && v3) {  // B0G0R0B1 G1R1B2G2 R2B3G3R3
      uint32_t* o4 = reinterpret_cast<uint32_t*>(o);
      __builtin_nontemporal_store(col[0] | (col[1] << 24), o4);
      __builtin_nontemporal_store((col[1] >> 8) | (col[2] << 16), o4 + 1);
      __builtin_nontemporal_store((col[2] >> 16) | (col[3] << 8), o4 + 2);
    } else {
      for (int j = 0; j < cnt; ++j) {
        o[3 * j] = col[j] & 255;
        o[3 * j + 1] = (col[j] >> 8) & 255;
        o[3 * j + 2] = (col[j] >> 16) & 255;
      }
    }
    if (gray) {
      uint32_t g4 = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t bb = col[j] & 255, gg = (col[j] >> 8) & 255, rr = (col[j] >> 16) & 255;
        g4 |= ((1868u * bb + 9617u * gg + 4899u * rr + 8192u) >> 14) << (8 * j);
      }
      if (cnt == 4 && vg) *reinterpret_cast<uint32_t*>(gray + q) = g4;
      else for (int j = 0; j < cnt; ++j) gray[q + j] = (g4 >> (8 * j)) & 255;
    }
  }
}

}  // namespace msg
