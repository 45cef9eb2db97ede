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
// Data in HBM (N = rows*cols pixels, all dense row-major):
//   mk   int32[N]  label state: >0 label, 0 unknown, -1 WSHED/frame, -2 queued (serial IN_QUEUE)
//   wr,wd u8[N]    L-inf BGR distance to the right / lower neighbour (the colour-distance stencil)
//   qpos int32[N]  absolute queue slot of a queued pixel (valid while mk == -2)
//   qbuf int32[..] 256 bucket FIFOs, bucket L = qbuf[qbase[L] + head[L] .. qbase[L] + tail[L])
//                  sized exactly by a per-level histogram of each pixel's distinct edge weights
//   tl   u64[N]    per-rank {epoch, label} granule of the current batch (in-launch hand-off)
//   desc u64[N]    per-rank push descriptor: mask (4 bits) << 32 | four 8-bit levels
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

__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------
// Stand-alone colour-distance stencil (exposed as msg_edge_weights_dev; the same arithmetic is
// fused into k_prep).  One thread = 4 consecutive pixels of a row.
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
// colour-distance stencil and the bucket-capacity histogram.  One block = one CH-pixel chunk.
// mk_in may alias ws.mk: a pixel's "> 0" status never changes here and frame neighbours are
// excluded by coordinates, so the in-place rewrite is race-free.
__global__ __launch_bounds__(BS) void k_prep(Ws ws, const int32_t* mk_in) {
  __shared__ unsigned caph[NQ];
  __shared__ int ntot;
  const int tid = threadIdx.x;
  caph[tid] = 0;
  if (tid == 0) ntot = 0;
  __syncthreads();
  const int H = ws.H, W = ws.W;
  const long long N = ws.N;
  const long long c0 = (long long)blockIdx.x * CH;
  int mycount = 0;
  for (int s = 0; s < SUB; ++s) {
    const long long p = c0 + s * BS + tid;
    if (p >= N) break;
    const int r = (int)(p / W), c = (int)(p - (long long)r * W);
    const uint8_t* ip = ws.img + p * 3;
    const int wright = (c + 1 < W) ? cdiff3(ip, ip + 3) : 0;
    const int wdown = (r + 1 < H) ? cdiff3(ip, ip + 3 * (long long)W) : 0;
    ws.wr[p] = (uint8_t)wright;
    ws.wd[p] = (uint8_t)wdown;
    int32_t out;
    if (r == 0 || r == H - 1 || c == 0 || c == W - 1) {
      out = WSHED;
    } else {
      const int32_t m = mk_in[p];
      if (m > 0) {
        out = m;
      } else {
        // interior neighbours (the frame is WSHED in the serial code and never counts)
        const int wleft = (c >= 2) ? cdiff3(ip, ip - 3) : -1;
        const int wup = (r >= 2) ? cdiff3(ip, ip - 3 * (long long)W) : -1;
        const int wr_i = (c <= W - 3) ? wright : -1;
        const int wd_i = (r <= H - 3) ? wdown : -1;
        int lvl = 256;
        if (wleft >= 0 && mk_in[p - 1] > 0) lvl = min(lvl, wleft);
        if (wr_i >= 0 && mk_in[p + 1] > 0) lvl = min(lvl, wr_i);
        if (wup >= 0 && mk_in[p - W] > 0) lvl = min(lvl, wup);
        if (wd_i >= 0 && mk_in[p + W] > 0) lvl = min(lvl, wd_i);
        if (lvl < 256) {
          out = INQ;
          ws.lv1[p] = (uint8_t)lvl;
          ++mycount;
        } else {
          out = 0;
        }
        // this pixel may be queued once, at one of its distinct interior edge weights
        if (wleft >= 0) atomicAdd(&caph[wleft], 1u);
        if (wr_i >= 0 && wr_i != wleft) atomicAdd(&caph[wr_i], 1u);
        if (wup >= 0 && wup != wleft && wup != wr_i) atomicAdd(&caph[wup], 1u);
        if (wd_i >= 0 && wd_i != wleft && wd_i != wr_i && wd_i != wup) atomicAdd(&caph[wd_i], 1u);
      }
    }
    ws.mk[p] = out;
  }
  if (mycount) atomicAdd(&ntot, mycount);
  __syncthreads();
  if (caph[tid]) atomicAdd(&ws.ctl->cap[tid], caph[tid]);
  if (tid == 0) ws.tot[blockIdx.x] = ntot;
}

// ---------------------------------------------------------------------------------------------
// Column scan: coff[c][lv] = tail[lv] + sum_{c' < c} cnt[c'][lv]   (c < nch), tail += totals.
// `partial` (LDS, may be null) replaces the counts of the last chunk.  1024 threads.
__device__ void column_scan(const int* cnt, int* coff, int nch, const int* partial, int* tail) {
  __shared__ int gs[4][NQ];
  const int tid = threadIdx.x;
  const int lv = tid & (NQ - 1), g = tid >> 8;
  const int per = (nch + 3) >> 2;
  const int a = min(nch, g * per), b = min(nch, a + per);
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
  __syncthreads();
  if (g == 0) tail[lv] += gs[0][lv] + gs[1][lv] + gs[2][lv] + gs[3][lv];
  __syncthreads();
}

__device__ int column_total(int lv_total) {
  __shared__ int acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  if (lv_total) atomicAdd(&acc, lv_total);
  __syncthreads();
  return acc;
}

// Pick the lowest non-empty bucket as the next batch (or finish).  1024 threads, after tails
// are final.  Writes bat[nxt].
__device__ void choose_next(Ctl* ctl, int nxt, unsigned epoch) {
  __shared__ int lmin;
  const int tid = threadIdx.x;
  if (tid == 0) lmin = NQ;
  __syncthreads();
  if (tid < NQ && ctl->qhead[tid] < ctl->qtail[tid]) atomicMin(&lmin, tid);
  __syncthreads();
  if (tid == 0) {
    Batch nb;
    nb.mode = 0;
    nb.epoch = epoch;
    nb.ncommit = 0;
    nb.nchunk = 0;
    if (lmin < NQ) {
      nb.L = lmin;
      nb.bstart = ctl->qbase[lmin] + ctl->qhead[lmin];
      nb.n = ctl->qtail[lmin] - ctl->qhead[lmin];
      ctl->batches += 1;
    } else {
      nb.L = -1;
      nb.bstart = 0;
      nb.n = 0;
      ctl->done = 1;
    }
    ctl->bat[nxt] = nb;
    ctl->cut[nxt] = NONE;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// Init scan (1 block x 1024): bucket bases from the capacity histogram; exclusive scan of the
// per-chunk phase-1 counts (compaction offsets); sets up the phase-1 pseudo-batch in bat[1].
__global__ __launch_bounds__(1024) void k_init_scan(Ws ws, int npxchunk, unsigned epoch0) {
  Ctl* ctl = ws.ctl;
  const int tid = threadIdx.x;
  __shared__ long long wsum[16];
  __shared__ long long total_items;
  if (tid == 0) {
    long long acc = 0;
    for (int l = 0; l < NQ; ++l) {
      ctl->qbase[l] = (int)acc;
      acc += ctl->cap[l];
    }
    ctl->qbase[NQ] = (int)min(acc, (long long)0x7fffffff);
    if (acc > ws.qcap) ctl->error = ERR_CAPACITY;
  }
  // exclusive scan of tot[0..npxchunk) -> choff, 1024 threads, contiguous per-thread ranges
  const int per = (npxchunk + 1023) / 1024;
  const int a = min(npxchunk, tid * per), b = min(npxchunk, a + per);
  long long s = 0;
  for (int c = a; c < b; ++c) s += ws.tot[c];
  // block exclusive scan of s
  const int lane = tid & 63, wv = tid >> 6;
  long long x = s;
  for (int o = 1; o < 64; o <<= 1) {
    long long y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (tid == 0) {
    long long acc = 0;
    for (int k = 0; k < 16; ++k) {
      long long t = wsum[k];
      wsum[k] = acc;
      acc += t;
    }
    total_items = acc;
  }
  __syncthreads();
  long long off = wsum[wv] + x - s;
  for (int c = a; c < b; ++c) {
    ws.choff[c] = (int)off;
    off += ws.tot[c];
  }
  const long long M = total_items;
  // zero the level histograms of the pseudo-batch's item chunks
  const long long nch = (M + CH - 1) / CH;
  for (long long k = tid; k < nch * NQ; k += blockDim.x) ws.cnt[k] = 0;
  if (tid == 0) {
    Batch pb;
    pb.mode = 1;
    pb.L = -1;
    pb.bstart = 0;
    pb.n = (int)M;
    pb.epoch = epoch0;
    pb.ncommit = (int)M;
    pb.nchunk = (int)nch;
    ctl->bat[1] = pb;
    ctl->cut[1] = NONE;
    Batch z = pb;
    z.mode = 0;
    z.n = 0;
    ctl->bat[0] = z;
    if (M == 0) ctl->done = 1;
  }
}

// Ordered compaction of the phase-1 pixels (raster order) into ilist/desc + level histograms.
__global__ __launch_bounds__(BS) void k_compact(Ws ws) {
  __shared__ int wt[BS / 64];
  __shared__ int run;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  if (ws.ctl->bat[1].n == 0) return;
  if (tid == 0) run = 0;
  const long long c0 = (long long)blockIdx.x * CH;
  const int base = ws.choff[blockIdx.x];
  for (int s = 0; s < SUB; ++s) {
    const long long p = c0 + s * BS + tid;
    const bool f = (p < ws.N) && ws.mk[p] == INQ;
    if (!__syncthreads_or(f)) continue;
    const unsigned long long bal = __ballot(f);
    if (lane == 0) wt[wv] = __popcll(bal);
    __syncthreads();
    if (f) {
      int off = run + lanes_below(bal);
      for (int k = 0; k < wv; ++k) off += wt[k];
      const long long k = (long long)base + off;
      const int lv = ws.lv1[p];
      ws.ilist[k] = (int32_t)p;
      ws.desc[k] = (1ull << 32) | (unsigned long long)lv;
      atomicAdd(&ws.cnt[(k / CH) * NQ + lv], 1);
    }
    __syncthreads();
    if (tid == 0) run += wt[0] + wt[1] + wt[2] + wt[3];
  }
}

// ---------------------------------------------------------------------------------------------
// Resolve one batch: labels (fold of settled + earlier-batch neighbours) and push decisions.
// Deadlock-free bounded spinning: an item only waits on strictly lower ranks, all blocks of the
// grid are co-resident (grid <= RES_GRID_MAX), each block walks its chunks in increasing order,
// and each wave resolves its lanes cooperatively (intra-wave dependencies via shuffles).
__global__ __launch_bounds__(BS) void k_resolve(Ws ws, int par) {
  Ctl* ctl = ws.ctl;
  const Batch B = ctl->bat[par];
  if (B.n == 0 || ctl->error) return;
  __shared__ int hist[NQ];
  const int tid = threadIdx.x, lane = lane_id();
  const int W = ws.W;
  const int nch = (B.n + CH - 1) / CH;
  const unsigned long long etag = (unsigned long long)B.epoch << 32;
  for (int ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    hist[tid] = 0;
    __syncthreads();
    for (int s = 0; s < SUB; ++s) {
      const int wbase = ch * CH + s * BS + (tid & ~63);
      if (wbase >= B.n) break;  // wave-uniform
      const int i = wbase + lane;
      const bool valid = i < B.n;
      // ---- gather phase: everything that does not change during this launch ----
      long long p = 0;
      int base_lab = 0;
      int ldep[4] = {-1, -1, -1, -1};
      int pdep[4][3];
      unsigned zero_mask = 0;
      unsigned wts = 0;  // 4 packed push levels
      for (int d = 0; d < 4; ++d) pdep[d][0] = pdep[d][1] = pdep[d][2] = -1;
      if (valid) {
        p = ws.qbuf[B.bstart + i];
        const long long nb[4] = {p - 1, p + 1, p - W, p + W};
        wts = (unsigned)ws.wr[p - 1] | ((unsigned)ws.wr[p] << 8) | ((unsigned)ws.wd[p - W] << 16) |
              ((unsigned)ws.wd[p] << 24);
        for (int d = 0; d < 4; ++d) {
          const int v = ws.mk[nb[d]];
          if (v > 0) {
            base_lab = (base_lab == 0) ? v : (base_lab == v ? v : WSHED);
          } else if (v == INQ) {
            const int r = ws.qpos[nb[d]] - B.bstart;
            if (r >= 0 && r < i) ldep[d] = r;
          } else if (v == 0) {
            zero_mask |= 1u << d;
            // neighbours of the 0-pixel other than p: earlier batch items would push it first
            const long long n = nb[d];
            const long long nn[4] = {n - 1, n + 1, n - W, n + W};
            int k = 0;
            for (int e = 0; e < 4; ++e) {
              if (nn[e] == p) continue;
              const int vm = ws.mk[nn[e]];
              if (vm == INQ) {
                const int r = ws.qpos[nn[e]] - B.bstart;
                if (r >= 0 && r < i) pdep[d][k] = r;
              }
              ++k;
            }
          }
        }
      }
      // ---- cooperative resolution loop ----
      bool pending = valid;
      int mylab = 0;  // resolved label (0 = not yet)
      unsigned mask = 0;
      long long t0 = 0;
      int spins = 0;
      for (;;) {
        // snapshot of in-wave resolved labels for every dependency slot (uniform shuffles)
        int lv_in[4], pv_in[4][3];
        for (int d = 0; d < 4; ++d) {
          const int r = ldep[d];
          const bool inw = r >= wbase && r < wbase + 64;
          lv_in[d] = __shfl(mylab, inw ? r - wbase : lane);
          for (int k = 0; k < 3; ++k) {
            const int rr = pdep[d][k];
            const bool inw2 = rr >= wbase && rr < wbase + 64;
            pv_in[d][k] = __shfl(mylab, inw2 ? rr - wbase : lane);
          }
        }
        if (pending) {
          bool ok = true;
          int lab = base_lab;
          for (int d = 0; d < 4 && ok; ++d) {
            const int r = ldep[d];
            if (r < 0) continue;
            int v;
            if (r >= wbase && r < wbase + 64) {
              v = lv_in[d];
            } else {
              const unsigned long long g = ld_granule(&ws.tl[r]);
              v = ((g & 0xffffffff00000000ull) == etag) ? (int)(uint32_t)g : 0;
            }
            if (v == 0) { ok = false; break; }
            if (v > 0) lab = (lab == 0) ? v : (lab == v ? v : WSHED);
          }
          unsigned m = 0;
          if (ok && lab != WSHED) {
            for (int d = 0; d < 4 && ok; ++d) {
              if (!((zero_mask >> d) & 1u)) continue;
              bool win = true, undecided = false;
              for (int k = 0; k < 3; ++k) {
                const int rr = pdep[d][k];
                if (rr < 0) continue;
                int v;
                if (rr >= wbase && rr < wbase + 64) {
                  v = pv_in[d][k];
                } else {
                  const unsigned long long g = ld_granule(&ws.tl[rr]);
                  v = ((g & 0xffffffff00000000ull) == etag) ? (int)(uint32_t)g : 0;
                }
                if (v > 0) { win = false; break; }
                if (v == 0) undecided = true;
              }
              if (win && undecided) ok = false;
              else if (win) m |= 1u << d;
            }
          }
          if (ok) {
            if (lab == 0) {  // impossible for an exact queue: flag, label as WSHED
              atomicOr(&ctl->error, ERR_STATE);
              lab = WSHED;
            }
            mylab = lab;
            mask = (lab == WSHED) ? 0u : m;
            st_granule(&ws.tl[i], etag | (uint32_t)lab);
            ws.desc[i] = ((unsigned long long)mask << 32) | wts;
            pending = false;
          }
        }
        if (!__any(pending)) break;
        if (++spins > 32) {
          __builtin_amdgcn_s_sleep(1);
          if (__hip_atomic_load(&ctl->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
          const long long now = (long long)__builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = now;
          else if (now - t0 > SPIN_LIMIT_TICKS) {
            if (pending) atomicOr(&ctl->error, ERR_TIMEOUT);
            break;
          }
        }
      }
      // histogram + interrupt cut
      if (valid && mask) {
        bool lower = false;
        for (int d = 0; d < 4; ++d) {
          if ((mask >> d) & 1u) {
            const int lv = (wts >> (8 * d)) & 255;
            atomicAdd(&hist[lv], 1);
            if (lv < B.L) lower = true;
          }
        }
        if (lower) atomicMin(&ctl->cut[par], i);
      }
    }
    __syncthreads();
    ws.cnt[(long long)ch * NQ + tid] = hist[tid];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Scan (1 block x 1024): committed prefix, recount of the cut chunk, column scan -> per-chunk
// bucket offsets, head/tail update, choice of the next batch.
__global__ __launch_bounds__(1024) void k_scan(Ws ws, int par) {
  Ctl* ctl = ws.ctl;
  const Batch B = ctl->bat[par];
  if (B.n == 0) return;
  __shared__ int partial[NQ];
  const int tid = threadIdx.x;
  if (ctl->error) {  // stop the flood: nothing may be scattered from unresolved descriptors
    __syncthreads();
    if (tid == 0) {
      ctl->bat[par].nchunk = 0;
      ctl->bat[par].ncommit = 0;
      ctl->bat[par ^ 1].n = 0;
      ctl->done = 1;
    }
    return;
  }
  const int cut = ctl->cut[par];
  const int ncommit = (B.mode == 1 || cut == NONE) ? B.n : cut + 1;
  const int nch = (ncommit + CH - 1) / CH;
  const bool haspartial = (ncommit % CH) != 0 && ncommit != B.n;
  if (haspartial) {
    if (tid < NQ) partial[tid] = 0;
    __syncthreads();
    for (int i = (nch - 1) * CH + tid; i < ncommit; i += blockDim.x) {
      const unsigned long long d = ws.desc[i];
      const unsigned m = (unsigned)(d >> 32) & 15u;
      for (int k = 0; k < 4; ++k)
        if ((m >> k) & 1u) atomicAdd(&partial[(d >> (8 * k)) & 255], 1);
    }
    __syncthreads();
  }
  const int oldt = (tid < NQ) ? ctl->qtail[tid] : 0;
  column_scan(ws.cnt, ws.coff, nch, haspartial ? partial : nullptr, ctl->qtail);
  const int npush = column_total((tid < NQ) ? ctl->qtail[tid] - oldt : 0);
  if (tid == 0) {
    ctl->pushes += npush;
    if (B.mode == 0) {
      ctl->qhead[B.L] += ncommit;
      ctl->pops += ncommit;
      ctl->items += B.n;
    }
    ctl->bat[par].ncommit = ncommit;
    ctl->bat[par].nchunk = nch;
    if (ctl->qbase[NQ] < 0) ctl->error |= ERR_CAPACITY;
  }
  __syncthreads();
  choose_next(ctl, par ^ 1, B.epoch + 1);
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
    const int lsel = __shfl(myl, leader);
    unsigned sel = 0;
    for (int d = 0; d < 4; ++d)
      if (((rem >> d) & 1u) && (int)((lvls >> (8 * d)) & 255u) == lsel) sel |= 1u << d;
    const int cnt = __popc(sel);
    int x = cnt;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    const int total = __shfl(x, 63);
    int k = x - cnt;
    for (int d = 0; d < 4; ++d)
      if ((sel >> d) & 1u) pos[d] = k++;
    if (lane == 0) wrow[lsel] = total;
    rem &= ~sel;
  }
}

// Ordered scatter: commit labels of the committed prefix and append its pushes to the buckets in
// exact (rank, dir) order.  mode 1 (phase-1 pseudo-batch): item i is pixel ilist[i] itself.
__global__ __launch_bounds__(BS) void k_scatter(Ws ws, int par) {
  Ctl* ctl = ws.ctl;
  const Batch B = ctl->bat[par];
  if (B.n == 0 || ctl->error) return;
  __shared__ int run[NQ];
  __shared__ int wcnt[BS / 64][NQ];
  __shared__ int qb[NQ];
  const int tid = threadIdx.x, wv = tid >> 6;
  const int W = ws.W;
  qb[tid] = ctl->qbase[tid];
  for (int ch = blockIdx.x; ch < B.nchunk; ch += gridDim.x) {
    run[tid] = ws.coff[(long long)ch * NQ + tid];
    for (int k = 0; k < BS / 64; ++k) wcnt[k][tid] = 0;
    __syncthreads();
    for (int s = 0; s < SUB; ++s) {
      const int i0 = ch * CH + s * BS;
      if (i0 >= B.ncommit) break;  // block-uniform
      const int i = i0 + tid;
      const bool valid = i < B.ncommit;
      unsigned mask = 0, lvls = 0;
      long long p = 0;
      if (valid) {
        const unsigned long long d = ws.desc[i];
        mask = (unsigned)(d >> 32) & 15u;
        lvls = (unsigned)d;
        if (B.mode == 0) {
          p = ws.qbuf[B.bstart + i];
          ws.mk[p] = (int32_t)(uint32_t)ws.tl[i];
        } else {
          p = ws.ilist[i];
        }
      }
      int pos[4] = {0, 0, 0, 0};
      wave_rank(mask, lvls, pos, wcnt[wv]);
      __syncthreads();
      for (int d = 0; d < 4; ++d) {
        if (!((mask >> d) & 1u)) continue;
        const int lv = (lvls >> (8 * d)) & 255;
        int off = run[lv] + pos[d];
        for (int k = 0; k < wv; ++k) off += wcnt[k][lv];
        const int dest = qb[lv] + off;
        if (dest < 0 || (long long)dest >= ws.qcap) {
          atomicOr(&ctl->error, ERR_CAPACITY);
          continue;
        }
        long long n;
        if (B.mode == 0) {
          n = (d == 0) ? p - 1 : (d == 1) ? p + 1 : (d == 2) ? p - W : p + W;
          ws.mk[n] = INQ;
        } else {
          n = p;
        }
        ws.qbuf[dest] = (int32_t)n;
        ws.qpos[n] = dest;
      }
      __syncthreads();
      int t = 0;
      for (int k = 0; k < BS / 64; ++k) {
        t += wcnt[k][tid];
        wcnt[k][tid] = 0;
      }
      run[tid] += t;
      __syncthreads();
    }
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

}  // namespace msg
