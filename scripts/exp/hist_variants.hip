// Experiment: 256-bin histogram of BGR2GRAY on gfx950, four LDS strategies, timed with HIP events
// on a uniform, a random and a mosaic-like 4096^2 frame.  Standalone (hipcc -O3 --offload-arch=gfx950).
//   A: one LDS sub-histogram per wave, ds_add (the library's k_gray_hist inner loop)
//   B: 16 padded copies per wave (lane & 15), ds_add: same-address conflicts / 16, banks skewed
//   C: per-lane 8-bit counters, plain read-modify-write (no atomics, conflict-free by layout)
//   D: wave match-aggregation (ballot over equal bins, one ds_add per distinct bin)
//   E<BS,C>: C padded copies per wave + a wave-uniform fast path (one ds_add for 256 equal pixels)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t gray_of(uint32_t b, uint32_t g, uint32_t r) {
  return (1868u * b + 9617u * g + 4899u * r + 8192u) >> 14;
}

__device__ __forceinline__ void grays(const uint32_t* b32, long long q, uint32_t y[4]) {
  const uint32_t w0 = b32[3 * q], w1 = b32[3 * q + 1], w2 = b32[3 * q + 2];
  y[0] = gray_of(w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
  y[1] = gray_of(w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
  y[2] = gray_of((w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
  y[3] = gray_of((w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
}

template <int BS>
__global__ __launch_bounds__(BS) void kA(const uint8_t* bgr, long long nq, uint8_t* gray, unsigned* hist) {
  __shared__ unsigned sh[BS / 64][256];
  for (int k = threadIdx.x; k < BS / 64 * 256; k += BS) (&sh[0][0])[k] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6;
  const uint32_t* b32 = (const uint32_t*)bgr;
  for (long long q = blockIdx.x * (long long)BS + threadIdx.x; q < nq; q += (long long)gridDim.x * BS) {
    uint32_t y[4];
    grays(b32, q, y);
    ((uint32_t*)gray)[q] = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
    for (int j = 0; j < 4; ++j) atomicAdd(&sh[wv][y[j]], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int k = 0; k < BS / 64; ++k) s += sh[k][t];
    atomicAdd(hist + t, s);
  }
}

template <int BS>
__global__ __launch_bounds__(BS) void kB(const uint8_t* bgr, long long nq, uint8_t* gray, unsigned* hist) {
  constexpr int C = 16, ST = 257;
  extern __shared__ unsigned shB[];  // [BS/64][C][ST]
  for (int k = threadIdx.x; k < BS / 64 * C * ST; k += BS) shB[k] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned* mine = shB + (wv * C + (lane & (C - 1))) * ST;
  const uint32_t* b32 = (const uint32_t*)bgr;
  for (long long q = blockIdx.x * (long long)BS + threadIdx.x; q < nq; q += (long long)gridDim.x * BS) {
    uint32_t y[4];
    grays(b32, q, y);
    ((uint32_t*)gray)[q] = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
    for (int j = 0; j < 4; ++j) atomicAdd(mine + y[j], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int k = 0; k < BS / 64 * C; ++k) s += shB[k * ST + t];
    atomicAdd(hist + t, s);
  }
}

template <int BS>
__global__ __launch_bounds__(BS) void kC(const uint8_t* bgr, long long nq, uint8_t* gray, unsigned* hist) {
  extern __shared__ uint8_t shC[];  // [BS/64][256 bins][64 lanes] bytes
  for (int k = threadIdx.x; k < BS / 64 * 256 * 64 / 4; k += BS) ((uint32_t*)shC)[k] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* base = shC + wv * 256 * 64 + lane;
  const uint32_t* b32 = (const uint32_t*)bgr;
  int since = 0;
  for (long long q = blockIdx.x * (long long)BS + threadIdx.x; q < nq; q += (long long)gridDim.x * BS) {
    uint32_t y[4];
    grays(b32, q, y);
    ((uint32_t*)gray)[q] = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
    for (int j = 0; j < 4; ++j) base[y[j] * 64] = (uint8_t)(base[y[j] * 64] + 1);
    (void)since;  // (no overflow at this size: <= 64 px per lane)
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int w = 0; w < BS / 64; ++w) {
      const uint32_t* row = (const uint32_t*)(shC + w * 256 * 64 + t * 64);
      for (int k = 0; k < 16; ++k) {
        const uint32_t x = row[k];
        s += (x & 255u) + ((x >> 8) & 255u) + ((x >> 16) & 255u) + (x >> 24);
      }
    }
    atomicAdd(hist + t, s);
  }
}

template <int BS>
__global__ __launch_bounds__(BS) void kD(const uint8_t* bgr, long long nq, uint8_t* gray, unsigned* hist) {
  __shared__ unsigned sh[BS / 64][256];
  for (int k = threadIdx.x; k < BS / 64 * 256; k += BS) (&sh[0][0])[k] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t* b32 = (const uint32_t*)bgr;
  for (long long q = blockIdx.x * (long long)BS + threadIdx.x; q < nq; q += (long long)gridDim.x * BS) {
    uint32_t y[4];
    grays(b32, q, y);
    ((uint32_t*)gray)[q] = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
    for (int j = 0; j < 4; ++j) {
      bool todo = true;
      while (__ballot(todo)) {
        const unsigned long long act = __ballot(todo);
        const int leader = __ffsll((long long)act) - 1;
        const uint32_t v = __shfl(y[j], leader);
        const unsigned long long m = __ballot(todo && y[j] == v);
        if (lane == leader) atomicAdd(&sh[wv][v], (unsigned)__popcll(m));
        if (y[j] == v) todo = false;
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int k = 0; k < BS / 64; ++k) s += sh[k][t];
    atomicAdd(hist + t, s);
  }
}

template <int BS, int C>
__global__ __launch_bounds__(BS) void kE(const uint8_t* bgr, long long nq, uint8_t* gray, unsigned* hist) {
  constexpr int ST = 257;
  __shared__ unsigned shE[BS / 64 * C * ST];
  for (int k = threadIdx.x; k < BS / 64 * C * ST; k += BS) shE[k] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned* mine = shE + (wv * C + (lane & (C - 1))) * ST;
  const uint32_t* b32 = (const uint32_t*)bgr;
  for (long long q = blockIdx.x * (long long)BS + threadIdx.x; q < nq; q += (long long)gridDim.x * BS) {
    uint32_t y[4];
    grays(b32, q, y);
    ((uint32_t*)gray)[q] = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
    const uint32_t y0 = __builtin_amdgcn_readfirstlane(y[0]);
    const unsigned nact = (unsigned)__popcll(__ballot(1));
    if (__all(y[0] == y0 && y[1] == y0 && y[2] == y0 && y[3] == y0)) {
      if (lane == 0) atomicAdd(mine + y0, 4u * nact);
    } else {
      for (int j = 0; j < 4; ++j) atomicAdd(mine + y[j], 1u);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int k = 0; k < BS / 64 * C; ++k) s += shE[k * ST + t];
    atomicAdd(hist + t, s);
  }
}

// H<BS,C,U,LAST>: E with U groups per thread in flight; LAST: partial rows + last-block reduce
template <int BS, int C, int U, bool LAST>
__global__ __launch_bounds__(BS) void kH(const uint8_t* bgr, long long nq, uint8_t* gray, unsigned* hist,
                                         unsigned* part, unsigned* ticket) {
  constexpr int ST = 257;
  __shared__ unsigned shE[BS / 64 * C * ST];
  __shared__ int last;
  for (int k = threadIdx.x; k < BS / 64 * C * ST; k += BS) shE[k] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned* mine = shE + (wv * C + (lane & (C - 1))) * ST;
  const uint32_t* b32 = (const uint32_t*)bgr;
  const long long stride = (long long)gridDim.x * BS * U;
  for (long long q0 = blockIdx.x * (long long)BS * U + threadIdx.x; q0 < nq; q0 += stride) {
    uint32_t w[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long q = q0 + (long long)u * BS;
      if (q < nq) { w[u][0] = b32[3 * q]; w[u][1] = b32[3 * q + 1]; w[u][2] = b32[3 * q + 2]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long q = q0 + (long long)u * BS;
      if (q >= nq) break;
      const uint32_t w0 = w[u][0], w1 = w[u][1], w2 = w[u][2];
      uint32_t y[4];
      y[0] = gray_of(w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
      y[1] = gray_of(w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
      y[2] = gray_of((w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
      y[3] = gray_of((w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
      ((uint32_t*)gray)[q] = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
      const uint32_t y0 = __builtin_amdgcn_readfirstlane(y[0]);
      const unsigned nact = (unsigned)__popcll(__ballot(1));
      if (__all(y[0] == y0 && y[1] == y0 && y[2] == y0 && y[3] == y0)) {
        if (lane == 0) atomicAdd(mine + y0, 4u * nact);
      } else {
        for (int j = 0; j < 4; ++j) atomicAdd(mine + y[j], 1u);
      }
    }
  }
  __syncthreads();
  if (!LAST) {
    for (int t = threadIdx.x; t < 256; t += BS) {
      unsigned s = 0;
      for (int k = 0; k < BS / 64 * C; ++k) s += shE[k * ST + t];
      atomicAdd(hist + t, s);
    }
    return;
  }
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int k = 0; k < BS / 64 * C; ++k) s += shE[k * ST + t];
    part[blockIdx.x * 256 + t] = s;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!last) return;
  for (int t = threadIdx.x; t < 256; t += BS) {
    unsigned s = 0;
    for (int r = 0; r < (int)gridDim.x; ++r) s += part[r * 256 + t];
    hist[t] = s;
  }
  if (threadIdx.x == 0) *ticket = 0;
}

int main() {
  const int H = 4096, W = 4096;
  const long long N = (long long)H * W, nq = N / 4;
  std::vector<uint8_t> img(N * 3);
  uint8_t *d_img, *d_gray;
  unsigned* d_hist;
  CK(hipMalloc(&d_img, N * 3));
  CK(hipMalloc(&d_gray, N));
  CK(hipMalloc(&d_hist, 1024));
  unsigned *d_part, *d_ticket;
  CK(hipMalloc(&d_part, 4096 * 1024));
  CK(hipMalloc(&d_ticket, 64));
  CK(hipMemset(d_ticket, 0, 64));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"uniform", "random", "mosaic"};
  for (int f = 0; f < 3; ++f) {
    unsigned long long x = 12345;
    for (long long i = 0; i < N; ++i) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      const int r = (int)(i / W), c = (int)(i % W);
      const unsigned cell = (unsigned)((r / 64) * 64 + c / 64) * 2654435761u;
      for (int k = 0; k < 3; ++k) {
        uint8_t v;
        if (f == 0) v = 77;
        else if (f == 1) v = (uint8_t)(x >> (24 + 8 * k));
        else v = (uint8_t)(((cell >> (8 * k)) & 255u) + ((x >> (40 + 4 * k)) & 3u));
        img[3 * i + k] = v;
      }
    }
    CK(hipMemcpy(d_img, img.data(), N * 3, hipMemcpyHostToDevice));
    std::vector<unsigned> ref;
    for (int v = 0; v < 11; ++v) {
      float best = 1e9f;
      for (int rep = 0; rep < 12; ++rep) {
        CK(hipMemset(d_hist, 0, 1024));
        CK(hipEventRecord(e0, 0));
        if (v == 0) hipLaunchKernelGGL(kA<512>, dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist);
        if (v == 1) hipLaunchKernelGGL(kB<256>, dim3(2 * cus), dim3(256), 4 * 16 * 257 * 4, 0, d_img, nq, d_gray, d_hist);
        if (v == 2) hipLaunchKernelGGL(kC<256>, dim3(2 * cus), dim3(256), 4 * 256 * 64, 0, d_img, nq, d_gray, d_hist);
        if (v == 3) hipLaunchKernelGGL(kD<512>, dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist);
        if (v == 4) hipLaunchKernelGGL((kE<512, 1>), dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist);
        if (v == 5) hipLaunchKernelGGL((kE<512, 4>), dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist);
        if (v == 6) hipLaunchKernelGGL((kE<256, 4>), dim3(4 * cus), dim3(256), 0, 0, d_img, nq, d_gray, d_hist);
        if (v == 7) hipLaunchKernelGGL((kH<512, 4, 4, false>), dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist, d_part, d_ticket);
        if (v == 8) hipLaunchKernelGGL((kH<512, 4, 4, true>), dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist, d_part, d_ticket);
        if (v == 9) hipLaunchKernelGGL((kH<512, 4, 2, false>), dim3(2 * cus), dim3(512), 0, 0, d_img, nq, d_gray, d_hist, d_part, d_ticket);
        if (v == 10) hipLaunchKernelGGL((kH<1024, 2, 4, false>), dim3(cus), dim3(1024), 0, 0, d_img, nq, d_gray, d_hist, d_part, d_ticket);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 1 && ms < best) best = ms;
      }
      std::vector<unsigned> h(256);
      CK(hipMemcpy(h.data(), d_hist, 1024, hipMemcpyDeviceToHost));
      if (v == 0) ref = h;
      const bool ok = h == ref;
      printf("%-8s variant %c  %7.1f us  %6.0f GB/s  %s\n", names[f], 'A' + v, best * 1e3,
             4.0 * N / (best * 1e-3) / 1e9, ok ? "ok" : "MISMATCH");
    }
  }
  return 0;
}
