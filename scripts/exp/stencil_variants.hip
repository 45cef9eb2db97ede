// Experiment: the colour-distance stencil (k_edge_weights16) with R rows per thread and with or
// without an XCD-aware block order (logical strip = (b % 8) * per + b / 8, so the blocks one XCD
// runs together own consecutive strips and the extra row each strip reads is the next strip's
// first row, which that XCD's L2 already holds).  Standalone: hipcc -O3 --offload-arch=gfx950.
// Prints us per launch (event pair per launch, and one pair over `reps` launches) and GB/s at
// 5 algorithmic B/px; every variant's output is compared with variant R=4/no-remap.
// Measured (MI355X, event pair per launch / back-to-back, us): 4096^2 R4 22.6/19.9, R4x 22.2/18.8,
// R2x 20.6/17.4, R8x 25.0/21.9, L2x 23.9/20.1; 8192^2 R4x 68.4/64.1, R2x 67.8/67.8, L2x 73.6/74.8;
// 16384^2 R4x 238/236, R2x 262/241, L2x 290/253.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t byte_of(const uint32_t* w, int i) { return (w[i >> 2] >> (8 * (i & 3))) & 255u; }
__device__ __forceinline__ uint32_t linf3(const uint32_t* wa, int ia, const uint32_t* wb, int ib) {
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int x = (int)byte_of(wa, ia + k), y = (int)byte_of(wb, ib + k);
    m = max(m, (uint32_t)abs(x - y));
  }
  return m;
}
__device__ __forceinline__ void ld48(const uint8_t* p, uint32_t* w) {
  const uint4* a = reinterpret_cast<const uint4*>(p);
  const uint4 x0 = a[0], x1 = a[1], x2 = a[2];
  w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w;
  w[4] = x1.x; w[5] = x1.y; w[6] = x1.z; w[7] = x1.w;
  w[8] = x2.x; w[9] = x2.y; w[10] = x2.z; w[11] = x2.w;
}

template <int R, bool REMAP>
__global__ __launch_bounds__(256) void kew(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                           uint8_t* __restrict__ wd, int H, int W) {
  const int segs = W >> 4;
  unsigned b = blockIdx.x;
  if (REMAP) {
    const unsigned nb = gridDim.x, per = nb / 8;
    if (b < per * 8) b = (b % 8) * per + b / 8;
  }
  const long long t = (long long)b * blockDim.x + threadIdx.x;
  const int strips = (H + R - 1) / R;
  if (t >= (long long)strips * segs) return;
  const int st = (int)(t / segs), sx = (int)(t - (long long)st * segs);
  const int r0 = st * R;
  const bool has_r = sx + 1 < segs;
  uint32_t rows[R + 1][13];
#pragma unroll
  for (int i = 0; i <= R; ++i) {
    const int r = r0 + i;
    const long long p0 = (long long)r * W + 16ll * sx;
    if (r < H) {
      ld48(img + 3 * p0, rows[i]);
      rows[i][12] = (has_r && i < R) ? *reinterpret_cast<const uint32_t*>(img + 3 * (p0 + 16)) : 0u;
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    if (r >= H) break;
    const bool has_d = r + 1 < H;
    uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t vr = (k < 15 || has_r) ? linf3(rows[i], 3 * k, rows[i], 3 * k + 3) : 0u;
      const uint32_t vd = has_d ? linf3(rows[i], 3 * k, rows[i + 1], 3 * k) : 0u;
      orr[k >> 2] |= vr << (8 * (k & 3));
      odd[k >> 2] |= vd << (8 * (k & 3));
    }
    const long long p0 = (long long)r * W + 16ll * sx;
    *reinterpret_cast<uint4*>(wr + p0) = make_uint4(orr[0], orr[1], orr[2], orr[3]);
    *reinterpret_cast<uint4*>(wd + p0) = make_uint4(odd[0], odd[1], odd[2], odd[3]);
  }
}


// L<R>: coalesced loads staged through LDS.  A block = 256 threads = one 4096-column chunk of an
// R-row strip (W % 4096 == 0 here): each of the R + 1 rows is loaded as 3 contiguous 4 KB wave-
// block instructions (lane i: bytes 16 i of each 4 KB), written to LDS, then every lane reads
// its own 48 B (+ the next lane's first dword) per row back with a 12-dword stride (conflict-free
// over 64 banks) and runs the same per-lane stencil.
template <int R, bool REMAP>
__global__ __launch_bounds__(256) void kewl(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                            uint8_t* __restrict__ wd, int H, int W) {
  __shared__ uint4 sh[R + 1][769];  // 12 KB of row + one pad uint4 (the right chunk's first bytes)
  unsigned b = blockIdx.x;
  if (REMAP) {
    const unsigned nb = gridDim.x, per = nb / 8;
    if (b < per * 8) b = (b % 8) * per + b / 8;
  }
  const int chunks = W >> 12;
  const int st = (int)(b / chunks), ch = (int)(b - (unsigned)st * chunks);
  const int r0 = st * R;
  if (r0 >= H) return;
  const int tid = threadIdx.x;
  const bool last_chunk = ch + 1 == chunks;
  // the right chunk's first dword, loaded by lane 255 only (a uniform guard let the compiler
  // hoist it into an unconditional scalar load past the frame's last row: a fault)
#pragma unroll
  for (int i = 0; i <= R; ++i) {
    const int r = r0 + i;
    if (r < H) {
      const uint4* rowp = reinterpret_cast<const uint4*>(img + 3 * ((long long)r * W + 4096ll * ch));
#pragma unroll
      for (int k = 0; k < 3; ++k) sh[i][256 * k + tid] = rowp[256 * k + tid];
      if (tid == 255) {
        uint32_t pw = 0;
        if (!last_chunk) pw = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(rowp + 768));
        reinterpret_cast<uint32_t*>(&sh[i][768])[0] = pw;
      }
    }
  }
  __syncthreads();
  const bool has_r = !(last_chunk && tid == 255);
  uint32_t rows[R + 1][13];
#pragma unroll
  for (int i = 0; i <= R; ++i) {
    if (r0 + i < H) {
      const uint4 a0 = sh[i][3 * tid], a1 = sh[i][3 * tid + 1], a2 = sh[i][3 * tid + 2];
      rows[i][0] = a0.x; rows[i][1] = a0.y; rows[i][2] = a0.z; rows[i][3] = a0.w;
      rows[i][4] = a1.x; rows[i][5] = a1.y; rows[i][6] = a1.z; rows[i][7] = a1.w;
      rows[i][8] = a2.x; rows[i][9] = a2.y; rows[i][10] = a2.z; rows[i][11] = a2.w;
      rows[i][12] = reinterpret_cast<const uint32_t*>(&sh[i][0])[12 * tid + 12];
    }
  }
  const int sx = ch * 256 + tid;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    if (r >= H) break;
    const bool has_d = r + 1 < H;
    uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t vr = (k < 15 || has_r) ? linf3(rows[i], 3 * k, rows[i], 3 * k + 3) : 0u;
      const uint32_t vd = has_d ? linf3(rows[i], 3 * k, rows[i + 1], 3 * k) : 0u;
      orr[k >> 2] |= vr << (8 * (k & 3));
      odd[k >> 2] |= vd << (8 * (k & 3));
    }
    const long long p0 = (long long)r * W + 16ll * sx;
    *reinterpret_cast<uint4*>(wr + p0) = make_uint4(orr[0], orr[1], orr[2], orr[3]);
    *reinterpret_cast<uint4*>(wd + p0) = make_uint4(odd[0], odd[1], odd[2], odd[3]);
  }
}

typedef void (*kfn)(const uint8_t*, uint8_t*, uint8_t*, int, int);
struct Var { const char* name; kfn f; int R; };

int main(int argc, char** argv) {
  std::vector<int> sizes;
  for (int i = 1; i < argc; ++i) sizes.push_back(atoi(argv[i]));
  if (sizes.empty()) sizes = {4096, 8192, 16384};
  Var vars[] = {
      {"R4", kew<4, false>, 4},   {"R4x", kew<4, true>, 4},   {"R8", kew<8, false>, 8},
      {"R8x", kew<8, true>, 8},   {"R2x", kew<2, true>, 2},   {"L1", kewl<1, false>, -1}, {"L2", kewl<2, false>, -2},
      {"L2x", kewl<2, true>, -2}, {"L4x", kewl<4, true>, -4}, {"L1x", kewl<1, true>, -1},
  };
  const int nv = sizeof(vars) / sizeof(vars[0]);
  for (int S : sizes) {
    const size_t N = (size_t)S * S;
    uint8_t *img, *wr, *wd, *wr0, *wd0;
    CK(hipMalloc(&img, 3 * N)); CK(hipMalloc(&wr, N)); CK(hipMalloc(&wd, N));
    CK(hipMalloc(&wr0, N)); CK(hipMalloc(&wd0, N));
    std::vector<uint8_t> h(3 * N);
    uint64_t x = 0x9E3779B97F4A7C15ull ^ S;
    for (size_t i = 0; i < 3 * N; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint8_t)(x >> 24); }
    CK(hipMemcpy(img, h.data(), 3 * N, hipMemcpyHostToDevice));
    std::vector<uint8_t> a(N), bb(N), c(N), d(N);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int v = 0; v < nv; ++v) {
      const int RR = vars[v].R < 0 ? -vars[v].R : vars[v].R;
      const int segs = S / 16, strips = (S + RR - 1) / RR;
      const long long th = (long long)strips * segs;
      dim3 g((unsigned)((th + 255) / 256)), blk(256);  // L: one block per 4096-column chunk of a strip
      uint8_t* o1 = v == 0 ? wr0 : wr;
      uint8_t* o2 = v == 0 ? wd0 : wd;
      CK(hipMemset(o1, 0x55, N)); CK(hipMemset(o2, 0x55, N));
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(vars[v].f, g, blk, 0, 0, img, o1, o2, S, S);
      CK(hipDeviceSynchronize());
      const int reps = 50;
      float per = 0;
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(vars[v].f, g, blk, 0, 0, img, o1, o2, S, S);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); per += ms;
      }
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(vars[v].f, g, blk, 0, 0, img, o1, o2, S, S);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      bool ok = true;
      if (v > 0) {
        CK(hipMemcpy(a.data(), wr0, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(bb.data(), wd0, N, hipMemcpyDeviceToHost));
        CK(hipMemcpy(c.data(), wr, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(d.data(), wd, N, hipMemcpyDeviceToHost));
        ok = memcmp(a.data(), c.data(), N) == 0 && memcmp(bb.data(), d.data(), N) == 0;
      }
      const double us1 = 1000.0 * per / reps, usb = 1000.0 * ms / reps;
      printf("%5d^2 %-5s per-launch %7.2f us %6.0f GB/s | back-to-back %7.2f us %6.0f GB/s | %s\n", S,
             vars[v].name, us1, 5.0 * N / us1 / 1e3, usb, 5.0 * N / usb / 1e3, ok ? "same" : "DIFFERENT");
      fflush(stdout);
    }
    CK(hipFree(img)); CK(hipFree(wr)); CK(hipFree(wd)); CK(hipFree(wr0)); CK(hipFree(wd0));
  }
  return 0;
}
