// Experiment: the streaming kernels of the watershed path against the product versions.
//   colour distance (5 B/px): msg::k_edge_weights16<2> vs lane-coalesced 12-B quads (ewq<R, NT>)
//   untile + colorByIndexes(colored=false) (11 B/px): msg::k_untile vs one tile row per lane (unt<NT>)
// Standalone: hipcc -O3 --offload-arch=gfx950 -I opencv-msegment_amd/csrc; run under
// rocprofv3 --kernel-trace --stats for per-kernel durations.  Outputs are compared with the
// product kernels' outputs byte for byte.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ws_kernels.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct alignas(4) u3 { uint32_t x, y, z; };
typedef int i4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ch(uint32_t w, int b) { return (w >> (8 * b)) & 255u; }
__device__ __forceinline__ uint32_t ad(uint32_t a, uint32_t b) { return a > b ? a - b : b - a; }
#ifdef USE_SAD
// |x - y| for x, y < 2^16 in one v_sad_u16 (the high halves are 0)
__device__ __forceinline__ uint32_t sad(uint32_t x, uint32_t y) { return __builtin_amdgcn_sad_u16(x, y, 0u); }
#else
__device__ __forceinline__ uint32_t sad(uint32_t x, uint32_t y) { return ad(x, y); }
#endif
__device__ __forceinline__ uint32_t linf(const uint32_t* p, const uint32_t* q) {
  return max(max(sad(p[0], q[0]), sad(p[1], q[1])), sad(p[2], q[2]));
}

// the product's strip layout (16 px x R rows per thread, 48-B loads) with every channel
// extracted once and the distances from v_sad_u16
template <int R>
__global__ __launch_bounds__(256) void kews(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                            uint8_t* __restrict__ wd, int H, int W) {
  const int segs = W >> 4;
  unsigned b = blockIdx.x;
  const unsigned per_xcd = gridDim.x / 8;
  if (b < per_xcd * 8) b = (b % 8) * per_xcd + b / 8;
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
#pragma unroll
    for (int k = 0; k < 13; ++k) rows[i][k] = 0;
    if (r < H) {
      msg::ld48(img + 3 * p0, rows[i]);
      rows[i][12] = (has_r && i < R) ? *reinterpret_cast<const uint32_t*>(img + 3 * (p0 + 16)) : 0u;
    }
  }
  uint32_t cur[17][3], nxt[17][3];
#pragma unroll
  for (int k = 0; k < 17; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) cur[k][c] = (rows[0][(3 * k + c) >> 2] >> (8 * ((3 * k + c) & 3))) & 255u;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    if (r >= H) break;
    const bool has_d = r + 1 < H;
#pragma unroll
    for (int k = 0; k < 17; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) nxt[k][c] = (rows[i + 1][(3 * k + c) >> 2] >> (8 * ((3 * k + c) & 3))) & 255u;
    uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t vr = (k < 15 || has_r) ? linf(cur[k], cur[k + 1]) : 0u;
      const uint32_t vd = has_d ? linf(cur[k], nxt[k]) : 0u;
      orr[k >> 2] |= vr << (8 * (k & 3));
      odd[k >> 2] |= vd << (8 * (k & 3));
    }
    const long long p0 = (long long)r * W + 16ll * sx;
    *reinterpret_cast<uint4*>(wr + p0) = make_uint4(orr[0], orr[1], orr[2], orr[3]);
    *reinterpret_cast<uint4*>(wd + p0) = make_uint4(odd[0], odd[1], odd[2], odd[3]);
#pragma unroll
    for (int k = 0; k < 17; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) cur[k][c] = nxt[k][c];
  }
}
// the 4 pixels of a 12-byte quad (+ the next quad's first dword) as 5 x 3 channels
__device__ __forceinline__ void unpack(const u3 a, uint32_t nb, uint32_t px[5][3]) {
  px[0][0] = ch(a.x, 0); px[0][1] = ch(a.x, 1); px[0][2] = ch(a.x, 2);
  px[1][0] = ch(a.x, 3); px[1][1] = ch(a.y, 0); px[1][2] = ch(a.y, 1);
  px[2][0] = ch(a.y, 2); px[2][1] = ch(a.y, 3); px[2][2] = ch(a.z, 0);
  px[3][0] = ch(a.z, 1); px[3][1] = ch(a.z, 2); px[3][2] = ch(a.z, 3);
  px[4][0] = ch(nb, 0); px[4][1] = ch(nb, 1); px[4][2] = ch(nb, 2);
}

template <int R, bool NT>
__global__ __launch_bounds__(256) void ewq(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                           uint8_t* __restrict__ wd, int H, int W) {
  const int qpr = W >> 2;  // W % 4 == 0
  unsigned b = blockIdx.x;
  const unsigned per_xcd = gridDim.x / 8;
  if (b < per_xcd * 8) b = (b % 8) * per_xcd + b / 8;
  const long long t = (long long)b * blockDim.x + threadIdx.x;
  const int strips = (H + R - 1) / R;
  const bool valid = t < (long long)strips * qpr;
  const int st = valid ? (int)(t / qpr) : 0, qx = valid ? (int)(t - (long long)st * qpr) : 0;
  const int r0 = st * R;
  const bool has_r = qx + 1 < qpr;
  const int lane = threadIdx.x & 63;
  u3 a[R + 1];
#pragma unroll
  for (int i = 0; i <= R; ++i) {
    const int r = r0 + i;
    if (valid && r < H) a[i] = *reinterpret_cast<const u3*>(img + 3ll * ((long long)r * W + 4 * qx));
    else a[i] = u3{0, 0, 0};
  }
  uint32_t cur[5][3], nxt[5][3];
  {
    uint32_t nb = __shfl_down(a[0].x, 1);
    if (lane == 63 && has_r && valid && r0 < H) nb = *reinterpret_cast<const uint32_t*>(img + 3ll * ((long long)r0 * W + 4 * qx + 4));
    unpack(a[0], nb, cur);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    const bool has_d = r + 1 < H;
    uint32_t nb = 0;
    if (i + 1 < R) {
      nb = __shfl_down(a[i + 1].x, 1);
      if (lane == 63 && has_r && valid && r + 1 < H)
        nb = *reinterpret_cast<const uint32_t*>(img + 3ll * ((long long)(r + 1) * W + 4 * qx + 4));
    }
    unpack(a[i + 1], nb, nxt);
    uint32_t orr = 0, odd = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t vr = (k < 3 || has_r) ? linf(cur[k], cur[k + 1]) : 0u;
      const uint32_t vd = has_d ? linf(cur[k], nxt[k]) : 0u;
      orr |= vr << (8 * k);
      odd |= vd << (8 * k);
    }
    if (valid && r < H) {
      const long long p0 = (long long)r * W + 4 * qx;
      if (NT) {
        __builtin_nontemporal_store(orr, reinterpret_cast<uint32_t*>(wr + p0));
        __builtin_nontemporal_store(odd, reinterpret_cast<uint32_t*>(wd + p0));
      } else {
        *reinterpret_cast<uint32_t*>(wr + p0) = orr;
        *reinterpret_cast<uint32_t*>(wd + p0) = odd;
      }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) cur[k][c] = nxt[k][c];
  }
}

// kews with 32-bit indexing and clamped (branch-free) row loads
template <int R>
__global__ __launch_bounds__(256) void kews2(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                             uint8_t* __restrict__ wd, int H, int W) {
  const unsigned segs = (unsigned)W >> 4;
  unsigned b = blockIdx.x;
  const unsigned per_xcd = gridDim.x / 8;
  if (b < per_xcd * 8) b = (b % 8) * per_xcd + b / 8;
  const unsigned t = b * blockDim.x + threadIdx.x;
  const unsigned strips = ((unsigned)H + R - 1) / R;
  if (t >= strips * segs) return;
  const unsigned st = t / segs, sx = t - st * segs;
  const int r0 = (int)st * R;
  const bool has_r = sx + 1 < segs;
  uint32_t rows[R + 1][13];
#pragma unroll
  for (int i = 0; i <= R; ++i) {
    const int r = min(r0 + i, H - 1);
    const unsigned p0 = (unsigned)r * (unsigned)W + 16u * sx;
    msg::ld48(img + 3u * p0, rows[i]);
    rows[i][12] = has_r ? *reinterpret_cast<const uint32_t*>(img + 3u * (p0 + 16u)) : 0u;
  }
  uint32_t cur[17][3], nxt[17][3];
#pragma unroll
  for (int k = 0; k < 17; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) cur[k][c] = (rows[0][(3 * k + c) >> 2] >> (8 * ((3 * k + c) & 3))) & 255u;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    const bool has_d = r + 1 < H;
#pragma unroll
    for (int k = 0; k < 17; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) nxt[k][c] = (rows[i + 1][(3 * k + c) >> 2] >> (8 * ((3 * k + c) & 3))) & 255u;
    uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t vr = (k < 15 || has_r) ? linf(cur[k], cur[k + 1]) : 0u;
      const uint32_t vd = has_d ? linf(cur[k], nxt[k]) : 0u;
      orr[k >> 2] |= vr << (8 * (k & 3));
      odd[k >> 2] |= vd << (8 * (k & 3));
    }
    if (r < H) {
      const unsigned p0 = (unsigned)r * (unsigned)W + 16u * sx;
      *reinterpret_cast<uint4*>(wr + p0) = make_uint4(orr[0], orr[1], orr[2], orr[3]);
      *reinterpret_cast<uint4*>(wd + p0) = make_uint4(odd[0], odd[1], odd[2], odd[3]);
    }
#pragma unroll
    for (int k = 0; k < 17; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) cur[k][c] = nxt[k][c];
  }
}

// product layout (R = 1) with nontemporal output stores
__global__ __launch_bounds__(512) void kews_nt(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                               uint8_t* __restrict__ wd, int H, int W) {
  const unsigned segs = (unsigned)W >> 4;
  unsigned b = blockIdx.x;
  const unsigned per_xcd = gridDim.x / 8;
  if (b < per_xcd * 8) b = (b % 8) * per_xcd + b / 8;
  const unsigned t = b * blockDim.x + threadIdx.x;
  if (t >= (unsigned)H * segs) return;
  const unsigned st = t / segs, sx = t - st * segs;
  const int r = (int)st;
  const bool has_r = sx + 1 < segs;
  uint32_t rows[2][13];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int k = 0; k < 13; ++k) rows[i][k] = 0;
    if (r + i < H) {
      const unsigned p0 = (unsigned)(r + i) * (unsigned)W + 16u * sx;
      msg::ld48(img + 3u * p0, rows[i]);
      if (has_r && i == 0) rows[i][12] = *reinterpret_cast<const uint32_t*>(img + 3u * (p0 + 16u));
    }
  }
  uint32_t cur[17][3], nxt[17][3];
  msg::unpack17(rows[0], cur);
  msg::unpack17(rows[1], nxt);
  const bool has_d = r + 1 < H;
  uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t vr = (k < 15 || has_r) ? msg::linf_ch(cur[k], cur[k + 1]) : 0u;
    const uint32_t vd = has_d ? msg::linf_ch(cur[k], nxt[k]) : 0u;
    orr[k >> 2] |= vr << (8 * (k & 3));
    odd[k >> 2] |= vd << (8 * (k & 3));
  }
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  const unsigned p0 = (unsigned)r * (unsigned)W + 16u * sx;
  u4v a = {orr[0], orr[1], orr[2], orr[3]}, c = {odd[0], odd[1], odd[2], odd[3]};
  __builtin_nontemporal_store(a, reinterpret_cast<u4v*>(wr + p0));
  __builtin_nontemporal_store(c, reinterpret_cast<u4v*>(wd + p0));
}

// the product kernel (R = 1) under other block sizes
__global__ __launch_bounds__(1024) void kews_bs(const uint8_t* __restrict__ img, uint8_t* __restrict__ wr,
                                                uint8_t* __restrict__ wd, int H, int W) {
  const unsigned segs = (unsigned)W >> 4;
  unsigned b = blockIdx.x;
  const unsigned per_xcd = gridDim.x / 8;
  if (b < per_xcd * 8) b = (b % 8) * per_xcd + b / 8;
  const unsigned t = b * blockDim.x + threadIdx.x;
  if (t >= (unsigned)H * segs) return;
  const unsigned st = t / segs, sx = t - st * segs;
  const int r = (int)st;
  const bool has_r = sx + 1 < segs;
  uint32_t rows[2][13];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int k = 0; k < 13; ++k) rows[i][k] = 0;
    if (r + i < H) {
      const unsigned p0 = (unsigned)(r + i) * (unsigned)W + 16u * sx;
      msg::ld48(img + 3u * p0, rows[i]);
      if (has_r && i == 0) rows[i][12] = *reinterpret_cast<const uint32_t*>(img + 3u * (p0 + 16u));
    }
  }
  uint32_t cur[17][3], nxt[17][3];
  msg::unpack17(rows[0], cur);
  msg::unpack17(rows[1], nxt);
  const bool has_d = r + 1 < H;
  uint32_t orr[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t vr = (k < 15 || has_r) ? msg::linf_ch(cur[k], cur[k + 1]) : 0u;
    const uint32_t vd = has_d ? msg::linf_ch(cur[k], nxt[k]) : 0u;
    orr[k >> 2] |= vr << (8 * (k & 3));
    odd[k >> 2] |= vd << (8 * (k & 3));
  }
  const unsigned p0 = (unsigned)r * (unsigned)W + 16u * sx;
  *reinterpret_cast<uint4*>(wr + p0) = make_uint4(orr[0], orr[1], orr[2], orr[3]);
  *reinterpret_cast<uint4*>(wd + p0) = make_uint4(odd[0], odd[1], odd[2], odd[3]);
}

// untile: lane = one tile row (16 B of states); labels as one 16-B store, colours as 12 B
template <bool NT>
__global__ __launch_bounds__(256) void unt(const int32_t* __restrict__ mk, int H, int W, int Wt,
                                           int32_t* __restrict__ lab, int depth, uint8_t* __restrict__ dst) {
  const long long nrows = (long long)((H + 3) >> 2) * Wt * 4;
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nrows;
       u += (long long)gridDim.x * blockDim.x) {
    const long long tt = u >> 2;
    const int k = (int)(u & 3);
    const int r = (int)(tt / Wt) * 4 + k, c = (int)(tt % Wt) * 4;
    if (r >= H) continue;
    const i4v s = NT ? __builtin_nontemporal_load(reinterpret_cast<const i4v*>(mk) + u)
                     : reinterpret_cast<const i4v*>(mk)[u];
    const long long q = (long long)r * W + c;
    const uint32_t w0 = (s.x > 0 && s.x <= depth) ? 0xffffffu : 0u;
    const uint32_t w1 = (s.y > 0 && s.y <= depth) ? 0xffffffu : 0u;
    const uint32_t w2 = (s.z > 0 && s.z <= depth) ? 0xffffffu : 0u;
    const uint32_t w3 = (s.w > 0 && s.w <= depth) ? 0xffffffu : 0u;
    // B0G0R0B1 G1R1B2G2 R2B3G3R3
    const u3 o{w0 | (w1 << 24), (w1 >> 8) | (w2 << 16), (w2 >> 16) | (w3 << 8)};
    if (NT) {
      __builtin_nontemporal_store(s, reinterpret_cast<i4v*>(lab + q));
      uint32_t* d = reinterpret_cast<uint32_t*>(dst + 3 * q);
      __builtin_nontemporal_store(o.x, d);
      __builtin_nontemporal_store(o.y, d + 1);
      __builtin_nontemporal_store(o.z, d + 2);
    } else {
      *reinterpret_cast<i4v*>(lab + q) = s;
      *reinterpret_cast<u3*>(dst + 3 * q) = o;
    }
  }
}

typedef void (*ewfn)(const uint8_t*, uint8_t*, uint8_t*, int, int);

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int S = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = 20;
  const size_t N = (size_t)S * S;
  uint8_t *img, *wr, *wd, *wr0, *wd0;
  CK(hipMalloc(&img, 3 * N)); CK(hipMalloc(&wr, N)); CK(hipMalloc(&wd, N));
  CK(hipMalloc(&wr0, N)); CK(hipMalloc(&wd0, N));
  std::vector<uint8_t> h(3 * N);
  uint64_t x = 0x9E3779B97F4A7C15ull ^ S;
  for (size_t i = 0; i < 3 * N; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint8_t)(x >> 24); }
  CK(hipMemcpy(img, h.data(), 3 * N, hipMemcpyHostToDevice));
  std::vector<uint8_t> A(N), B(N), C(N), D(N);
  // baseline: the product kernel
  {
    const long long th = (long long)((S + 1) / 2) * (S / 16);
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(msg::k_edge_weights16<2>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, 0, img, wr0, wd0, S, S);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(A.data(), wr0, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(B.data(), wd0, N, hipMemcpyDeviceToHost));
  }
  struct V { const char* name; ewfn f; int R; } vars[] = {{"ewq<2>", ewq<2, false>, 2}};
  struct VS { const char* name; ewfn f; int R; } svars[] = {
      {"prod<1>", msg::k_edge_weights16<1>, 1}, {"prod<2>", msg::k_edge_weights16<2>, 2}};
  for (auto& v : svars) {
    CK(hipMemset(wr, 0x55, N)); CK(hipMemset(wd, 0x55, N));
    const long long th = (long long)((S + v.R - 1) / v.R) * (S / 16);
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(v.f, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, 0, img, wr, wd, S, S);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(C.data(), wr, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(D.data(), wd, N, hipMemcpyDeviceToHost));
    printf("%-10s %s\n", v.name, (memcmp(A.data(), C.data(), N) == 0 && memcmp(B.data(), D.data(), N) == 0) ? "same" : "DIFFERENT");
  }
  for (int bs : {64, 128, 512, 1024}) {
    CK(hipMemset(wr, 0x55, N)); CK(hipMemset(wd, 0x55, N));
    const long long th = (long long)S * (S / 16);
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(kews_bs, dim3((unsigned)((th + bs - 1) / bs)), dim3(bs), 0, 0, img, wr, wd, S, S);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(C.data(), wr, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(D.data(), wd, N, hipMemcpyDeviceToHost));
    printf("kews_bs/%d %s\n", bs, (memcmp(A.data(), C.data(), N) == 0 && memcmp(B.data(), D.data(), N) == 0) ? "same" : "DIFFERENT");
  }
  for (auto& v : vars) {
    CK(hipMemset(wr, 0x55, N)); CK(hipMemset(wd, 0x55, N));
    const long long th = (long long)((S + v.R - 1) / v.R) * (S / 4);
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(v.f, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, 0, img, wr, wd, S, S);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(C.data(), wr, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(D.data(), wd, N, hipMemcpyDeviceToHost));
    printf("%-10s %s\n", v.name, (memcmp(A.data(), C.data(), N) == 0 && memcmp(B.data(), D.data(), N) == 0) ? "same" : "DIFFERENT");
  }
  for (int bs : {64, 128, 512, 1024}) {
    CK(hipMemset(wr, 0x55, N)); CK(hipMemset(wd, 0x55, N));
    const long long th = (long long)S * (S / 16);
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(kews_bs, dim3((unsigned)((th + bs - 1) / bs)), dim3(bs), 0, 0, img, wr, wd, S, S);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(C.data(), wr, N, hipMemcpyDeviceToHost)); CK(hipMemcpy(D.data(), wd, N, hipMemcpyDeviceToHost));
    printf("kews_bs/%d %s\n", bs, (memcmp(A.data(), C.data(), N) == 0 && memcmp(B.data(), D.data(), N) == 0) ? "same" : "DIFFERENT");
  }
  // untile
  const int Wt = (S + 3) / 4, Ht = (S + 3) / 4;
  const size_t NT_ = (size_t)Wt * Ht * 16;
  int32_t *mk, *lab, *lab0;
  uint8_t *dst, *dst0;
  CK(hipMalloc(&mk, 4 * NT_)); CK(hipMalloc(&lab, 4 * N)); CK(hipMalloc(&lab0, 4 * N));
  CK(hipMalloc(&dst, 3 * N)); CK(hipMalloc(&dst0, 3 * N));
  int* d_err;
  CK(hipMalloc(&d_err, 4)); CK(hipMemset(d_err, 0, 4));
  std::vector<int32_t> hm(NT_);
  const int depth = 4000;
  for (size_t i = 0; i < NT_; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; hm[i] = (int)(x % (depth + 20)) - 1; }
  CK(hipMemcpy(mk, hm.data(), 4 * NT_, hipMemcpyHostToDevice));
  {
    const long long nunits = (long long)Ht * Wt * 8;
    const int grid = (int)std::min<long long>((nunits + 255) / 256, 8192);
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(msg::k_untile, dim3(grid), dim3(256), 0, 0, mk, S, S, Wt, lab0, depth, (const uint8_t*)nullptr, dst0, (uint8_t*)nullptr, d_err);
    CK(hipDeviceSynchronize());
  }
  std::vector<uint8_t> L0(4 * N), L1(4 * N), D0(3 * N), D1(3 * N);
  CK(hipMemcpy(L0.data(), lab0, 4 * N, hipMemcpyDeviceToHost)); CK(hipMemcpy(D0.data(), dst0, 3 * N, hipMemcpyDeviceToHost));
  for (int g : {2048, 4096, 8192, 16384}) {
    for (int nt = 0; nt < 2; ++nt) {
      CK(hipMemset(lab, 0x55, 4 * N)); CK(hipMemset(dst, 0x55, 3 * N));
      for (int i = 0; i < reps; ++i) {
        if (nt) hipLaunchKernelGGL(unt<true>, dim3(g), dim3(256), 0, 0, mk, S, S, Wt, lab, depth, dst);
        else hipLaunchKernelGGL(unt<false>, dim3(g), dim3(256), 0, 0, mk, S, S, Wt, lab, depth, dst);
      }
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(L1.data(), lab, 4 * N, hipMemcpyDeviceToHost)); CK(hipMemcpy(D1.data(), dst, 3 * N, hipMemcpyDeviceToHost));
      printf("unt<%d> grid %5d %s\n", nt, g, (L0 == L1 && D0 == D1) ? "same" : "DIFFERENT");
    }
  }
  printf("done\n");
  return 0;
}
