// Calibration of the TCC FETCH_SIZE counter on gfx950 for the access shapes of the flood kernels:
// run under `rocprofv3 --pmc FETCH_SIZE` and compare each kernel's counter (KiB) with the bytes it
// must fetch.  k_seq: 256 MiB of coalesced 16-B loads.  k_rand4 / k_rand16: 2^22 threads, each
// one 4-B (or 16-B) load from its own 128-B line of a 2 GiB buffer (lines in a scattered order,
// no line touched twice), i.e. 2^22 distinct lines = 512 MiB at 128 B per line, 256 MiB at 64 B.
// Standalone: hipcc -O3 --offload-arch=gfx950 -o build/exp/fetch_calib scripts/exp/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_seq(const uint4* __restrict__ a, long long n, unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads
}

// line index of thread t: a bijection on [0, 2^28 / 32) lines (odd multiplier mod a power of two)
__device__ __forceinline__ unsigned long long line_of(unsigned t, unsigned nlines) {
  return ((unsigned long long)t * 2654435761ull) & (nlines - 1);
}

__global__ void k_rand4(const unsigned* __restrict__ a, unsigned nthreads, unsigned nlines, unsigned* __restrict__ out) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const unsigned v = a[line_of(t, nlines) * 32ull];
  if (v == 0x9e3779b9u) out[0] = v;
}

__global__ void k_rand16(const uint4* __restrict__ a, unsigned nthreads, unsigned nlines, unsigned* __restrict__ out) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const uint4 v = a[line_of(t, nlines) * 8ull];
  if ((v.x ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

int main() {
  const size_t bytes = 2ull << 30;  // 2 GiB
  unsigned* buf;
  unsigned* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, bytes));
  const unsigned nlines = (unsigned)(bytes / 128);  // 2^24 lines
  const unsigned nthreads = 1u << 22;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_seq, dim3(8192), dim3(256), 0, 0, (const uint4*)buf, (long long)((256ull << 20) / 16), out);
    hipLaunchKernelGGL(k_rand4, dim3(nthreads / 256), dim3(256), 0, 0, buf, nthreads, nlines, out);
    hipLaunchKernelGGL(k_rand16, dim3(nthreads / 256), dim3(256), 0, 0, (const uint4*)buf, nthreads, nlines, out);
    CK(hipDeviceSynchronize());
  }
  printf("expected per launch: k_seq 262144 KiB; k_rand4/k_rand16 %u lines = %u KiB at 128 B, %u KiB at 64 B\n",
         nthreads, nthreads / 8, nthreads / 16);
  return 0;
}
