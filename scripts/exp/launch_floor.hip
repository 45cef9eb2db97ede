// Launch floor of grid shapes like the flood's per-generation kernels (no work): back-to-back
// launches on one stream between two events.  hipcc --offload-arch=gfx950 -O3 launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int BS, int LDSW>
__global__ __launch_bounds__(BS) void k_empty(int* ctl, int iter) {
  __shared__ int lds[LDSW];
  if (threadIdx.x == 0) lds[0] = ctl[0];
  __syncthreads();
  if (threadIdx.x == 0 && lds[0] == 12345 + iter) ctl[1] = blockIdx.x;  // never true
}

template <int BS, int LDSW>
float run(int grid, int* ctl, hipStream_t st, int n) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) k_empty<BS, LDSW><<<grid, BS, 0, st>>>(ctl, i);
  hipEventRecord(a, st);
  for (int i = 0; i < n; ++i) k_empty<BS, LDSW><<<grid, BS, 0, st>>>(ctl, i);
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return 1000.f * ms / n;
}

int main() {
  int* ctl;
  hipMalloc(&ctl, 64);
  hipMemset(ctl, 0, 64);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  const int n = 2000;
  printf("grid 481 x 1024 thr, 27 KB LDS : %.2f us\n", run<1024, 6912>(481, ctl, st, n));
  printf("grid 481 x 1024 thr, 1 KB LDS  : %.2f us\n", run<1024, 256>(481, ctl, st, n));
  printf("grid 481 x 256 thr, 27 KB LDS  : %.2f us\n", run<256, 6912>(481, ctl, st, n));
  printf("grid 121 x 1024 thr, 27 KB LDS : %.2f us\n", run<1024, 6912>(121, ctl, st, n));
  printf("grid 512 x 512 thr, 13 KB LDS  : %.2f us\n", run<512, 3334>(512, ctl, st, n));
  printf("grid 256 x 256 thr, 1 KB LDS   : %.2f us\n", run<256, 256>(256, ctl, st, n));
  printf("grid 1 x 1024 thr, 1 KB LDS    : %.2f us\n", run<1024, 256>(1, ctl, st, n));
  printf("grid 1 x 64 thr                : %.2f us\n", run<64, 64>(1, ctl, st, n));
  return 0;
}
