// idle_launch.hip — what an idle conditional launch between two streaming
// kernels costs on the step's critical path.  Each iteration: a 256 MB copy
// (kernel A), then variant X, then another 256 MB copy (kernel B), all on one
// stream; the per-iteration time minus the no-X time is X's cost.  Variants:
//   none          A, B only
//   w1            one 64-thread workgroup that reads a flag word and exits
//   wg1024        one 1024-thread workgroup, 64 KiB static LDS (K4r's shape)
//   wg1024_noflag the same, exiting without the flag read
//   wg256_16k     one 256-thread workgroup, 16 KiB static LDS
//   hipcc --offload-arch=gfx950 -O3 tools/micro/idle_launch.hip -o tools/micro/idle_launch
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

__global__ __launch_bounds__(64) void k_w1(const unsigned* flag, unsigned epoch, unsigned* sink) {
  if (*flag == epoch) sink[threadIdx.x] = 1u;
}

__global__ __launch_bounds__(1024) void k_wg1024(const unsigned* flag, unsigned epoch, unsigned* sink) {
  __shared__ unsigned t[16384];
  if (*flag != epoch) return;
  t[threadIdx.x] = threadIdx.x;
  __syncthreads();
  sink[threadIdx.x] = t[1023 - threadIdx.x];
}

__global__ __launch_bounds__(1024) void k_wg1024_noflag(unsigned* sink, unsigned go) {
  __shared__ unsigned t[16384];
  if (go == 0u) return;
  t[threadIdx.x] = threadIdx.x;
  __syncthreads();
  sink[threadIdx.x] = t[1023 - threadIdx.x];
}

__global__ __launch_bounds__(256) void k_wg256(const unsigned* flag, unsigned epoch, unsigned* sink) {
  __shared__ unsigned t[4096];
  if (*flag != epoch) return;
  t[threadIdx.x] = threadIdx.x;
  __syncthreads();
  sink[threadIdx.x] = t[255 - threadIdx.x];
}

int main() {
  const size_t n = (256u << 20) / 16;  // 16-byte vectors in 256 MB
  u32x4 *a, *b, *c;
  unsigned *flag, *sink;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMalloc(&c, n * 16));
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(a, 0, n * 16));
  CK(hipMemset(flag, 0, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"none", "w1", "wg1024", "wg1024_noflag", "wg256_16k"};
  const int iters = 50;
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 5; ++v) {
      auto iter = [&]() {
        k_copy<<<4096, 256>>>(a, b, n);
        if (v == 1) k_w1<<<1, 64>>>(flag, 7u, sink);
        if (v == 2) k_wg1024<<<1, 1024>>>(flag, 7u, sink);
        if (v == 3) k_wg1024_noflag<<<1, 1024>>>(sink, 0u);
        if (v == 4) k_wg256<<<1, 256>>>(flag, 7u, sink);
        k_copy<<<4096, 256>>>(b, c, n);
      };
      for (int i = 0; i < 5; ++i) iter();
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) iter();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("rep %d %-14s %8.2f us per iteration\n", rep, names[v], ms * 1e3 / iters);
    }
  }
  return 0;
}
