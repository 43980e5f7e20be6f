// Does hipExtLaunchKernel(..., hipExtAnyOrderLaunch) let a kernel start before
// the previous kernel on the same stream has finished, on gfx950?  Kernel A
// spins ~2 ms (one workgroup) and stamps its end; kernel B (one workgroup)
// stamps its start.  Printed: B's start relative to A's end (negative = B
// overlapped A), for a plain launch and an any-order launch.  Both kernels
// finish on their own; no workgroup waits on another.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>

__global__ void k_spin(unsigned long long* t, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0) t[0] = __builtin_amdgcn_s_memrealtime();
}

__global__ void k_mark(unsigned long long* t) {
  if (threadIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  unsigned long long* d = nullptr;
  unsigned long long h[2];
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  hipStream_t st;
  if (hipStreamCreate(&st) != hipSuccess) return 1;
  for (int flags : {0, (int)hipExtAnyOrderLaunch}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemsetAsync(d, 0, 16, st);
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, d, 200000ull);  // 100 MHz: 2 ms
      hipExtLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, st, nullptr, nullptr, (uint32_t)flags, d);
      if (hipStreamSynchronize(st) != hipSuccess) return 2;
      hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      std::printf("flags %d: B started %+.1f us after A ended\n", flags, ((double)h[1] - (double)h[0]) / 100.0);
    }
  }
  hipFree(d);
  return 0;
}
