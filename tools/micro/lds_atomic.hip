// LDS atomic throughput microbenchmark (gfx950): ds_add_f32 vs ds_max_u32 vs
// ds_add_u32, distinct addresses (stride 1) vs k-way same-address conflicts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ __launch_bounds__(1024) void k(float* out, int iters, int conflict) {
  __shared__ uint32_t t[16384];
  for (int i = threadIdx.x; i < 16384; i += 1024) t[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x;
  uint32_t a = conflict ? (lane / conflict) * 97u : lane * 13u;
  for (int it = 0; it < iters; ++it) {
    const uint32_t idx = (a + it * 1031u) & 16383u;
    if (OP == 0) atomicAdd(reinterpret_cast<float*>(&t[idx]), 1.0f);
    if (OP == 1) atomicMax(&t[idx], (uint32_t)it);
    if (OP == 2) atomicAdd(&t[idx], 1u);
    if (OP == 3) {  // float add as an integer compare-and-swap loop
      uint32_t old = t[idx], assumed;
      do {
        assumed = old;
        old = atomicCAS(&t[idx], assumed, __float_as_uint(__uint_as_float(assumed) + 1.0f));
      } while (old != assumed);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = __uint_as_float(t[5]);
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096, grid = 256;
  const char* names[] = {"ds_add_f32(atomicAdd)", "ds_max_u32", "ds_add_u32", "f32 add via ds_cmpst loop"};
  for (int conflict : {0, 1, 2, 4, 16, 64}) {
    for (int op = 0; op < 4; ++op) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (op == 0) k<0><<<grid, 1024>>>(out, iters, conflict);
        if (op == 1) k<1><<<grid, 1024>>>(out, iters, conflict);
        if (op == 2) k<2><<<grid, 1024>>>(out, iters, conflict);
        if (op == 3) k<3><<<grid, 1024>>>(out, iters, conflict);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1)
          printf("conflict=%2d %-26s %8.3f ms  %7.1f G atomics/s\n", conflict, names[op], ms,
                 (double)grid * 1024 * iters / ms / 1e6);
      }
    }
  }
  return 0;
}
