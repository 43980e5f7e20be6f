// LDS atomic rates on gfx950 at RANDOM addresses (a hash table's pattern), the
// shape of K5a's insert phase: one 1024-thread workgroup per CU, 16 Ki-slot
// table, 8 keys per lane per pass.  Ops: ds_cmpst_rtn_b32 (claim a slot),
// ds_max_u32 (no return), ds_add_rtn_u32, ds_read_b32; addresses uniform
// random, or with a Zipf-like share of lanes on a few hot slots.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/lds_atomic_rand.hip -o tools/micro/lds_atomic_rand
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// hot: of every 64 lanes, this many go to one of 4 hot slots; hot = -1: random
// rows but lane l of each 32-lane group on bank l (conflict-free: the bank a
// random table slot would need to land on to cost one LDS cycle per group)
template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t* out, int passes, int hot) {
  __shared__ uint32_t t[16384];
  uint32_t acc = 0;
  for (int p = 0; p < passes; ++p) {
    for (int i = threadIdx.x; i < 16384; i += 1024) t[i] = 0xFFFFFFFFu;
    __syncthreads();
    uint32_t slot[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t h = mix((blockIdx.x * 131u + p) * 8192u + q * 1024u + threadIdx.x);
      slot[q] = hot < 0 ? (((h & 16383u) & ~31u) | (threadIdx.x & 31u))
                        : ((threadIdx.x & 63) < (uint32_t)hot) ? (h & 3u) : (h & 16383u);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (OP == 0) acc += atomicCAS(&t[slot[q]], 0xFFFFFFFFu, threadIdx.x);
      if (OP == 1) atomicMax(&t[slot[q]], threadIdx.x);
      if (OP == 2) acc += atomicAdd(&t[slot[q]], 1u);
      if (OP == 3) acc += t[slot[q]];
    }
    __syncthreads();
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 4096 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int passes = 200, grid = 256;
  const char* names[] = {"ds_cmpst_rtn_b32", "ds_max_u32", "ds_add_rtn_u32", "ds_read_b32"};
  for (int hot : {0, -1, 4, 16}) {
    for (int op = 0; op < 4; ++op) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        if (op == 0) k<0><<<grid, 1024>>>(out, passes, hot);
        if (op == 1) k<1><<<grid, 1024>>>(out, passes, hot);
        if (op == 2) k<2><<<grid, 1024>>>(out, passes, hot);
        if (op == 3) k<3><<<grid, 1024>>>(out, passes, hot);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
      }
      // per CU: passes * 8 wave-instructions * 16 waves, 64 lanes each
      const double lane_ops = (double)passes * 8 * 1024;
      const double us = best * 1e3;
      std::printf("hot %2d/64  %-18s %8.1f us  %6.2f lane-ops/ns per CU  (%.0f cycles per pass at 2.1 GHz)\n",
                  hot, names[op], us, lane_ops / (us * 1e3), us * 2.1e3 / passes);
    }
  }
  hipFree(out);
  return 0;
}
