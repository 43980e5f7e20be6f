// cold_stream.hip — the HBM ceiling of the dense step's access patterns, every
// byte served by HBM (round 4).  Each launch works on a
// region of a 16 GB pool that no launch touched for ≥ 12 GB of traffic, so
// neither L2 nor the 256 MB Infinity Cache holds any of it.  Shapes, 16 bytes
// per lane, U = 8 loads per lane in flight (K1's and K2g's own geometry:
// 256-thread workgroups, one 8 Ki-element chunk each):
//   read     sum a                          (4 B / element)
//   copy     c = a                          (8 B)
//   add      c = a ^ b                      (12 B: K2g's keys + values -> params)
//   gather   c = b[a[i] - base]             (12 B: K1's keys -> params -> outs; a holds
//                                            consecutive keys, so the parameter load
//                                            depends on the key load as in K1)
//   step     add into one region, then gather from another (the dense step:
//            K2g's writes left dirty, then K1)
// Cache policy per stream: loads plain / nt, stores plain / nt.  GB/s counts
// every byte of every stream once.  Not part of libpskv: a measurement.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/cold_stream.hip -o tools/micro/cold_stream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

namespace {

constexpr int kBlock = 256;
constexpr int U = 8;
constexpr int CH = kBlock * 4 * U;  // elements per workgroup
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint32_t* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(uint32_t* p, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else
    *reinterpret_cast<u32x4*>(p) = v;
}

template <bool NTA>
__global__ __launch_bounds__(kBlock) void k_read(const uint32_t* __restrict__ a, uint32_t* __restrict__ sink) {
  const uint64_t base = (uint64_t)blockIdx.x * CH;
  u32x4 s = {0, 0, 0, 0};
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NTA>(a + base + (uint64_t)(u * kBlock + threadIdx.x) * 4);
#pragma unroll
  for (int u = 0; u < U; ++u) s ^= v[u];
  if ((s.x ^ s.y ^ s.z ^ s.w) == 0x9e3779b9u) sink[blockIdx.x] = s.x;  // never in practice
}

template <bool NTA, bool NTS>
__global__ __launch_bounds__(kBlock) void k_copy(const uint32_t* __restrict__ a, uint32_t* __restrict__ c) {
  const uint64_t base = (uint64_t)blockIdx.x * CH;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NTA>(a + base + (uint64_t)(u * kBlock + threadIdx.x) * 4);
#pragma unroll
  for (int u = 0; u < U; ++u) st<NTS>(c + base + (uint64_t)(u * kBlock + threadIdx.x) * 4, v[u]);
}

template <bool NTA, bool NTB, bool NTS>
__global__ __launch_bounds__(kBlock) void k_add(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                uint32_t* __restrict__ c) {
  const uint64_t base = (uint64_t)blockIdx.x * CH;
  u32x4 v[U], w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    v[u] = ld<NTA>(a + base + (uint64_t)(u * kBlock + threadIdx.x) * 4);
    w[u] = ld<NTB>(b + base + (uint64_t)(u * kBlock + threadIdx.x) * 4);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) st<NTS>(c + base + (uint64_t)(u * kBlock + threadIdx.x) * 4, v[u] ^ w[u]);
}

// c[i] = b[a[i] - key0]: a holds consecutive keys, so every lane's four keys
// are a run and one 16-byte parameter load serves them (K1's dense case)
template <bool NTA, bool NTB, bool NTS>
__global__ __launch_bounds__(kBlock) void k_gather(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                   uint32_t key0, uint32_t* __restrict__ c) {
  const uint64_t base = (uint64_t)blockIdx.x * CH;
  u32x4 k[U], v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) k[u] = ld<NTA>(a + base + (uint64_t)(u * kBlock + threadIdx.x) * 4);
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NTB>(b + (uint64_t)(k[u].x - key0));
#pragma unroll
  for (int u = 0; u < U; ++u) st<NTS>(c + base + (uint64_t)(u * kBlock + threadIdx.x) * 4, v[u]);
}

__global__ void k_iota(uint32_t* a, uint64_t n, uint32_t key0) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = key0 + (uint32_t)i;
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (64ull << 20);  // elements per stream
  const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
  const uint64_t pool_bytes = 16ull << 30;
  const uint64_t region = n * 4;
  const uint64_t nreg = pool_bytes / region;
  if (n % CH != 0 || nreg < 24) {
    std::fprintf(stderr, "n must be a multiple of %d and at most %llu\n", CH,
                 (unsigned long long)(pool_bytes / 24 / 4));
    return 2;
  }
  char* pool = nullptr;
  CHECK(hipMalloc(&pool, pool_bytes));
  CHECK(hipMemset(pool, 0, pool_bytes));
  uint32_t* sink = nullptr;
  CHECK(hipMalloc(&sink, 1 << 20));
  // the key streams of the gather: regions of consecutive keys that no kernel
  // writes (a gather index is always inside its parameter region)
  const uint64_t nkey = 16;
  char* keypool = nullptr;
  CHECK(hipMalloc(&keypool, nkey * region));
  const uint32_t key0 = 12345;
  for (uint64_t r = 0; r < nkey; ++r)
    k_iota<<<4096, 256>>>(reinterpret_cast<uint32_t*>(keypool + r * region), n, key0);
  CHECK(hipDeviceSynchronize());
  const uint32_t nwg = (uint32_t)(n / CH);
  uint64_t next = 0, next_key = 0;
  auto take = [&]() { return reinterpret_cast<uint32_t*>(pool + (next++ % nreg) * region); };
  auto take_key = [&]() { return reinterpret_cast<uint32_t*>(keypool + (next_key++ % nkey) * region); };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // p[0..2]: data regions (any kernel may write p[1] / p[2]); p[3]: a key region
  auto timed = [&](const char* name, int streams, bool cold, auto launch) {
    std::vector<float> ms;
    uint32_t* fixed[4] = {take(), take(), take(), take_key()};
    for (int r = 0; r < reps + 1; ++r) {
      uint32_t* p[4];
      for (int q = 0; q < 3; ++q) p[q] = cold ? take() : fixed[q];
      p[3] = cold ? take_key() : fixed[3];
      CHECK(hipEventRecord(e0));
      launch(p);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float t = 0;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      if (r) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const float med = ms[ms.size() / 2];
    std::printf("%-44s %s %8.1f us  %7.0f GB/s\n", name, cold ? "cold" : "warm", med * 1e3,
                (double)streams * region / (med * 1e-3) / 1e9);
    std::fflush(stdout);
  };
  for (int cold = 1; cold >= 0; --cold) {
    timed("read", 1, cold, [&](uint32_t** p) { k_read<false><<<nwg, kBlock>>>(p[0], sink); });
    timed("read nt", 1, cold, [&](uint32_t** p) { k_read<true><<<nwg, kBlock>>>(p[0], sink); });
    timed("copy", 2, cold, [&](uint32_t** p) { k_copy<false, false><<<nwg, kBlock>>>(p[0], p[1]); });
    timed("copy nt-ld", 2, cold, [&](uint32_t** p) { k_copy<true, false><<<nwg, kBlock>>>(p[0], p[1]); });
    timed("copy nt-st", 2, cold, [&](uint32_t** p) { k_copy<false, true><<<nwg, kBlock>>>(p[0], p[1]); });
    timed("copy nt-ld nt-st", 2, cold, [&](uint32_t** p) { k_copy<true, true><<<nwg, kBlock>>>(p[0], p[1]); });
    timed("add (K2g) plain", 3, cold, [&](uint32_t** p) { k_add<false, false, false><<<nwg, kBlock>>>(p[0], p[1], p[2]); });
    timed("add (K2g) nt-ld, plain st", 3, cold,
          [&](uint32_t** p) { k_add<true, true, false><<<nwg, kBlock>>>(p[0], p[1], p[2]); });
    timed("add (K2g) nt-ld, nt st", 3, cold,
          [&](uint32_t** p) { k_add<true, true, true><<<nwg, kBlock>>>(p[0], p[1], p[2]); });
    timed("add (K2g) plain ld, nt st", 3, cold,
          [&](uint32_t** p) { k_add<false, false, true><<<nwg, kBlock>>>(p[0], p[1], p[2]); });
    timed("gather (K1) nt keys, plain params, nt out", 3, cold,
          [&](uint32_t** p) { k_gather<true, false, true><<<nwg, kBlock>>>(p[3], p[1], key0, p[2]); });
    timed("gather (K1) nt keys, nt params, nt out", 3, cold,
          [&](uint32_t** p) { k_gather<true, true, true><<<nwg, kBlock>>>(p[3], p[1], key0, p[2]); });
    timed("gather (K1) plain keys/params, plain out", 3, cold,
          [&](uint32_t** p) { k_gather<false, false, false><<<nwg, kBlock>>>(p[3], p[1], key0, p[2]); });
    timed("gather (K1) nt keys, nt params, plain out", 3, cold,
          [&](uint32_t** p) { k_gather<true, true, false><<<nwg, kBlock>>>(p[3], p[1], key0, p[2]); });
  }
  // the step: K2g-like add (nt loads, plain param stores) then K1-like gather
  // from other parameters, both cold, back to back; time of the pair
  for (int pol = 0; pol < 4; ++pol) {
    const bool ntp_st = pol & 1, ntp_ld = pol & 2;
    char name[96];
    std::snprintf(name, sizeof(name), "step: add (%s param st) + gather (%s param ld)", ntp_st ? "nt" : "plain",
                  ntp_ld ? "nt" : "plain");
    timed(name, 6, true, [&](uint32_t** p) {
      uint32_t* q[3] = {take_key(), take(), take()};
      if (ntp_st)
        k_add<true, true, true><<<nwg, kBlock>>>(p[0], p[1], p[2]);
      else
        k_add<true, true, false><<<nwg, kBlock>>>(p[0], p[1], p[2]);
      if (ntp_ld)
        k_gather<true, true, true><<<nwg, kBlock>>>(q[0], q[1], key0, q[2]);
      else
        k_gather<true, false, true><<<nwg, kBlock>>>(q[0], q[1], key0, q[2]);
    });
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipFree(pool));
  CHECK(hipFree(keypool));
  CHECK(hipFree(sink));
  return 0;
}
