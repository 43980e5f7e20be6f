// scatter_order.hip — does the ORDER of random single-value parameter stores
// matter?  K5b (cfg 3 resolve) stores ~2.6 M distinct 4-byte winners into a
// 1e8-float array, each lane its own winners, i.e. in random order inside a
// bucket; its ablation puts ~34 us on those stores.  This times the same
// store set issued
//   random     one store per lane, addresses in random order
//   bucketed   sorted inside 64 Ki-key buckets, buckets in random order
//              (what a K5b sweep over its bucket table in index order issues)
//   sorted     globally ascending
// and the same three for loads (the Zipf Get's line fills).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/scatter_order.hip -o /tmp/scatter_order
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

constexpr size_t kP = 100000000;  // parameters (floats)
constexpr uint32_t kN = 2600000;  // distinct stores

__global__ __launch_bounds__(256) void k_store(const uint32_t* __restrict__ off, uint32_t n,
                                               float* __restrict__ p) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[off[i]] = (float)i;
}

__global__ __launch_bounds__(256) void k_load(const uint32_t* __restrict__ off, uint32_t n,
                                              const float* __restrict__ p, float* __restrict__ out) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) out[i] = p[off[i]];
}

// reads a buffer larger than the Infinity Cache (clean lines only, so the
// timed kernel sees no write-back of it)
__global__ __launch_bounds__(256) void k_sweep(const float4* __restrict__ f, size_t n, float* sink) {
  float a = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a += f[i].x;
  if (a == 12345.f) *sink = a;
}

int main() {
  std::mt19937_64 rng(7);
  std::vector<uint32_t> all(kN);
  {  // kN distinct offsets, uniformly spread (a random subset of [0, kP))
    std::vector<uint32_t> pick;
    pick.reserve(kN * 11 / 10);
    while (pick.size() < kN * 11 / 10) pick.push_back((uint32_t)(rng() % kP));
    std::sort(pick.begin(), pick.end());
    pick.erase(std::unique(pick.begin(), pick.end()), pick.end());
    std::shuffle(pick.begin(), pick.end(), rng);
    pick.resize(kN);
    all = pick;
  }
  std::vector<uint32_t> rnd = all, srt = all, bkt = all;
  std::sort(srt.begin(), srt.end());
  {
    constexpr uint32_t B = 65536;
    const uint32_t nb = (uint32_t)((kP + B - 1) / B);
    std::vector<uint32_t> order(nb);
    std::iota(order.begin(), order.end(), 0u);
    std::shuffle(order.begin(), order.end(), rng);
    std::vector<uint32_t> rank(nb);
    for (uint32_t i = 0; i < nb; ++i) rank[order[i]] = i;
    std::sort(bkt.begin(), bkt.end(), [&](uint32_t a, uint32_t b) {
      const uint32_t ra = rank[a / B], rb = rank[b / B];
      return ra != rb ? ra < rb : a < b;
    });
  }
  float *p, *out;
  uint32_t* d;
  CK(hipMalloc(&p, kP * 4));
  CK(hipMalloc(&out, kN * 4));
  CK(hipMalloc(&d, kN * 4));
  CK(hipMemset(p, 0, kP * 4));
  // a 512 MB buffer read between runs: no run finds the previous one's lines
  // in the 256 MB Infinity Cache
  float* flush;
  const size_t fl = 128u << 20;
  CK(hipMalloc(&flush, fl * 4));
  CK(hipMemset(flush, 0, fl * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, const std::vector<uint32_t>& v, bool store) {
    CK(hipMemcpy(d, v.data(), kN * 4, hipMemcpyHostToDevice));
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
      k_sweep<<<4096, 256>>>(reinterpret_cast<const float4*>(flush), fl / 4, out);
      CK(hipEventRecord(e0, 0));
      if (store)
        k_store<<<4096, 256>>>(d, kN, p);
      else
        k_load<<<4096, 256>>>(d, kN, p, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    std::printf("%-6s %-9s %8.1f us  %6.1f G accesses/s\n", store ? "store" : "load", name, med * 1e3,
                kN / (med * 1e-3) / 1e9);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("random", rnd, true);
    run("bucketed", bkt, true);
    run("sorted", srt, true);
    run("random", rnd, false);
    run("bucketed", bkt, false);
    run("sorted", srt, false);
  }
  return 0;
}
