// stream_mix.hip — what limits the dense grouped Add (K2g) relative to the
// gather (K1)?  Both move three 16-byte-per-lane streams (K1: keys + params
// in, values out; K2g: keys + values in, params out), yet K1 sustains ~7.1 TB/s
// of real traffic and K2g ~6.0.  This program times K1/K2g-shaped kernels that
// differ in ONE property each, on cfg-2 data (64 windows of 1M keys at
// seed-style 1M-aligned bases in a 1e8-float array).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/stream_mix.hip -o /tmp/stream_mix
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256;
constexpr uint32_t kN = 1000000;   // keys per window
constexpr int kJ = 64;             // windows

struct Win {
  uint32_t order[kJ];  // processing order of the windows (identity, or by base)
  uint32_t first[kJ];
  uint32_t covered[kJ];  // 1: a later window repeats this one (its values cannot survive)
};

template <bool NT>
__device__ __forceinline__ u32x4 ld(const void* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(void* p, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else
    *reinterpret_cast<u32x4*>(p) = v;
}

// chunk c of the concatenated windows -> (window, base offset); whole chunks
// only (kN is not a multiple of the chunk: the tail chunk is skipped, same for
// every variant)
template <int U>
__device__ __forceinline__ bool chunk_of(const Win& w, uint32_t c, int& j, uint32_t& base) {
  constexpr uint32_t CH = kB * 4 * U;
  constexpr uint32_t per = kN / CH;
  const uint32_t q = c / per;
  if (q >= (uint32_t)kJ) return false;
  j = (int)w.order[q];
  base = (c % per) * CH;
  return true;
}

// MODE 0: K1 gather  keys(nt) + param(plain) -> out(nt)
// MODE 1: K2g add    keys(nt) + vals(nt) -> param (store policy STNT)
// MODE 2: vals only  vals(nt) -> param (no key stream)
// MODE 3: K2g add honouring `covered` (keys only for covered windows)
// MODE 4: K2g add, keys and values interleaved per u (load k,v ; k,v ; ...)
// MODE 5: K2g add pattern but the values go to `out` (contiguous) instead of the param windows
// MODE 6: MODE 3 behind a K2g-style prologue: waves 0-1 load the first and last
//         key of every window (128 dependent scattered loads) and the workgroup
//         waits for them (barrier) before its chunk loads
// MODE 7: MODE 3 checking all four keys of every 16-byte group (as K2g does)
template <int MODE, int U, bool STNT, bool KNT = true, bool VNT = true>
__global__ __launch_bounds__(kB) void k_mix(const uint32_t* __restrict__ keys,
                                            const uint32_t* __restrict__ vals,
                                            uint32_t* __restrict__ param, uint32_t* __restrict__ out,
                                            Win w, uint32_t* bad) {
  int j;
  uint32_t base;
  if (!chunk_of<U>(w, blockIdx.x, j, base)) return;
  const uint32_t t = threadIdx.x;
  const size_t g0 = (size_t)j * kN + base;  // element index in the concatenation
  const uint32_t first = w.first[j];
  bool b = false;
  if (MODE == 6) {
    __shared__ uint32_t s_fl[2 * kJ];
    if (t < 2 * kJ) {
      const int q = (int)t % kJ;
      s_fl[t] = keys[(size_t)q * kN + (t < kJ ? 0 : kN - 1)];
    }
    __syncthreads();
    b |= s_fl[j] != first;
  }
  if (MODE == 0) {
    u32x4 k[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) k[u] = ld<true>(keys + g0 + (u * kB + t) * 4);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<false>(param + k[u].x);
#pragma unroll
    for (int u = 0; u < U; ++u) st<true>(out + g0 + (u * kB + t) * 4, v[u]);
  } else if (MODE == 2) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<VNT>(vals + g0 + (u * kB + t) * 4);
#pragma unroll
    for (int u = 0; u < U; ++u) st<STNT>(param + first + base + (u * kB + t) * 4, v[u]);
  } else if (MODE == 4) {
    u32x4 k[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      k[u] = ld<true>(keys + g0 + (u * kB + t) * 4);
      v[u] = ld<true>(vals + g0 + (u * kB + t) * 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k0 = first + base + (u * kB + t) * 4;
      b |= k[u].x != k0 || k[u].w != k0 + 3;
      st<STNT>(param + k0, v[u]);
    }
  } else {
    const bool cov = (MODE == 3 || MODE == 6 || MODE == 7) && w.covered[j];
    u32x4 k[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) k[u] = ld<KNT>(keys + g0 + (u * kB + t) * 4);
    if (!cov) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld<VNT>(vals + g0 + (u * kB + t) * 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k0 = first + base + (u * kB + t) * 4;
      if (MODE == 7)
        b |= (k[u].x != k0) | (k[u].y != k0 + 1) | (k[u].z != k0 + 2) | (k[u].w != k0 + 3);
      else
        b |= k[u].x != k0 || k[u].w != k0 + 3;
      if (!cov) {
        if (MODE == 5)
          st<STNT>(out + g0 + (u * kB + t) * 4, v[u]);
        else
          st<STNT>(param + k0, v[u]);
      }
    }
  }
  if (b) *bad = 1;
}

int main() {
  const size_t P = 100000000;
  std::vector<uint32_t> hk((size_t)kJ * kN);
  Win w{};
  std::mt19937_64 rng(42);
  std::vector<int> last(100, -1);
  for (int j = 0; j < kJ; ++j) {
    w.first[j] = (uint32_t)(rng() % 100) * kN;
    for (uint32_t i = 0; i < kN; ++i) hk[(size_t)j * kN + i] = w.first[j] + i;
  }
  for (int j = 0; j < kJ; ++j) last[w.first[j] / kN] = j;
  for (int j = 0; j < kJ; ++j) w.order[j] = j;
  Win ws = w;  // windows in ascending base order
  std::sort(ws.order, ws.order + kJ, [&](uint32_t x, uint32_t y) { return w.first[x] < w.first[y]; });
  int ncov = 0;
  for (int j = 0; j < kJ; ++j) {
    w.covered[j] = last[w.first[j] / kN] != j;
    ncov += w.covered[j];
  }
  uint32_t *keys, *vals, *param, *out, *bad;
  CK(hipMalloc(&keys, hk.size() * 4));
  CK(hipMalloc(&vals, hk.size() * 4));
  CK(hipMalloc(&out, hk.size() * 4));
  CK(hipMalloc(&param, P * 4));
  CK(hipMalloc(&bad, 4));
  CK(hipMemcpy(keys, hk.data(), hk.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(vals, 1, hk.size() * 4));
  CK(hipMemset(param, 0, P * 4));
  CK(hipMemset(bad, 0, 4));
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  std::printf("%d of %d windows covered by a later one\n", ncov, kJ);
  // lds > 0: dynamic LDS per workgroup that caps the workgroups per CU (30 KiB:
  // 5 per CU = 5 waves per SIMD, K2g's register-limited occupancy)
  auto run = [&](const char* name, auto kern, int U, double bytes_per_key_full, double bytes_cov,
                 bool sorted = false, size_t lds = 0) {
    const uint32_t CH = kB * 4 * U;
    const uint32_t grid = kJ * (kN / CH);
    const double keys_done = (double)grid * CH;
    const double frac_cov = (double)ncov / kJ;
    const double bytes = keys_done * (bytes_per_key_full * (1 - frac_cov) + bytes_cov * frac_cov);
    std::vector<float> ts;
    for (int r = 0; r < 30; ++r) {
      CK(hipEventRecord(ev0, 0));
      kern<<<grid, kB, lds, 0>>>(keys, vals, param, out, sorted ? ws : w, bad);
      CK(hipEventRecord(ev1, 0));
      CK(hipEventSynchronize(ev1));
      float ms;
      CK(hipEventElapsedTime(&ms, ev0, ev1));
      if (r >= 5) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    std::printf("%-44s %8.1f us  %7.0f GB/s real\n", name, med * 1e3, bytes / (med * 1e-3) / 1e9);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("K1 gather keys+param->out", k_mix<0, 8, false>, 8, 12, 12);
    run("K2g add keys+vals->param (plain st)", k_mix<1, 8, false>, 8, 12, 12);
    run("K2g covered-skip behind a first/last prologue", k_mix<6, 8, false>, 8, 12, 4);
    run("K2g add keys+vals->param (nt st)", k_mix<1, 8, true>, 8, 12, 12);
    run("K2g add covered-skip (plain st)", k_mix<3, 8, false>, 8, 12, 4);
    run("K2g add interleaved loads (plain st)", k_mix<4, 8, false>, 8, 12, 12);
    run("vals->param only (plain st)", k_mix<2, 8, false>, 8, 8, 8);
    run("K2g add U=4 (plain st)", k_mix<1, 4, false>, 4, 12, 12);
    run("K2g add, keys nt, vals plain", k_mix<1, 8, false, true, false>, 8, 12, 12);
    run("K2g add, keys plain, vals nt", k_mix<1, 8, false, false, true>, 8, 12, 12);
    run("K2g add, keys plain, vals plain", k_mix<1, 8, false, false, false>, 8, 12, 12);
    run("K2g add, keys nt, vals plain, nt st", k_mix<1, 8, true, true, false>, 8, 12, 12);
    run("K2g covered-skip, keys nt, vals plain", k_mix<3, 8, false, true, false>, 8, 12, 4);
    run("vals(plain)->param only", k_mix<2, 8, false, true, false>, 8, 8, 8);
    run("K2g add, values -> contiguous out", k_mix<5, 8, false>, 8, 12, 12);
    run("K2g add, values -> contiguous out (nt)", k_mix<5, 8, true>, 8, 12, 12);
    run("K2g add, windows in base order", k_mix<1, 8, false>, 8, 12, 12, true);
    run("K2g covered-skip, windows in base order", k_mix<3, 8, false>, 8, 12, 4, true);
    run("vals->param only, windows in base order", k_mix<2, 8, false>, 8, 8, 8, true);
    run("K1 gather, windows in base order", k_mix<0, 8, false>, 8, 12, 12, true);
    run("K1 gather U=4", k_mix<0, 4, false>, 4, 12, 12);
    run("K2g covered-skip, all four keys checked", k_mix<7, 8, false>, 8, 12, 4);
    run("K2g covered-skip, all keys, 5 waves/SIMD", k_mix<7, 8, false>, 8, 12, 4, false, 30 << 10);
    run("K2g covered-skip, 5 waves/SIMD", k_mix<3, 8, false>, 8, 12, 4, false, 30 << 10);
    run("K1 gather, 5 waves/SIMD", k_mix<0, 8, false>, 8, 12, 12, false, 30 << 10);
  }
  uint32_t hb = 0;
  CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  std::printf("key check: %s\n", hb ? "FAILED" : "ok");
  return 0;
}
