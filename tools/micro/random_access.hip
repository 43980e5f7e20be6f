// random_access.hip — the random single-value access ceiling of this part, as
// a small library bench.py loads (ctypes) to price the cfg-3 kernels on the
// same box: each thread reads four 4-byte offsets with one 16-byte load and
// issues their four independent gathers (or scatters) together, 16 offsets
// per lane in flight over a grid-stride loop.  A random 4-byte access costs a
// DRAM row activation and a 64-byte sector (a store: a partial-line write the
// memory side must merge), so the rate of these — not 8 TB/s — bounds a
// kernel that touches one value per key (K1 on Zipf pulls, K5b's winner
// stores).  Not part of libpskv; built by parameter_server_amd/build.py.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kBlock = 256;
constexpr int kPer = 16;  // offsets per lane per grid-stride step (4 x 16-byte loads)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kBlock) void k_ra_gather(const uint32_t* __restrict__ off, uint32_t n,
                                                      const float* __restrict__ p,
                                                      float* __restrict__ out) {
  const uint32_t n4 = n / 4;
  for (uint32_t g = blockIdx.x * kBlock + threadIdx.x; g < (n4 + 3) / 4; g += gridDim.x * kBlock) {
    u32x4 o[4];
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t q = g * 4 + j;
      o[j] = q < n4 ? reinterpret_cast<const u32x4*>(off)[q] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j * 4 + e] = g * 4 + j < n4 ? p[o[j][e]] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (g * 4 + j < n4)
        reinterpret_cast<float4*>(out)[g * 4 + j] = float4{v[j * 4], v[j * 4 + 1], v[j * 4 + 2], v[j * 4 + 3]};
  }
  // the n % 4 tail
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t < n - n4 * 4) out[n4 * 4 + t] = p[off[n4 * 4 + t]];
}

__global__ __launch_bounds__(kBlock) void k_ra_scatter(const uint32_t* __restrict__ off, uint32_t n,
                                                       const float* __restrict__ val,
                                                       float* __restrict__ p) {
  const uint32_t n4 = n / 4;
  for (uint32_t g = blockIdx.x * kBlock + threadIdx.x; g < (n4 + 3) / 4; g += gridDim.x * kBlock) {
    u32x4 o[4];
    float4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t q = g * 4 + j;
      o[j] = q < n4 ? reinterpret_cast<const u32x4*>(off)[q] : u32x4{0u, 0u, 0u, 0u};
      v[j] = q < n4 ? reinterpret_cast<const float4*>(val)[q] : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (g * 4 + j < n4) {
        p[o[j][0]] = v[j].x;
        p[o[j][1]] = v[j].y;
        p[o[j][2]] = v[j].z;
        p[o[j][3]] = v[j].w;
      }
  }
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t < n - n4 * 4) p[off[n4 * 4 + t]] = val[n4 * 4 + t];
}

}  // namespace

// off, p, out / val: device pointers (off and out / val 16-byte aligned);
// every offset < the array's length.  Returns a hipError_t.
extern "C" int ra_gather(const uint32_t* off, uint32_t n, const float* p, float* out, void* stream) {
  if (n == 0) return 0;
  const uint32_t lanes = (n / 4 + 3) / 4;
  uint32_t grid = (lanes + kBlock - 1) / kBlock;
  if (grid == 0) grid = 1;
  k_ra_gather<<<grid, kBlock, 0, static_cast<hipStream_t>(stream)>>>(off, n, p, out);
  return (int)hipGetLastError();
}

extern "C" int ra_scatter(const uint32_t* off, uint32_t n, const float* val, float* p, void* stream) {
  if (n == 0) return 0;
  const uint32_t lanes = (n / 4 + 3) / 4;
  uint32_t grid = (lanes + kBlock - 1) / kBlock;
  if (grid == 0) grid = 1;
  k_ra_scatter<<<grid, kBlock, 0, static_cast<hipStream_t>(stream)>>>(off, n, val, p);
  return (int)hipGetLastError();
}
