// On-device synthetic data.
//
// The reference builds every batch on the CPU (`torch.rand` `PY1:60`, `torch.randn/randint`
// `NB01:54-55`, `randn` + one-hot `scatter_` `NB03:375-377`) and copies it host→device inside the
// timed loop.  Benchmarks here generate batches in HBM with a counter-based Philox4x32-10
// generator: deterministic per (seed, offset), so every rank / step gets an independent, reproducible
// stream and nothing crosses PCIe.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;

struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox(uint64_t counter, uint64_t key64) {
  uint32_t c0 = (uint32_t)counter, c1 = (uint32_t)(counter >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)key64, k1 = (uint32_t)(key64 >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

__device__ __forceinline__ float u01(uint32_t v) { return ((float)(v >> 8) + 0.5f) * (1.f / 16777216.f); }

// kind: 0 uniform [a, b), 1 normal(mean=a, std=b)
template <typename T>
__global__ void __launch_bounds__(kThreads) fill_kernel(T* __restrict__ out, int64_t n, uint64_t seed, uint64_t offset,
                                                        int kind, float a, float b) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q * 4 < n; q += stride) {
    const u32x4 r = philox(offset + (uint64_t)q, seed);
    float v[4];
    if (kind == 0) {
      v[0] = a + (b - a) * u01(r.x);
      v[1] = a + (b - a) * u01(r.y);
      v[2] = a + (b - a) * u01(r.z);
      v[3] = a + (b - a) * u01(r.w);
    } else {
      const float r1 = sqrtf(-2.f * __logf(u01(r.x))), t1 = 6.2831853f * u01(r.y);
      const float r2 = sqrtf(-2.f * __logf(u01(r.z))), t2 = 6.2831853f * u01(r.w);
      v[0] = a + b * r1 * __cosf(t1);
      v[1] = a + b * r1 * __sinf(t1);
      v[2] = a + b * r2 * __cosf(t2);
      v[3] = a + b * r2 * __sinf(t2);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (q * 4 + j < n) Elem<T>::store(out, q * 4 + j, v[j]);
  }
}

__global__ void __launch_bounds__(kThreads) randint_kernel(int64_t* __restrict__ out, int64_t n, uint64_t seed,
                                                           uint64_t offset, int64_t low, int64_t high) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uint64_t range = (uint64_t)(high - low);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32x4 r = philox(offset + (uint64_t)i, seed ^ 0x5851F42D4C957F2DULL);
    const uint64_t v = ((uint64_t)r.x << 32) | r.y;
    out[i] = low + (int64_t)(v % range);
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

hipError_t fill_random(void* out, int dtype, int64_t n, uint64_t seed, uint64_t offset, int kind, float a, float b,
                       hipStream_t st) {
  const int g = grid_for((n + 3) / 4);
  if (dtype == 0) fill_kernel<float><<<g, kThreads, 0, st>>>((float*)out, n, seed, offset, kind, a, b);
  else fill_kernel<bf16_t><<<g, kThreads, 0, st>>>((bf16_t*)out, n, seed, offset, kind, a, b);
  return hipGetLastError();
}

hipError_t fill_randint(int64_t* out, int64_t n, uint64_t seed, uint64_t offset, int64_t low, int64_t high,
                        hipStream_t st) {
  randint_kernel<<<grid_for(n), kThreads, 0, st>>>(out, n, seed, offset, low, high);
  return hipGetLastError();
}

}  // namespace pda
