// Standalone lab for the BatchNorm+residual+ReLU forward apply (bn_apply_reg_kernel<true,true>):
// y = relu(x*scale + shift + res) and the 1-bit ReLU mask.  In the ResNet-50 bs512 step it streams
// at ~4.3 TB/s on the layer1/2 shapes while the backward apply (same 2-read/1-write traffic, mask
// read instead of written) reaches ~5.5: this lab isolates the mask store.  Buffers rotate over 4
// sets so every pass streams from HBM.
//   hipcc -O3 --offload-arch=gfx950 -I csrc/include tools/bnlab/apply_lab.hip -o /tmp/apply_lab
// Variants:
//   0 current kernel (grid-stride, a lane's 4 vectors a grid stride apart, one mask byte per vector)
//   1 current kernel without the mask store (upper bound)
//   2 wave-contiguous: a wave iteration covers 256 consecutive vectors (4 coalesced 1-KB
//     instructions per tensor) and writes their 256 mask bytes as one 4-B store per lane
//     (bytes regrouped with 4 shuffles)
//   3 variant 2 with nontemporal stores of y and the mask
//   4 plain 16-B copy x -> y (roofline reference; bytes counted as 2 tensors)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "pda_common.h"
using namespace pda;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int NT = 256;

__device__ __forceinline__ uint32_t relu8(float (&a)[8], const float (&xv)[8], const float (&rv)[8],
                                          const float (&sc)[8], const float (&sh)[8]) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = fmaf(xv[j], sc[j], sh[j]) + rv[j];
    m |= (a[j] > 0.f ? 1u : 0u) << j;
    a[j] = fmaxf(a[j], 0.f);
  }
  return m;
}

template <bool BITS>
__global__ void __launch_bounds__(NT) apply_cur(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                bf16_t* __restrict__ y, uint8_t* __restrict__ bits, int64_t nvec,
                                                int cv, const float* __restrict__ scale,
                                                const float* __restrict__ shift) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(v % cv) * 8;
  float sc[8], sh[8];
  load8(scale + c0, sc);
  load8(shift + c0, sh);
  constexpr int U = 4;
  for (; v + (U - 1) * stride < nvec; v += U * stride) {
    float a[U][8], r[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) load8(x + (v + u * stride) * 8, a[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) load8(res + (v + u * stride) * 8, r[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float o[8];
      const uint32_t m = relu8(o, a[u], r[u], sc, sh);
      if (BITS) bits[v + u * stride] = (uint8_t)m;
      store8(y + (v + u * stride) * 8, o);
    }
  }
  for (; v < nvec; v += stride) {
    float a[8], r[8], o[8];
    load8(x + v * 8, a);
    load8(res + v * 8, r);
    const uint32_t m = relu8(o, a, r, sc, sh);
    if (BITS) bits[v] = (uint8_t)m;
    store8(y + v * 8, o);
  }
}

// NS = coefficient sets per lane (cv <= 64: 1; cv = 128: 2; cv = 256: 4)
template <int NS, bool NTS>
__global__ void __launch_bounds__(NT) apply_wave(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                 bf16_t* __restrict__ y, uint8_t* __restrict__ bits, int64_t nvec,
                                                 int cv, const float* __restrict__ scale,
                                                 const float* __restrict__ shift) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int64_t tw = (int64_t)gridDim.x * (NT / 64);
  float sc[NS][8], sh[NS][8];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c0 = (int)((s * 64 + lane) % cv) * 8;
    load8(scale + c0, sc[s]);
    load8(shift + c0, sh[s]);
  }
  int64_t base = gw * 256;
  for (; base + 256 <= nvec; base += tw * 256) {
    float a[4][8], r[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8(x + (base + u * 64 + lane) * 8, a[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) load8(res + (base + u * 64 + lane) * 8, r[u]);
    uint32_t w = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float o[8];
      const uint32_t m = relu8(o, a[u], r[u], sc[u % NS], sh[u % NS]);
      w |= m << (8 * u);
      bf16_t* dst = y + (base + u * 64 + lane) * 8;
      if (NTS) {
        u16x8 q;
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = f2bf(o[j]);
        __builtin_nontemporal_store(q, reinterpret_cast<u16x8*>(dst));
      } else {
        store8(dst, o);
      }
    }
    // lane l stores the mask bytes of vectors base + 4l .. 4l+3: vector j = 4l + k lives in lane j & 63
    // as byte j >> 6 (= l >> 4) of that lane's packed word
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t t = (uint32_t)__shfl((int)w, (4 * lane + k) & 63, 64);
      out |= ((t >> (8 * (lane >> 4))) & 0xFFu) << (8 * k);
    }
    uint32_t* bdst = reinterpret_cast<uint32_t*>(bits + base) + lane;
    if (NTS) __builtin_nontemporal_store(out, bdst);
    else *bdst = out;
  }
  // tail (< 256 vectors for this wave): one byte per vector
  for (int64_t v = base + lane; base < nvec && v < nvec && v < base + 256; v += 64) {
    const int c0 = (int)(v % cv) * 8;
    float s1[8], h1[8], a[8], r[8], o[8];
    load8(scale + c0, s1);
    load8(shift + c0, h1);
    load8(x + v * 8, a);
    load8(res + v * 8, r);
    bits[v] = (uint8_t)relu8(o, a, r, s1, h1);
    store8(y + v * 8, o);
  }
}

// pseudo-random bf16 in +-[0.5, 2) with random signs
__global__ void fill_k(bf16_t* p, int64_t n, uint32_t seed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (bf16_t)(0x3f00 + (h & 0xFF) + ((h >> 8) & 1 ? 0x8000 : 0));
  }
}

__global__ void copy_k(const u16x8* __restrict__ a, u16x8* __restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

int main() {
  const int64_t shapes[][2] = {{512LL * 56 * 56, 256}, {512LL * 28 * 28, 512}, {512LL * 14 * 14, 1024},
                               {512LL * 7 * 7, 2048}, {512LL * 56 * 56, 64}};
  const int SETS = 4;
  for (auto& sh : shapes) {
    const int64_t M = sh[0], C = sh[1], n = M * C, nvec = n / 8;
    const int cv = (int)(C / 8);
    std::vector<bf16_t*> X(SETS), R(SETS), Y(SETS);
    std::vector<uint8_t*> B(SETS), B2(SETS);
    for (int s = 0; s < SETS; ++s) {
      CK(hipMalloc(&X[s], n * 2));
      CK(hipMalloc(&R[s], n * 2));
      CK(hipMalloc(&Y[s], n * 2));
      CK(hipMalloc(&B[s], nvec));
      CK(hipMalloc(&B2[s], nvec));
      fill_k<<<2048, NT>>>(X[s], n, 12345u + s);
      fill_k<<<2048, NT>>>(R[s], n, 777u + s);
    }
    float *scale, *shift;
    CK(hipMalloc(&scale, C * 4));
    CK(hipMalloc(&shift, C * 4));
    std::vector<float> hs(C), hh(C);
    for (int c = 0; c < C; ++c) { hs[c] = 0.5f + 0.01f * (c % 7); hh[c] = -0.1f * (c % 3); }
    CK(hipMemcpy(scale, hs.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(shift, hh.data(), C * 4, hipMemcpyHostToDevice));
    int64_t g = (nvec + NT - 1) / NT;
    if (g > 2048) g = 2048;
    const int grid = (int)g;
    const int NS = cv <= 64 ? 1 : cv / 64;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("M=%lld C=%lld (%.0f MB per tensor)\n", (long long)M, (long long)C, n * 2 / 1e6);
    for (int var = 0; var <= 4; ++var) {
      auto run = [&](int s) {
        if (var == 0) apply_cur<true><<<grid, NT>>>(X[s], R[s], Y[s], B[s], nvec, cv, scale, shift);
        else if (var == 1) apply_cur<false><<<grid, NT>>>(X[s], R[s], Y[s], B[s], nvec, cv, scale, shift);
        else if (var == 4) copy_k<<<grid, NT>>>((const u16x8*)X[s], (u16x8*)Y[s], nvec);
        else {
          const bool nts = var == 3;
#define L(NSV, NTV) apply_wave<NSV, NTV><<<grid, NT>>>(X[s], R[s], Y[s], B2[s], nvec, cv, scale, shift)
          if (NS == 1) { if (nts) L(1, true); else L(1, false); }
          else if (NS == 2) { if (nts) L(2, true); else L(2, false); }
          else { if (nts) L(4, true); else L(4, false); }
#undef L
        }
      };
      for (int s = 0; s < SETS; ++s) run(s);
      CK(hipDeviceSynchronize());
      const int IT = 12;
      CK(hipEventRecord(e0));
      for (int i = 0; i < IT; ++i) run(i % SETS);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= IT;
      const double bytes = var == 4 ? 2.0 * n * 2 : (var == 1 ? 3.0 * n * 2 : 3.0 * n * 2 + nvec);
      printf("  var %d: %8.1f us  %5.2f TB/s\n", var, ms * 1e3, bytes / ms / 1e9);
    }
    // the wave-contiguous mask must equal the per-vector one
    std::vector<uint8_t> b0(nvec), b2(nvec);
    apply_cur<true><<<grid, NT>>>(X[0], R[0], Y[0], B[0], nvec, cv, scale, shift);
    if (NS == 1) apply_wave<1, false><<<grid, NT>>>(X[0], R[0], Y[1], B2[0], nvec, cv, scale, shift);
    else if (NS == 2) apply_wave<2, false><<<grid, NT>>>(X[0], R[0], Y[1], B2[0], nvec, cv, scale, shift);
    else apply_wave<4, false><<<grid, NT>>>(X[0], R[0], Y[1], B2[0], nvec, cv, scale, shift);
    CK(hipMemcpy(b0.data(), B[0], nvec, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b2.data(), B2[0], nvec, hipMemcpyDeviceToHost));
    std::vector<bf16_t> y0(n), y1(n);
    CK(hipMemcpy(y0.data(), Y[0], n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y1.data(), Y[1], n * 2, hipMemcpyDeviceToHost));
    printf("  mask equal: %s  y equal: %s\n", b0 == b2 ? "yes" : "NO", y0 == y1 ? "yes" : "NO");
    for (int s = 0; s < SETS; ++s) {
      CK(hipFree(X[s])); CK(hipFree(R[s])); CK(hipFree(Y[s])); CK(hipFree(B[s])); CK(hipFree(B2[s]));
    }
    CK(hipFree(scale));
    CK(hipFree(shift));
  }
  return 0;
}
