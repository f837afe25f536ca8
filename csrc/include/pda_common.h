// Common device helpers for the pytorchdistributed_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors are passed as `uint16_t*` storage; conversion goes through the clang `__bf16`
//     type so hipcc emits `v_cvt_pk_bf16_f32` (round-to-nearest-even, NaN preserving).
//   * wavefronts are 64 lanes (hard-coded, never `warpSize`).
//   * global memory is touched 16 bytes per lane (8 x bf16 / 4 x f32) wherever shapes allow.
//   * launch functions never allocate or synchronise, so they are safe inside hipGraph capture.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PDA_WAVE 64

#define PDA_CHECK_HIP(expr)                                                                    \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return _e;                                                           \
  } while (0)

namespace pda {

typedef uint16_t bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __builtin_bit_cast(float, (uint32_t)v << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// Typed load/store helpers so templated kernels can serve fp32 and bf16 storage alike.
template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float load(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void store(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float load(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void store(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
};

// 8-element vector I/O (16 B for bf16, 32 B for fp32).
__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  u16x8 r = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(r[j]);
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
  *reinterpret_cast<u16x8*>(p) = r;
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  f32x4 a, b;
#pragma unroll
  for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[j + 4]; }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` must hold >= 16 floats. Result on every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, scratch[i]);
  return t;
}

// Bijective XCD-aware remap of a 1-D workgroup id (guide §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD so their shared operand panels hit one L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd, xcd = orig % nxcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / nxcd;
}

// Grouped tile order: consecutive tile ids walk GM rows of tiles before moving one column right, so
// the workgroups in flight on one XCD (consecutive ids after xcd_remap) share GM A-panels and a few
// B-panels instead of one A-panel and a whole row of B-panels (L2 / MALL traffic on wide GEMMs).
__device__ __forceinline__ void grouped_tile(int tile, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per_group = gm * tiles_n;
  const int g = tile / per_group, first = g * gm;
  const int rows = min(tiles_m - first, gm);
  const int r = tile - g * per_group;
  tm = first + r % rows;
  tn = r / rows;
}

// GELU (tanh approximation, GPT-2's gelu_new) and its derivative: shared by the elementwise kernels
// (act.hip) and the GEMM epilogues that fuse them (gemm_conv.hip, act = 1 / 2).  Written with the
// identity 0.5 (1 + tanh(u)) = sigmoid(2u) on the bare v_exp_f32 + v_rcp_f32: a few VALU ops per
// element instead of tanhf's libcall, which a GEMM epilogue (one 512-thread workgroup per CU, 128
// elements per lane) cannot hide.
__device__ __forceinline__ float gelu_sig2u(float x, float& du) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u2 = 2.f * k0 * fmaf(k1 * x2, x, x);                 // 2u
  const float s = __frcp_rn(1.f + __builtin_amdgcn_exp2f(-u2 * 1.4426950408889634f));  // sigmoid(2u)
  du = 2.f * k0 * fmaf(3.f * k1, x2, 1.f);                         // d(2u)/dx
  return s;
}
__device__ __forceinline__ float gelu_tanh(float x) {
  float du;
  return x * gelu_sig2u(x, du);
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  float du;
  const float s = gelu_sig2u(x, du);
  return fmaf(x * s * (1.f - s), du, s);
}

}  // namespace pda
