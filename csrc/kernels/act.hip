// Elementwise activations (SURVEY §2.5 K03 ReLU, K21 GELU(tanh) / SwiGLU) for fp32 or bf16 tensors.
// Memory-bound: 16-B vector accesses per lane, grid-stride, tail handled element-wise.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;

inline int grid_for(int64_t n8) {
  int64_t g = (n8 + kThreads - 1) / kThreads;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// op: 0 relu, 1 gelu_tanh
template <typename T>
__global__ void __launch_bounds__(kThreads) act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int op) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; b < n; b += stride) {
    if (b + 8 <= n) {
      float v[8];
      load8(x + b, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = op == 0 ? fmaxf(v[j], 0.f) : gelu_tanh(v[j]);
      store8(y + b, v);
    } else {
      for (int64_t i = b; i < n; ++i) {
        const float v = Elem<T>::load(x, i);
        Elem<T>::store(y, i, op == 0 ? fmaxf(v, 0.f) : gelu_tanh(v));
      }
    }
  }
}

// relu: dx = dy * (ref > 0) with ref = output;  gelu: dx = dy * gelu'(ref) with ref = input
template <typename T>
__global__ void __launch_bounds__(kThreads) act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ ref,
                                                           T* __restrict__ dx, int64_t n, int op) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; b < n; b += stride) {
    if (b + 8 <= n) {
      float g[8], r[8];
      load8(dy + b, g);
      load8(ref + b, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = op == 0 ? (r[j] > 0.f ? g[j] : 0.f) : g[j] * gelu_tanh_grad(r[j]);
      store8(dx + b, g);
    } else {
      for (int64_t i = b; i < n; ++i) {
        const float g = Elem<T>::load(dy, i), r = Elem<T>::load(ref, i);
        Elem<T>::store(dx, i, op == 0 ? (r > 0.f ? g : 0.f) : g * gelu_tanh_grad(r));
      }
    }
  }
}

// SwiGLU over a fused [rows, 2F] gate|up tensor: y[r, f] = silu(gu[r, f]) * gu[r, F + f]
template <typename T>
__global__ void __launch_bounds__(kThreads) swiglu_fwd_kernel(const T* __restrict__ gu, T* __restrict__ y, int64_t rows,
                                                              int64_t F) {
  const int64_t nv = rows * F / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t r = (v * 8) / F, f = (v * 8) % F;
    float g[8], u[8];
    load8(gu + r * 2 * F + f, g);
    load8(gu + r * 2 * F + F + f, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = silu(g[j]) * u[j];
    store8(y + v * 8, g);
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) swiglu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ gu,
                                                              T* __restrict__ dgu, int64_t rows, int64_t F) {
  const int64_t nv = rows * F / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t r = (v * 8) / F, f = (v * 8) % F;
    float d[8], g[8], u[8], dg[8], du[8];
    load8(dy + v * 8, d);
    load8(gu + r * 2 * F + f, g);
    load8(gu + r * 2 * F + F + f, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = 1.f / (1.f + __expf(-g[j]));
      const float sl = g[j] * s;
      du[j] = d[j] * sl;
      dg[j] = d[j] * u[j] * (s + sl * (1.f - s));
    }
    store8(dgu + r * 2 * F + f, dg);
    store8(dgu + r * 2 * F + F + f, du);
  }
}

// Column sums of a [rows, cols] matrix with any column count (classifier bias gradients):
// out[c] = sum_r x[r, c] (fp32).  A block owns 32 columns; its 8 row lanes stride over all rows and
// are combined through LDS, so the result is deterministic and needs no pre-zeroed output (no memset
// node when the step is captured into a HIP graph).
constexpr int kCsCols = 32, kCsLanes = kThreads / kCsCols;
template <typename T>
__global__ void __launch_bounds__(kThreads) colsum_kernel(const T* __restrict__ x, float* __restrict__ out, int64_t rows,
                                                          int64_t cols) {
  __shared__ float part[kCsLanes][kCsCols];
  const int cl = threadIdx.x % kCsCols, rl = threadIdx.x / kCsCols;
  const int64_t c = (int64_t)blockIdx.x * kCsCols + cl;
  float acc = 0.f;
  if (c < cols)
    for (int64_t r = rl; r < rows; r += kCsLanes) acc += Elem<T>::load(x, r * cols + c);
  part[rl][cl] = acc;
  __syncthreads();
  if (rl == 0 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kCsLanes; ++i) s += part[i][cl];
    out[c] = s;
  }
}

}  // namespace

hipError_t act_fwd(const void* x, void* y, bool bf16, int64_t n, int op, hipStream_t st) {
  const int g = grid_for((n + 7) / 8);
  if (bf16) act_fwd_kernel<bf16_t><<<g, kThreads, 0, st>>>((const bf16_t*)x, (bf16_t*)y, n, op);
  else act_fwd_kernel<float><<<g, kThreads, 0, st>>>((const float*)x, (float*)y, n, op);
  return hipGetLastError();
}

hipError_t act_bwd(const void* dy, const void* ref, void* dx, bool bf16, int64_t n, int op, hipStream_t st) {
  const int g = grid_for((n + 7) / 8);
  if (bf16) act_bwd_kernel<bf16_t><<<g, kThreads, 0, st>>>((const bf16_t*)dy, (const bf16_t*)ref, (bf16_t*)dx, n, op);
  else act_bwd_kernel<float><<<g, kThreads, 0, st>>>((const float*)dy, (const float*)ref, (float*)dx, n, op);
  return hipGetLastError();
}

hipError_t swiglu_fwd(const void* gu, void* y, bool bf16, int64_t rows, int64_t F, hipStream_t st) {
  const int g = grid_for(rows * F / 8);
  if (bf16) swiglu_fwd_kernel<bf16_t><<<g, kThreads, 0, st>>>((const bf16_t*)gu, (bf16_t*)y, rows, F);
  else swiglu_fwd_kernel<float><<<g, kThreads, 0, st>>>((const float*)gu, (float*)y, rows, F);
  return hipGetLastError();
}

hipError_t swiglu_bwd(const void* dy, const void* gu, void* dgu, bool bf16, int64_t rows, int64_t F, hipStream_t st) {
  const int g = grid_for(rows * F / 8);
  if (bf16)
    swiglu_bwd_kernel<bf16_t><<<g, kThreads, 0, st>>>((const bf16_t*)dy, (const bf16_t*)gu, (bf16_t*)dgu, rows, F);
  else
    swiglu_bwd_kernel<float><<<g, kThreads, 0, st>>>((const float*)dy, (const float*)gu, (float*)dgu, rows, F);
  return hipGetLastError();
}

hipError_t colsum_unaligned(const void* x, bool bf16, float* out, int64_t rows, int64_t cols, hipStream_t st) {
  const unsigned grid = (unsigned)((cols + kCsCols - 1) / kCsCols);
  if (bf16) colsum_kernel<bf16_t><<<grid, kThreads, 0, st>>>((const bf16_t*)x, out, rows, cols);
  else colsum_kernel<float><<<grid, kThreads, 0, st>>>((const float*)x, out, rows, cols);
  return hipGetLastError();
}

}  // namespace pda
