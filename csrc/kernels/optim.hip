// Fused optimizer kernels over FLAT parameter / gradient buffers.
//
// The reference calls torch's foreach SGD / Adam (`PY1:42` optim.SGD(lr=1e-3), `NB03:383,391`
// optim.Adam(lr=1e-3)).  Here the whole model is ONE launch: parameters live in a contiguous fp32
// master buffer, gradients are the DDP bucket buffers themselves (bf16 or fp32, gradient-as-bucket
// view), and the kernel also writes the bf16 working copy the model computes with.  The
// gradient scale (1/world_size for the DDP average, times a clip coefficient) is read from device
// memory so the step can be replayed inside a hipGraph without host synchronisation.
//
// Memory-bound: each element is read/written once, 16 B per lane.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;

inline int grid_for(int64_t n_vec) {
  int64_t g = (n_vec + kThreads - 1) / kThreads;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

__device__ __forceinline__ float read_scale(const float* scale_ptr, float scale) {
  return scale_ptr ? scale * scale_ptr[0] : scale;
}

template <typename G>
__global__ void __launch_bounds__(kThreads) sgd_kernel(float* __restrict__ master, bf16_t* __restrict__ param_bf16,
                                                       const G* __restrict__ grad, float* __restrict__ mom, int64_t n,
                                                       float lr, float momentum, float dampening, float wd,
                                                       int nesterov, int first, float gscale,
                                                       const float* __restrict__ gscale_ptr,
                                                       const float* __restrict__ lr_ptr) {
  const float s = read_scale(gscale_ptr, gscale);
  const float lr_ = lr_ptr ? lr_ptr[0] : lr;
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv + (n % 8 ? 1 : 0); v += stride) {
    const int64_t base = v * 8;
    if (base + 8 <= n) {
      float p[8], g[8], b[8];
      load8(master + base, p);
      load8(grad + base, g);
      if (momentum != 0.f && !first) load8(mom + base, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float gj = g[j] * s + wd * p[j];
        if (momentum != 0.f) {
          b[j] = first ? gj : momentum * b[j] + (1.f - dampening) * gj;
          gj = nesterov ? gj + momentum * b[j] : b[j];
        }
        p[j] -= lr_ * gj;
      }
      store8(master + base, p);
      if (momentum != 0.f) store8(mom + base, b);
      if (param_bf16) store8(param_bf16 + base, p);
    } else {
      for (int64_t i = base; i < n; ++i) {
        float p = master[i];
        float gj = Elem<G>::load(grad, i) * s + wd * p;
        if (momentum != 0.f) {
          float b = first ? gj : momentum * mom[i] + (1.f - dampening) * gj;
          mom[i] = b;
          gj = nesterov ? gj + momentum * b : b;
        }
        p -= lr_ * gj;
        master[i] = p;
        if (param_bf16) param_bf16[i] = f2bf(p);
      }
    }
  }
}

template <typename G>
__global__ void __launch_bounds__(kThreads) adam_kernel(float* __restrict__ master, bf16_t* __restrict__ param_bf16,
                                                        const G* __restrict__ grad, float* __restrict__ m_,
                                                        float* __restrict__ v_, int64_t n, float lr, float beta1,
                                                        float beta2, float eps, float wd, int adamw, float bc1,
                                                        float bc2_sqrt, float gscale,
                                                        const float* __restrict__ gscale_ptr,
                                                        const float* __restrict__ lr_ptr,
                                                        const float* __restrict__ step_ptr) {
  const float s = read_scale(gscale_ptr, gscale);
  const float lr_ = lr_ptr ? lr_ptr[0] : lr;
  if (step_ptr) {  // step count on the device: the launch can be replayed from a HIP graph
    const float t = step_ptr[0];
    bc1 = 1.f - powf(beta1, t);
    bc2_sqrt = sqrtf(1.f - powf(beta2, t));
  }
  const float step_size = lr_ / bc1;
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv + (n % 8 ? 1 : 0); v += stride) {
    const int64_t base = v * 8;
    const int cnt = (base + 8 <= n) ? 8 : (int)(n - base);
    float p[8], g[8], m[8], vv[8];
    if (cnt == 8) {
      load8(master + base, p);
      load8(grad + base, g);
      load8(m_ + base, m);
      load8(v_ + base, vv);
    } else {
      for (int j = 0; j < cnt; ++j) {
        p[j] = master[base + j];
        g[j] = Elem<G>::load(grad, base + j);
        m[j] = m_[base + j];
        vv[j] = v_[base + j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gj = g[j] * s;
      if (adamw) p[j] *= (1.f - lr_ * wd);
      else gj += wd * p[j];
      m[j] = beta1 * m[j] + (1.f - beta1) * gj;
      vv[j] = beta2 * vv[j] + (1.f - beta2) * gj * gj;
      const float denom = sqrtf(vv[j]) / bc2_sqrt + eps;
      p[j] -= step_size * m[j] / denom;
    }
    if (cnt == 8) {
      store8(master + base, p);
      store8(m_ + base, m);
      store8(v_ + base, vv);
      if (param_bf16) store8(param_bf16 + base, p);
    } else {
      for (int j = 0; j < cnt; ++j) {
        master[base + j] = p[j];
        m_[base + j] = m[j];
        v_[base + j] = vv[j];
        if (param_bf16) param_bf16[base + j] = f2bf(p[j]);
      }
    }
  }
}

// Sum of squares, stage 1: one partial per block.
template <typename G>
__global__ void __launch_bounds__(kThreads) sumsq_partial_kernel(const G* __restrict__ x, int64_t n,
                                                                 float* __restrict__ partial) {
  __shared__ float scratch[16];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; base < n; base += stride) {
    if (base + 8 <= n) {
      float v[8];
      load8(x + base, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
    } else {
      for (int64_t i = base; i < n; ++i) {
        float t = Elem<G>::load(x, i);
        acc += t * t;
      }
    }
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Stage 2: total norm and clip coefficient; out[0] = ||g||, out[1] = min(1, max_norm/(||g||*pre+1e-6)).
// `pre` is the gradient pre-scale (e.g. 1/world_size) so the clip is taken on the averaged gradient.
__global__ void __launch_bounds__(1024) norm_finalize_kernel(const float* __restrict__ partial, int np, float pre,
                                                             float max_norm, float* __restrict__ out) {
  __shared__ float scratch[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(acc) * pre;
    out[0] = norm;
    out[1] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
  }
}

template <typename S, typename D>
__global__ void __launch_bounds__(kThreads) cast_scale_kernel(const S* __restrict__ src, D* __restrict__ dst, int64_t n,
                                                              float scale, const float* __restrict__ scale_ptr) {
  const float s = read_scale(scale_ptr, scale);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; base < n; base += stride) {
    if (base + 8 <= n) {
      float v[8];
      load8(src + base, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= s;
      store8(dst + base, v);
    } else {
      for (int64_t i = base; i < n; ++i) Elem<D>::store(dst, i, Elem<S>::load(src, i) * s);
    }
  }
}

}  // namespace

hipError_t sgd_step(float* master, bf16_t* param_bf16, const void* grad, bool grad_bf16, float* mom, int64_t n,
                    float lr, float momentum, float dampening, float wd, bool nesterov, bool first, float gscale,
                    const float* gscale_ptr, const float* lr_ptr, hipStream_t st) {
  const int g = grid_for((n + 7) / 8);
  if (grad_bf16)
    sgd_kernel<bf16_t><<<g, kThreads, 0, st>>>(master, param_bf16, (const bf16_t*)grad, mom, n, lr, momentum,
                                               dampening, wd, nesterov, first, gscale, gscale_ptr, lr_ptr);
  else
    sgd_kernel<float><<<g, kThreads, 0, st>>>(master, param_bf16, (const float*)grad, mom, n, lr, momentum,
                                              dampening, wd, nesterov, first, gscale, gscale_ptr, lr_ptr);
  return hipGetLastError();
}

hipError_t adam_step(float* master, bf16_t* param_bf16, const void* grad, bool grad_bf16, float* m, float* v,
                     int64_t n, float lr, float beta1, float beta2, float eps, float wd, bool adamw, int64_t step,
                     float gscale, const float* gscale_ptr, const float* lr_ptr, const float* step_ptr,
                     hipStream_t st) {
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2_sqrt = sqrtf(1.f - powf(beta2, (float)step));
  const int g = grid_for((n + 7) / 8);
  if (grad_bf16)
    adam_kernel<bf16_t><<<g, kThreads, 0, st>>>(master, param_bf16, (const bf16_t*)grad, m, v, n, lr, beta1, beta2,
                                                eps, wd, adamw, bc1, bc2_sqrt, gscale, gscale_ptr, lr_ptr, step_ptr);
  else
    adam_kernel<float><<<g, kThreads, 0, st>>>(master, param_bf16, (const float*)grad, m, v, n, lr, beta1, beta2,
                                               eps, wd, adamw, bc1, bc2_sqrt, gscale, gscale_ptr, lr_ptr, step_ptr);
  return hipGetLastError();
}

int grad_norm_partials() { return 1024; }

hipError_t grad_norm(const void* grad, bool grad_bf16, int64_t n, float pre, float max_norm, float* partial,
                     float* out, hipStream_t st) {
  const int np = grad_norm_partials();
  if (grad_bf16)
    sumsq_partial_kernel<bf16_t><<<np, kThreads, 0, st>>>((const bf16_t*)grad, n, partial);
  else
    sumsq_partial_kernel<float><<<np, kThreads, 0, st>>>((const float*)grad, n, partial);
  norm_finalize_kernel<<<1, 1024, 0, st>>>(partial, np, pre, max_norm, out);
  return hipGetLastError();
}

hipError_t cast_scale(const void* src, bool src_bf16, void* dst, bool dst_bf16, int64_t n, float scale,
                      const float* scale_ptr, hipStream_t st) {
  const int g = grid_for((n + 7) / 8);
  if (src_bf16 && dst_bf16)
    cast_scale_kernel<bf16_t, bf16_t><<<g, kThreads, 0, st>>>((const bf16_t*)src, (bf16_t*)dst, n, scale, scale_ptr);
  else if (src_bf16)
    cast_scale_kernel<bf16_t, float><<<g, kThreads, 0, st>>>((const bf16_t*)src, (float*)dst, n, scale, scale_ptr);
  else if (dst_bf16)
    cast_scale_kernel<float, bf16_t><<<g, kThreads, 0, st>>>((const float*)src, (bf16_t*)dst, n, scale, scale_ptr);
  else
    cast_scale_kernel<float, float><<<g, kThreads, 0, st>>>((const float*)src, (float*)dst, n, scale, scale_ptr);
  return hipGetLastError();
}

}  // namespace pda
