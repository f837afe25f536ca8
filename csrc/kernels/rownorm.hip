// Row normalisations for the transformer configs (SURVEY §2.5 K19 LayerNorm — GPT-2, K20 RMSNorm —
// Llama-3).  x: [rows, D] (fp32 or bf16, D % 8 == 0, D <= 8192), gamma/beta: [D].
// One 256-thread workgroup per row (ROWS_PER_BLOCK rows in sequence for the backward so the
// gamma/beta gradient is accumulated in registers and flushed with one fp32 atomic per column per
// workgroup).  The row lives in registers between the statistics and the normalisation (one HBM read).
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxV = 4;  // 8-element vectors per thread: D <= 256*8*4 = 8192
constexpr int kBwdRows = 8;

template <typename T, typename P, bool RMS>
__global__ void __launch_bounds__(kThreads) rownorm_fwd_kernel(const T* __restrict__ x, const P* __restrict__ gamma,
                                                               const P* __restrict__ beta, T* __restrict__ y,
                                                               float* __restrict__ mean_out,
                                                               float* __restrict__ rstd_out, int64_t D, float eps) {
  __shared__ float scratch[16];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * D;
  float v[kMaxV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxV; ++i) {
    const int64_t c = ((int64_t)i * kThreads + threadIdx.x) * 8;
    if (c < D) {
      load8(xr + c, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  float mean = 0.f;
  if (!RMS) mean = block_sum(s, scratch) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxV; ++i) {
    const int64_t c = ((int64_t)i * kThreads + threadIdx.x) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(block_sum(q, scratch) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < kMaxV; ++i) {
    const int64_t c = ((int64_t)i * kThreads + threadIdx.x) * 8;
    if (c < D) {
      float g[8], b[8], o[8];
      load8(gamma + c, g);
      if (!RMS) load8(beta + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + (RMS ? 0.f : b[j]);
      store8(y + row * D + c, o);
    }
  }
  if (threadIdx.x == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat))        (LayerNorm)
// dx = rstd * (g*dy - xhat * mean(g*dy*xhat))                      (RMSNorm)
template <typename T, typename P, bool RMS>
__global__ void __launch_bounds__(kThreads) rownorm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const P* __restrict__ gamma,
                                                               const float* __restrict__ mean_in,
                                                               const float* __restrict__ rstd_in,
                                                               T* __restrict__ dx, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta, int64_t rows, int64_t D) {
  __shared__ float scratch[16];
  float dg[kMaxV][8], db[kMaxV][8];
#pragma unroll
  for (int i = 0; i < kMaxV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[i][j] = db[i][j] = 0.f;
  for (int rr = 0; rr < kBwdRows; ++rr) {
    const int64_t row = (int64_t)blockIdx.x * kBwdRows + rr;
    if (row >= rows) break;
    const float mean = RMS ? 0.f : mean_in[row], rstd = rstd_in[row];
    float xh[kMaxV][8], gd[kMaxV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < kMaxV; ++i) {
      const int64_t c = ((int64_t)i * kThreads + threadIdx.x) * 8;
      if (c < D) {
        float xv[8], d[8], g[8];
        load8(x + row * D + c, xv);
        load8(dy + row * D + c, d);
        load8(gamma + c, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = (xv[j] - mean) * rstd;
          gd[i][j] = g[j] * d[j];
          s1 += gd[i][j];
          s2 += gd[i][j] * xh[i][j];
          dg[i][j] += d[j] * xh[i][j];
          db[i][j] += d[j];
        }
      }
    }
    const float m1 = RMS ? 0.f : block_sum(s1, scratch) / (float)D;
    const float m2 = block_sum(s2, scratch) / (float)D;
#pragma unroll
    for (int i = 0; i < kMaxV; ++i) {
      const int64_t c = ((int64_t)i * kThreads + threadIdx.x) * 8;
      if (c < D) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (gd[i][j] - m1 - xh[i][j] * m2);
        store8(dx + row * D + c, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kMaxV; ++i) {
    const int64_t c = ((int64_t)i * kThreads + threadIdx.x) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(dgamma + c + j, dg[i][j]);
        if (!RMS) atomicAdd(dbeta + c + j, db[i][j]);
      }
    }
  }
}

}  // namespace

hipError_t rownorm_fwd(const void* x, bool x_bf16, const void* gamma, const void* beta, bool p_bf16, void* y,
                       float* mean, float* rstd, int64_t rows, int64_t D, float eps, bool rms, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  const unsigned grid = (unsigned)rows;
#define ARGS_F(T, P) (const T*)x, (const P*)gamma, (const P*)beta, (T*)y, mean, rstd, D, eps
  if (rms) {
    if (x_bf16 && p_bf16) rownorm_fwd_kernel<bf16_t, bf16_t, true><<<grid, kThreads, 0, st>>>(ARGS_F(bf16_t, bf16_t));
    else if (x_bf16) rownorm_fwd_kernel<bf16_t, float, true><<<grid, kThreads, 0, st>>>(ARGS_F(bf16_t, float));
    else if (p_bf16) rownorm_fwd_kernel<float, bf16_t, true><<<grid, kThreads, 0, st>>>(ARGS_F(float, bf16_t));
    else rownorm_fwd_kernel<float, float, true><<<grid, kThreads, 0, st>>>(ARGS_F(float, float));
  } else {
    if (x_bf16 && p_bf16) rownorm_fwd_kernel<bf16_t, bf16_t, false><<<grid, kThreads, 0, st>>>(ARGS_F(bf16_t, bf16_t));
    else if (x_bf16) rownorm_fwd_kernel<bf16_t, float, false><<<grid, kThreads, 0, st>>>(ARGS_F(bf16_t, float));
    else if (p_bf16) rownorm_fwd_kernel<float, bf16_t, false><<<grid, kThreads, 0, st>>>(ARGS_F(float, bf16_t));
    else rownorm_fwd_kernel<float, float, false><<<grid, kThreads, 0, st>>>(ARGS_F(float, float));
  }
#undef ARGS_F
  return hipGetLastError();
}

hipError_t rownorm_bwd(const void* dy, const void* x, bool x_bf16, const void* gamma, bool p_bf16, const float* mean,
                       const float* rstd, void* dx, float* dgamma, float* dbeta, int64_t rows, int64_t D, bool rms,
                       hipStream_t st) {
  if (rows == 0) return hipSuccess;
  PDA_CHECK_HIP(hipMemsetAsync(dgamma, 0, D * sizeof(float), st));
  if (!rms) PDA_CHECK_HIP(hipMemsetAsync(dbeta, 0, D * sizeof(float), st));
  const unsigned grid = (unsigned)((rows + kBwdRows - 1) / kBwdRows);
#define ARGS_B(T, P) (const T*)dy, (const T*)x, (const P*)gamma, mean, rstd, (T*)dx, dgamma, dbeta, rows, D
  if (rms) {
    if (x_bf16 && p_bf16) rownorm_bwd_kernel<bf16_t, bf16_t, true><<<grid, kThreads, 0, st>>>(ARGS_B(bf16_t, bf16_t));
    else if (x_bf16) rownorm_bwd_kernel<bf16_t, float, true><<<grid, kThreads, 0, st>>>(ARGS_B(bf16_t, float));
    else if (p_bf16) rownorm_bwd_kernel<float, bf16_t, true><<<grid, kThreads, 0, st>>>(ARGS_B(float, bf16_t));
    else rownorm_bwd_kernel<float, float, true><<<grid, kThreads, 0, st>>>(ARGS_B(float, float));
  } else {
    if (x_bf16 && p_bf16) rownorm_bwd_kernel<bf16_t, bf16_t, false><<<grid, kThreads, 0, st>>>(ARGS_B(bf16_t, bf16_t));
    else if (x_bf16) rownorm_bwd_kernel<bf16_t, float, false><<<grid, kThreads, 0, st>>>(ARGS_B(bf16_t, float));
    else if (p_bf16) rownorm_bwd_kernel<float, bf16_t, false><<<grid, kThreads, 0, st>>>(ARGS_B(float, bf16_t));
    else rownorm_bwd_kernel<float, float, false><<<grid, kThreads, 0, st>>>(ARGS_B(float, float));
  }
#undef ARGS_B
  return hipGetLastError();
}

}  // namespace pda
