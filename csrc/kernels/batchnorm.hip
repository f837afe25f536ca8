// Training-mode BatchNorm over channels-last (NHWC) activations, with fused residual-add + ReLU
// (SURVEY §2.5 K05, K03).
//
// The reference's ResNet-50 (`NB03:314`, Bottleneck BN x53, `model.train()` at `NB03:381`) runs
// torch's BN followed by separate ReLU / add kernels.  Here every BN is viewed as an [M = N*H*W, C]
// matrix (C contiguous, a multiple of 8) and handled in two memory-bound passes per direction:
//   forward : stats  — per-channel shifted sums (x - K_c), (x - K_c)^2 with pivot K_c = x[0, c]
//                      (cancellation-safe when |mean| >> std), block-reduced in LDS, one fp32 atomic
//                      per channel per workgroup into a [2, C] accumulator (zeroed by a memset node);
//             apply  — every workgroup first turns the accumulator into per-channel scale/shift in
//                      LDS, then streams y = relu(x * scale + shift [+ residual]); workgroup 0 also
//                      writes the saved mean / invstd and the running statistics.
//   backward: reduce — sum(dz), sum(dz * (x - mean)) with dz = dy * [y > 0] recomputed from the
//                      saved output, same atomic scheme;
//             apply  — dx = A*dz + B*x + C per channel (coefficients built in LDS), dz also emitted
//                      for the residual branch; workgroup 0 writes dgamma / dbeta in the parameter dtype.
// No separate "finalize" launches: each direction is memset + 2 kernels.
// Each lane owns 8 consecutive channels (16-B loads); workgroups tile rows x channel groups.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxC = 2048;  // per-channel tables staged in LDS by the apply kernels

struct BnGeom {
  int cv;       // 8-channel vectors per row
  int cols;     // vector columns per block
  int rpi;      // rows per block iteration (threads stacked along rows)
  int gy;       // channel-group blocks
  int64_t rpb;  // rows per block
  int nrb;      // row blocks
};

BnGeom bn_geom(int64_t M, int64_t C) {
  BnGeom g;
  g.cv = (int)(C / 8);
  if (g.cv >= kThreads) {
    g.cols = kThreads;
    g.rpi = 1;
    g.gy = (g.cv + kThreads - 1) / kThreads;
  } else {
    g.cols = g.cv;
    g.rpi = kThreads / g.cv;
    g.gy = 1;
  }
  const int target = 1024 / g.gy > 0 ? 1024 / g.gy : 1;
  int64_t rpb = (M + target - 1) / target;
  const int64_t min_rpb = (int64_t)g.rpi * 8;
  if (rpb < min_rpb) rpb = min_rpb;
  g.rpb = rpb;
  g.nrb = (int)((M + rpb - 1) / rpb);
  return g;
}

inline int ew_grid(int64_t nvec) {
  int64_t g = (nvec + kThreads - 1) / kThreads;
  if (g > 2048) g = 2048;
  return g < 1 ? 1 : (int)g;
}

// Reduce per-thread 8-channel partials (a, b) over the `rpi` row-threads of a column, then one
// atomic per channel per block.
__device__ __forceinline__ void block_col_reduce_atomic(float (&a)[8], float (&b)[8], int tx, int ty, int cols,
                                                        int rpi, int vcol, int C, float* acc) {
  __shared__ float s_a[kThreads * 8];
  __shared__ float s_b[kThreads * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s_a[threadIdx.x * 8 + j] = a[j];
    s_b[threadIdx.x * 8 + j] = b[j];
  }
  __syncthreads();
  if (ty == 0 && vcol * 8 < C) {
    for (int k = 1; k < rpi; ++k) {
      const int t = k * cols + tx;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] += s_a[t * 8 + j];
        b[j] += s_b[t * 8 + j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(acc + vcol * 8 + j, a[j]);
      atomicAdd(acc + C + vcol * 8 + j, b[j]);
    }
  }
}

// ---------------------------------------------------------------- forward statistics
__global__ void __launch_bounds__(kThreads) bn_stats_kernel(const bf16_t* __restrict__ x, int64_t M, int C, int cols,
                                                            int rpi, int64_t rpb, float* __restrict__ acc) {
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(r0 + rpb, M);
  float s1[8], s2[8], piv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    load8(x + vcol * 8, piv);  // row 0 is the pivot
    for (int64_t r = r0 + ty; r < r1; r += rpi) {
      float v[8];
      load8(x + r * C + vcol * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - piv[j];
        s1[j] += d;
        s2[j] += d * d;
      }
    }
  }
  block_col_reduce_atomic(s1, s2, tx, ty, cols, rpi, vcol, C, acc);
}

__device__ __forceinline__ float param_at(const float* f, const bf16_t* b, int c, float dflt) {
  return f ? f[c] : (b ? bf2f(b[c]) : dflt);
}

// ---------------------------------------------------------------- forward apply (+ finalize)
template <bool RES, bool RELU, bool TRAIN>
__global__ void __launch_bounds__(kThreads) bn_apply_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, bf16_t* __restrict__ y, int64_t M, int C,
    const float* __restrict__ acc, const float* __restrict__ gamma_f, const bf16_t* __restrict__ gamma_b,
    const float* __restrict__ beta_f, const bf16_t* __restrict__ beta_b, float* __restrict__ running_mean,
    float* __restrict__ running_var, float momentum, float eps, float* __restrict__ save_mean,
    float* __restrict__ save_invstd) {
  __shared__ __attribute__((aligned(16))) float s_scale[kMaxC];
  __shared__ __attribute__((aligned(16))) float s_shift[kMaxC];
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, invstd;
    if (TRAIN) {
      const float piv = bf2f(x[c]);
      const float m1 = acc[c] * invM;
      const float var = fmaxf(acc[C + c] * invM - m1 * m1, 0.f);
      mean = piv + m1;
      invstd = rsqrtf(var + eps);
      if (blockIdx.x == 0) {
        save_mean[c] = mean;
        save_invstd[c] = invstd;
        if (running_mean) {
          running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
          const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
          running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
        }
      }
    } else {
      mean = running_mean[c];
      invstd = rsqrtf(running_var[c] + eps);
    }
    const float g = param_at(gamma_f, gamma_b, c, 1.f), b = param_at(beta_f, beta_b, c, 0.f);
    s_scale[c] = g * invstd;
    s_shift[c] = b - mean * g * invstd;
  }
  __syncthreads();
  const int cv = C / 8;
  const int64_t nvec = M * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % cv) * 8;
    float a[8];
    load8(x + v * 8, a);
    const f32x4 sc0 = *reinterpret_cast<const f32x4*>(s_scale + c0), sc1 = *reinterpret_cast<const f32x4*>(s_scale + c0 + 4);
    const f32x4 sh0 = *reinterpret_cast<const f32x4*>(s_shift + c0), sh1 = *reinterpret_cast<const f32x4*>(s_shift + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = a[j] * sc0[j] + sh0[j];
      a[j + 4] = a[j + 4] * sc1[j] + sh1[j];
    }
    if (RES) {
      float r[8];
      load8(res + v * 8, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += r[j];
    }
    if (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = fmaxf(a[j], 0.f);
    }
    store8(y + v * 8, a);
  }
}

// ---------------------------------------------------------------- backward reduction
template <bool RELU>
__global__ void __launch_bounds__(kThreads) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ x,
                                                                 const bf16_t* __restrict__ y,
                                                                 const float* __restrict__ mean, int64_t M, int C,
                                                                 int cols, int rpi, int64_t rpb,
                                                                 float* __restrict__ acc) {
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(r0 + rpb, M);
  float sa[8], sb[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.f;
  if (active) {
    load8(mean + vcol * 8, mu);
    for (int64_t r = r0 + ty; r < r1; r += rpi) {
      const int64_t off = r * C + vcol * 8;
      float g[8], xv[8];
      load8(dy + off, g);
      load8(x + off, xv);
      if (RELU) {
        u16x8 yr = *reinterpret_cast<const u16x8*>(y + off);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = bf2f(yr[j]) > 0.f ? g[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sa[j] += g[j];
        sb[j] += g[j] * (xv[j] - mu[j]);
      }
    }
  }
  block_col_reduce_atomic(sa, sb, tx, ty, cols, rpi, vcol, C, acc);
}

// dgamma = invstd * sum(dz (x-mean)), dbeta = sum(dz);  dx = A*dz + B*x + Cc
template <bool RELU, bool DRES>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y, int64_t M, int C,
    const float* __restrict__ acc, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma_f, const bf16_t* __restrict__ gamma_b, float* __restrict__ dgamma_f,
    bf16_t* __restrict__ dgamma_b, float* __restrict__ dbeta_f, bf16_t* __restrict__ dbeta_b, bf16_t* __restrict__ dx,
    bf16_t* __restrict__ dres) {
  __shared__ __attribute__((aligned(16))) float s_A[kMaxC];
  __shared__ __attribute__((aligned(16))) float s_B[kMaxC];
  __shared__ __attribute__((aligned(16))) float s_C[kMaxC];
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float sdz = acc[c], sdx = acc[C + c];
    const float is = invstd[c], mu = mean[c];
    const float g = param_at(gamma_f, gamma_b, c, 1.f);
    const float dg = sdx * is;
    if (blockIdx.x == 0) {
      if (dgamma_f) dgamma_f[c] = dg;
      if (dgamma_b) dgamma_b[c] = f2bf(dg);
      if (dbeta_f) dbeta_f[c] = sdz;
      if (dbeta_b) dbeta_b[c] = f2bf(sdz);
    }
    const float A = g * is;
    const float B = -A * is * dg * invM;
    s_A[c] = A;
    s_B[c] = B;
    s_C[c] = -A * sdz * invM - B * mu;
  }
  __syncthreads();
  const int cv = C / 8;
  const int64_t nvec = M * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % cv) * 8;
    float g[8], xv[8];
    load8(dy + v * 8, g);
    load8(x + v * 8, xv);
    if (RELU) {
      u16x8 yr = *reinterpret_cast<const u16x8*>(y + v * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = bf2f(yr[j]) > 0.f ? g[j] : 0.f;
    }
    if (DRES) store8(dres + v * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = s_A[c0 + j] * g[j] + s_B[c0 + j] * xv[j] + s_C[c0 + j];
    store8(dx + v * 8, xv);
  }
}

template <bool TRAIN>
hipError_t launch_apply(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int C, const float* acc,
                        const float* gf, const bf16_t* gb, const float* bfp, const bf16_t* bb, float* rm, float* rv,
                        float momentum, float eps, bool relu, float* save_mean, float* save_invstd, hipStream_t st) {
  const int grid = ew_grid(M * C / 8);
#define PDA_BN_APPLY(R, L)                                                                                    \
  bn_apply_kernel<R, L, TRAIN><<<grid, kThreads, 0, st>>>(x, res, y, M, C, acc, gf, gb, bfp, bb, rm, rv, momentum, \
                                                          eps, save_mean, save_invstd)
  if (res && relu) PDA_BN_APPLY(true, true);
  else if (res) PDA_BN_APPLY(true, false);
  else if (relu) PDA_BN_APPLY(false, true);
  else PDA_BN_APPLY(false, false);
#undef PDA_BN_APPLY
  return hipGetLastError();
}

}  // namespace

int64_t bn_workspace_floats(int64_t M, int64_t C) {
  (void)M;
  return 2 * C;
}

hipError_t bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                        const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, float* running_mean,
                        float* running_var, float momentum, float eps, bool relu, float* save_mean,
                        float* save_invstd, float* ws, hipStream_t st) {
  if (C > kMaxC || C % 8) return hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C);
  PDA_CHECK_HIP(hipMemsetAsync(ws, 0, 2 * C * sizeof(float), st));
  bn_stats_kernel<<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(x, M, (int)C, g.cols, g.rpi, g.rpb, ws);
  PDA_CHECK_HIP(hipGetLastError());
  return launch_apply<true>(x, res, y, M, (int)C, ws, gamma_f, gamma_b, beta_f, beta_b, running_mean, running_var,
                            momentum, eps, relu, save_mean, save_invstd, st);
}

hipError_t bn_fwd_eval(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                       const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, const float* running_mean,
                       const float* running_var, float eps, bool relu, float* ws, hipStream_t st) {
  if (C > kMaxC || C % 8) return hipErrorInvalidValue;
  (void)ws;
  return launch_apply<false>(x, res, y, M, (int)C, nullptr, gamma_f, gamma_b, beta_f, beta_b,
                             const_cast<float*>(running_mean), const_cast<float*>(running_var), 0.f, eps, relu,
                             nullptr, nullptr, st);
}

hipError_t bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, int64_t M, int64_t C, const float* save_mean,
                  const float* save_invstd, const float* gamma_f, const bf16_t* gamma_b, bool relu, bf16_t* dx,
                  bf16_t* dres, float* dgamma_f, bf16_t* dgamma_b, float* dbeta_f, bf16_t* dbeta_b, float* ws,
                  hipStream_t st) {
  if (C > kMaxC || C % 8) return hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C);
  PDA_CHECK_HIP(hipMemsetAsync(ws, 0, 2 * C * sizeof(float), st));
  if (relu)
    bn_bwd_reduce_kernel<true><<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(dy, x, y, save_mean, M, (int)C, g.cols, g.rpi,
                                                                       g.rpb, ws);
  else
    bn_bwd_reduce_kernel<false><<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(dy, x, y, save_mean, M, (int)C, g.cols,
                                                                        g.rpi, g.rpb, ws);
  PDA_CHECK_HIP(hipGetLastError());
  const int grid = ew_grid(M * C / 8);
#define PDA_BN_BWD(R, D)                                                                                          \
  bn_bwd_apply_kernel<R, D><<<grid, kThreads, 0, st>>>(dy, x, y, M, (int)C, ws, save_mean, save_invstd, gamma_f,   \
                                                       gamma_b, dgamma_f, dgamma_b, dbeta_f, dbeta_b, dx, dres)
  if (relu && dres) PDA_BN_BWD(true, true);
  else if (relu) PDA_BN_BWD(true, false);
  else if (dres) PDA_BN_BWD(false, true);
  else PDA_BN_BWD(false, false);
#undef PDA_BN_BWD
  return hipGetLastError();
}

}  // namespace pda
