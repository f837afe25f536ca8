// fp32 training path for the reference's own workloads (NB03 trains ResNet-50 in fp32 on A100,
// `03 模型并行/03_model_parallel.ipynb` raw lines 369-391 / 314 / 417; cuDNN runs those convs in TF32).
//
// gfx950 has no xf32 MFMA and its f32-input MFMA runs at 1/16 of the bf16 rate, so fp32 GEMM-shaped
// work here is a split-bf16 product on the bf16 MFMA path:
//     x = x_hi + x_lo,  x_hi = bf16(x),  x_lo = bf16(x - x_hi)       (16 significant bits of x)
//     x . w ~= x_hi.w_hi + x_hi.w_lo + x_lo.w_hi  (+ x_lo.w_lo with 4 segments)
// accumulated in fp32 by one MFMA GEMM over a K dimension three (four) times longer: the split
// segments are laid out along the GEMM's K so the existing conv / GEMM kernels run unchanged —
//   conv fwd:    x -> [.., 3C] (hi, hi, lo) channels,    w -> [Co, R, S, 3C] (hi, lo, hi)
//   conv dgrad:  dy -> [.., 3Co] (hi, hi, lo) channels,  w -> [3Co, R, S, C] stacked (hi, lo, hi)
//   conv wgrad:  dy -> [3N, ..] stacked (hi, lo, hi),    x -> [3N, ..] stacked (hi, hi, lo)
// hi + lo carries 16 significant bits: ~1e-5 relative per GEMM (TF32 keeps 11 bits: ~5e-4); a 4th
// product (lo.lo) does not lower that representation floor.
//
// Plus the fp32 elementwise / reduction kernels the fp32 ResNet needs: BatchNorm2d (training batch
// statistics in two passes with shifted sums and a double-precision finalize, fused residual add +
// ReLU; backward reduce + apply), maxpool 3x3/2 and global average pool, all NHWC.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kT = 256;

inline int grid_for(int64_t n, int64_t per_thread = 1) {
  int64_t g = (n / per_thread + kT - 1) / kT;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

// ------------------------------------------------------------------ hi / lo split
// out[row * row_stride + seg * seg_stride + c] = seg's part of x[row * C + c] (bit seg of lo_mask set:
// the lo part).  Four floats per thread (C % 4 == 0).
__global__ void __launch_bounds__(kT) split_kernel(const float* __restrict__ x, bf16_t* __restrict__ out, int64_t rows,
                                                   int64_t C, int nseg, int lo_mask, int64_t seg_stride,
                                                   int64_t row_stride) {
  const int64_t cq = C / 4, total = rows * cq;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t row = t / cq, c = (t - row * cq) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + row * C + c);
    u16x4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hi[j] = f2bf(v[j]);
      lo[j] = f2bf(v[j] - bf2f(hi[j]));
    }
    bf16_t* o = out + row * row_stride + c;
    for (int s = 0; s < nseg; ++s) *reinterpret_cast<u16x4*>(o + s * seg_stride) = ((lo_mask >> s) & 1) ? lo : hi;
  }
}

// ------------------------------------------------------------------ BatchNorm (fp32, NHWC [M, C])
// Partial shifted sums: grid (gx, gy); a block covers qpb channel quads x rpb row lanes; writes
// part[bx][0][c] = sum(x - shift), part[bx][1][c] = sum((x - shift)^2) over its rows.
// bwd flavour (BWD): sums of g and g * (x - mean), g = dy masked by relu(y) when y is given.
template <bool BWD>
__global__ void __launch_bounds__(kT) bn_reduce_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                       const float* __restrict__ y, const float* __restrict__ shift,
                                                       float* __restrict__ part, int64_t M, int C, int qpb) {
  __shared__ f32x4 red[2][kT];
  const int cq = C / 4, rpb = kT / qpb;
  const int lq = threadIdx.x % qpb, lr = threadIdx.x / qpb;
  const int q = blockIdx.y * qpb + lq;
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  if (q < cq && lr < rpb) {
    const f32x4 k = *reinterpret_cast<const f32x4*>(shift + 4 * q);
    for (int64_t r = (int64_t)blockIdx.x * rpb + lr; r < M; r += (int64_t)gridDim.x * rpb) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * C + 4 * q) - k;
      if constexpr (BWD) {
        f32x4 g = *reinterpret_cast<const f32x4*>(dy + r * C + 4 * q);
        if (y) {
          const f32x4 yy = *reinterpret_cast<const f32x4*>(y + r * C + 4 * q);
#pragma unroll
          for (int j = 0; j < 4; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
        }
        s1 += g;
        s2 += g * v;
      } else {
        s1 += v;
        s2 += v * v;
      }
    }
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (lr == 0 && q < cq) {
    for (int i = 1; i < rpb; ++i) {
      s1 += red[0][i * qpb + lq];
      s2 += red[1][i * qpb + lq];
    }
    *reinterpret_cast<f32x4*>(part + (int64_t)blockIdx.x * 2 * C + 4 * q) = s1;
    *reinterpret_cast<f32x4*>(part + (int64_t)blockIdx.x * 2 * C + C + 4 * q) = s2;
  }
}

// Forward finalize (one thread per channel, double-precision sum of the partials): batch mean /
// biased variance, running statistics (unbiased variance, momentum), saved mean / invstd and the
// apply coefficients ss[c] = gamma * invstd, ss[C + c] = beta - mean * gamma * invstd.
__global__ void __launch_bounds__(kT) bn_fwd_finalize_kernel(const float* __restrict__ part, int G, int64_t M, int C,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* running_mean,
                                                             float* running_var, float momentum, float eps,
                                                             float* __restrict__ save_mean,
                                                             float* __restrict__ save_invstd, float* __restrict__ ss,
                                                             int64_t* num_batches) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && num_batches) *num_batches += 1;
  if (c >= C) return;
  double a = 0.0, b = 0.0;
  for (int g = 0; g < G; ++g) {
    a += part[(int64_t)g * 2 * C + c];
    b += part[(int64_t)g * 2 * C + C + c];
  }
  const double dm = a / (double)M;
  double var = b / (double)M - dm * dm;
  if (var < 0.0) var = 0.0;
  const float mean = (float)(shift[c] + dm);
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) {
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
  save_mean[c] = mean;
  save_invstd[c] = invstd;
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  ss[c] = g * invstd;
  ss[C + c] = bt - mean * g * invstd;
}

// y = x * ss[c] + ss[C + c] (+ res) (relu)
__global__ void __launch_bounds__(kT) bn_apply_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                      const float* __restrict__ ss, float* __restrict__ y, int64_t M,
                                                      int C, int relu) {
  const int cq = C / 4;
  const int64_t total = M * cq, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % cq) * 4;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(ss + c);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(ss + C + c);
    f32x4 v = *reinterpret_cast<const f32x4*>(x + t * 4) * sc + sh;
    if (res) v += *reinterpret_cast<const f32x4*>(res + t * 4);
    if (relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    *reinterpret_cast<f32x4*>(y + t * 4) = v;
  }
}

// Backward finalize: dgamma = sum(g (x - mean)) invstd, dbeta = sum(g); apply coefficients
// co[c] = gamma invstd, co[C + c] = -gamma invstd dbeta / M, co[2C + c] = -gamma invstd^3 sum(g(x-mean)) / M.
__global__ void __launch_bounds__(kT) bn_bwd_finalize_kernel(const float* __restrict__ part, int G, int64_t M, int C,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             float* __restrict__ co) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sg = 0.0, sgx = 0.0;
  for (int g = 0; g < G; ++g) {
    sg += part[(int64_t)g * 2 * C + c];
    sgx += part[(int64_t)g * 2 * C + C + c];
  }
  const float is = invstd[c], ga = gamma ? gamma[c] : 1.f;
  if (dgamma) dgamma[c] = (float)(sgx * is);
  if (dbeta) dbeta[c] = (float)sg;
  const float a = ga * is;
  co[c] = a;
  co[C + c] = (float)(-(double)a * sg / (double)M);
  co[2 * C + c] = (float)(-(double)a * is * is * sgx / (double)M);
}

// dx = co0 * g + co1 + co2 * (x - mean); g = dy masked by relu(y); optionally also writes g (the
// residual branch's gradient).
__global__ void __launch_bounds__(kT) bn_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          const float* __restrict__ y, const float* __restrict__ mean,
                                                          const float* __restrict__ co, float* __restrict__ dx,
                                                          float* __restrict__ gout, int64_t M, int C) {
  const int cq = C / 4;
  const int64_t total = M * cq, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % cq) * 4;
    f32x4 g = *reinterpret_cast<const f32x4*>(dy + t * 4);
    if (y) {
      const f32x4 yy = *reinterpret_cast<const f32x4*>(y + t * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
    }
    const f32x4 xm = *reinterpret_cast<const f32x4*>(x + t * 4) - *reinterpret_cast<const f32x4*>(mean + c);
    const f32x4 d = *reinterpret_cast<const f32x4*>(co + c) * g + *reinterpret_cast<const f32x4*>(co + C + c) +
                    *reinterpret_cast<const f32x4*>(co + 2 * C + c) * xm;
    *reinterpret_cast<f32x4*>(dx + t * 4) = d;
    if (gout) *reinterpret_cast<f32x4*>(gout + t * 4) = g;
  }
}

// ------------------------------------------------------------------ pooling (fp32, NHWC)
// maxpool forward: 4 channels per thread; idx = argmax window position (first max, PyTorch's rule)
__global__ void __launch_bounds__(kT) maxpool_f32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                             int P, int Q, int k, int s, int pad) {
  const int cq = C / 4;
  const int64_t total = (int64_t)N * P * Q * cq, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % cq) * 4;
    int64_t r = t / cq;
    const int q = (int)(r % Q);
    r /= Q;
    const int p = (int)(r % P);
    const int n = (int)(r / P);
    f32x4 best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    uint8_t bi[4] = {0, 0, 0, 0};
    for (int a = 0; a < k; ++a) {
      const int h = p * s - pad + a;
      if (h < 0 || h >= H) continue;
      for (int b = 0; b < k; ++b) {
        const int w = q * s - pad + b;
        if (w < 0 || w >= W) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(x + (((int64_t)n * H + h) * W + w) * C + c);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {  // NaN propagates like torch
            best[j] = v[j];
            bi[j] = (uint8_t)(a * k + b);
          }
      }
    }
    *reinterpret_cast<f32x4*>(y + t * 4) = best;
#pragma unroll
    for (int j = 0; j < 4; ++j) idx[t * 4 + j] = bi[j];
  }
}

// maxpool backward as a gather (no atomics): every input element sums dy of the windows whose argmax
// it is.
__global__ void __launch_bounds__(kT) maxpool_f32_bwd_kernel(const float* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx, float* __restrict__ dx,
                                                             int N, int H, int W, int C, int P, int Q, int k, int s,
                                                             int pad) {
  const int64_t total = (int64_t)N * H * W * C, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % C);
    int64_t r = t / C;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    const int p0 = max(0, (h + pad - k + s) / s), p1 = min(P - 1, (h + pad) / s);
    const int q0 = max(0, (w + pad - k + s) / s), q1 = min(Q - 1, (w + pad) / s);
    float acc = 0.f;
    for (int p = p0; p <= p1; ++p) {
      const int a = h - (p * s - pad);
      if (a < 0 || a >= k) continue;
      for (int q = q0; q <= q1; ++q) {
        const int b = w - (q * s - pad);
        if (b < 0 || b >= k) continue;
        const int64_t o = (((int64_t)n * P + p) * Q + q) * C + c;
        if (idx[o] == a * k + b) acc += dy[o];
      }
    }
    dx[t] = acc;
  }
}

__global__ void __launch_bounds__(kT) avgpool_f32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int N,
                                                             int HW, int C) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * C) return;
  const int n = (int)(t / C), c = (int)(t % C);
  const float* p = x + (int64_t)n * HW * C + c;
  float acc = 0.f;
  for (int i = 0; i < HW; ++i) acc += p[(int64_t)i * C];
  y[t] = acc / (float)HW;
}

__global__ void __launch_bounds__(kT) avgpool_f32_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx,
                                                             int N, int HW, int C) {
  const int64_t total = (int64_t)N * HW * C, stride = (int64_t)gridDim.x * blockDim.x;
  const float r = 1.f / (float)HW;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % C);
    const int n = (int)(t / C / HW);
    dx[t] = dy[(int64_t)n * C + c] * r;
  }
}

// grid of the reduce: rows chunked so each thread sums ~32 rows, at most 1024 partial rows
void reduce_grid(int64_t M, int C, int& qpb, dim3& grid) {
  const int cq = C / 4;
  qpb = cq < kT ? cq : kT;
  while (kT % qpb) --qpb;  // qpb divides the block (C/4 = 3 * 2^k for some widths)
  const int rpb = kT / qpb;
  int64_t gx = (M + (int64_t)rpb * 32 - 1) / ((int64_t)rpb * 32);
  if (gx > 1024) gx = 1024;
  if (gx < 1) gx = 1;
  grid = dim3((unsigned)gx, (unsigned)((cq + qpb - 1) / qpb));
}

}  // namespace

hipError_t split_bf16(const float* x, bf16_t* out, int64_t rows, int64_t C, int nseg, int lo_mask, int64_t seg_stride,
                      int64_t row_stride, hipStream_t st) {
  if (C % 4 || nseg < 1 || nseg > 4) return hipErrorInvalidValue;
  split_kernel<<<grid_for(rows * (C / 4)), kT, 0, st>>>(x, out, rows, C, nseg, lo_mask, seg_stride, row_stride);
  return hipGetLastError();
}

int bn_f32_partials(int64_t M, int C) {
  int qpb;
  dim3 g;
  reduce_grid(M, C, qpb, g);
  return (int)g.x;
}

hipError_t bn_f32_fwd_train(const float* x, const float* res, const float* gamma, const float* beta,
                            float* running_mean, float* running_var, const float* shift, float momentum, float eps,
                            int relu, float* y, float* save_mean, float* save_invstd, float* ss, float* part,
                            int64_t* num_batches, int64_t M, int C, hipStream_t st) {
  if (C % 4) return hipErrorInvalidValue;
  int qpb;
  dim3 g;
  reduce_grid(M, C, qpb, g);
  bn_reduce_kernel<false><<<g, kT, 0, st>>>(x, nullptr, nullptr, shift, part, M, C, qpb);
  PDA_CHECK_HIP(hipGetLastError());
  bn_fwd_finalize_kernel<<<(C + kT - 1) / kT, kT, 0, st>>>(part, (int)g.x, M, C, shift, gamma, beta, running_mean,
                                                           running_var, momentum, eps, save_mean, save_invstd, ss,
                                                           num_batches);
  PDA_CHECK_HIP(hipGetLastError());
  bn_apply_kernel<<<grid_for(M * C, 4), kT, 0, st>>>(x, res, ss, y, M, C, relu);
  return hipGetLastError();
}

hipError_t bn_f32_apply(const float* x, const float* res, const float* ss, float* y, int64_t M, int C, int relu,
                        hipStream_t st) {
  if (C % 4) return hipErrorInvalidValue;
  bn_apply_kernel<<<grid_for(M * C, 4), kT, 0, st>>>(x, res, ss, y, M, C, relu);
  return hipGetLastError();
}

hipError_t bn_f32_bwd(const float* dy, const float* x, const float* y, const float* mean, const float* invstd,
                      const float* gamma, float* dx, float* gout, float* dgamma, float* dbeta, float* part, float* co,
                      int64_t M, int C, hipStream_t st) {
  if (C % 4) return hipErrorInvalidValue;
  int qpb;
  dim3 g;
  reduce_grid(M, C, qpb, g);
  bn_reduce_kernel<true><<<g, kT, 0, st>>>(x, dy, y, mean, part, M, C, qpb);
  PDA_CHECK_HIP(hipGetLastError());
  bn_bwd_finalize_kernel<<<(C + kT - 1) / kT, kT, 0, st>>>(part, (int)g.x, M, C, invstd, gamma, dgamma, dbeta, co);
  PDA_CHECK_HIP(hipGetLastError());
  bn_bwd_apply_kernel<<<grid_for(M * C, 4), kT, 0, st>>>(dy, x, y, mean, co, dx, gout, M, C);
  return hipGetLastError();
}

hipError_t maxpool2d_f32_fwd(const float* x, float* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int k,
                             int s, int pad, hipStream_t st) {
  if (C % 4) return hipErrorInvalidValue;
  maxpool_f32_fwd_kernel<<<grid_for((int64_t)N * P * Q * C, 4), kT, 0, st>>>(x, y, idx, N, H, W, C, P, Q, k, s, pad);
  return hipGetLastError();
}

hipError_t maxpool2d_f32_bwd(const float* dy, const uint8_t* idx, float* dx, int N, int H, int W, int C, int P, int Q,
                             int k, int s, int pad, hipStream_t st) {
  maxpool_f32_bwd_kernel<<<grid_for((int64_t)N * H * W * C), kT, 0, st>>>(dy, idx, dx, N, H, W, C, P, Q, k, s, pad);
  return hipGetLastError();
}

hipError_t avgpool_f32_fwd(const float* x, float* y, int N, int HW, int C, hipStream_t st) {
  avgpool_f32_fwd_kernel<<<(unsigned)(((int64_t)N * C + kT - 1) / kT), kT, 0, st>>>(x, y, N, HW, C);
  return hipGetLastError();
}

hipError_t avgpool_f32_bwd(const float* dy, float* dx, int N, int HW, int C, hipStream_t st) {
  avgpool_f32_bwd_kernel<<<grid_for((int64_t)N * HW * C), kT, 0, st>>>(dy, dx, N, HW, C);
  return hipGetLastError();
}

}  // namespace pda
