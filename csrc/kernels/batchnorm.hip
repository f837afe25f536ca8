// Training-mode BatchNorm over channels-last (NHWC) activations, with fused residual-add + ReLU
// (SURVEY §2.5 K05, K03).
//
// The reference's ResNet-50 (`NB03:314`, Bottleneck BN ×53, `model.train()` at `NB03:381`) runs
// torch's BN followed by separate ReLU / add kernels.  Here every BN is viewed as an [M = N*H*W, C]
// matrix (C contiguous, a multiple of 8) and handled by three memory-bound passes:
//   stats   : per-channel Welford (count, mean, M2) per workgroup → partial slabs
//   finalize: Chan-merge the partial slabs → mean / invstd / running stats / per-channel affine
//   apply   : y = relu(x * scale_c + shift_c [+ residual])          (one read, one write)
// Backward mirrors it: a reduction of (dz, dz*(x-mean)) with dz = dy * [y > 0] recomputed from the
// saved output, a finalize producing dgamma / dbeta and per-channel (A, B, C) such that
// dx = A*dz + B*x + C, and one apply pass that also emits dz for the residual branch.
// Each lane owns 8 consecutive channels (16-B loads); workgroups tile rows × channel groups.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 2048;

struct BnGeom {
  int cv;         // 8-channel vectors per row
  int cols;       // vector columns per block
  int rpi;        // rows per block iteration (threads stacked along rows)
  int gy;         // channel-group blocks
  int64_t rpb;    // rows per block
  int nrb;        // row blocks
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
  const int target = kMaxBlocks / g.gy > 0 ? kMaxBlocks / g.gy : 1;
  int64_t rpb = (M + target - 1) / target;
  const int64_t min_rpb = (int64_t)g.rpi * 8;
  if (rpb < min_rpb) rpb = min_rpb;
  g.rpb = rpb;
  g.nrb = (int)((M + rpb - 1) / rpb);
  return g;
}

__device__ __forceinline__ void chan_merge(float& na, float& ma, float& qa, float nb, float mb, float qb) {
  const float n = na + nb;
  if (nb == 0.f) return;
  if (na == 0.f) {
    na = nb;
    ma = mb;
    qa = qb;
    return;
  }
  const float d = mb - ma, f = nb / n;
  ma += d * f;
  qa += qb + d * d * na * f;
  na = n;
}

// ---------------------------------------------------------------- forward statistics
// partial layout: [nrb][C] mean, then [nrb][C] M2 ; counts are implied by the row-block extents.
__global__ void __launch_bounds__(kThreads) bn_stats_kernel(const bf16_t* __restrict__ x, int64_t M, int C, int cols,
                                                            int rpi, int64_t rpb, float* __restrict__ pmean,
                                                            float* __restrict__ pm2) {
  __shared__ float s_mean[kThreads * 8];
  __shared__ float s_m2[kThreads * 8];
  __shared__ float s_n[kThreads];
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(r0 + rpb, M);
  float mean[8], m2[8], n = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) mean[j] = m2[j] = 0.f;
  if (active) {
    for (int64_t r = r0 + ty; r < r1; r += rpi) {
      float v[8];
      load8(x + r * C + vcol * 8, v);
      n += 1.f;
      const float rn = 1.f / n;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - mean[j];
        mean[j] += d * rn;
        m2[j] += d * (v[j] - mean[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s_mean[threadIdx.x * 8 + j] = mean[j];
    s_m2[threadIdx.x * 8 + j] = m2[j];
  }
  s_n[threadIdx.x] = active ? n : 0.f;
  __syncthreads();
  if (ty == 0 && vcol * 8 < C) {
    for (int k = 1; k < rpi; ++k) {
      const int t = k * cols + tx;
      const float nb = s_n[t];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float nn = n;
        chan_merge(nn, mean[j], m2[j], nb, s_mean[t * 8 + j], s_m2[t * 8 + j]);
      }
      n += nb;
    }
    float* pm = pmean + (int64_t)blockIdx.x * C + vcol * 8;
    float* pq = pm2 + (int64_t)blockIdx.x * C + vcol * 8;
    store8(pm, mean);
    store8(pq, m2);
  }
}

// One block handles 8 channels; 32 lanes per channel each merge a strided subset of the partials.
__global__ void __launch_bounds__(kThreads) bn_stats_finalize_kernel(
    const float* __restrict__ pmean, const float* __restrict__ pm2, int nrb, int64_t rpb, int64_t M, int C, float eps,
    float momentum, const float* __restrict__ gamma_f, const bf16_t* __restrict__ gamma_b,
    const float* __restrict__ beta_f, const bf16_t* __restrict__ beta_b, float* __restrict__ running_mean,
    float* __restrict__ running_var, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float sn[kThreads], sm[kThreads], sq[kThreads];
  const int ch = blockIdx.x * 8 + (threadIdx.x & 7);
  const int lane = threadIdx.x >> 3;  // 0..31
  float n = 0.f, m = 0.f, q = 0.f;
  if (ch < C) {
    for (int b = lane; b < nrb; b += 32) {
      const int64_t r0 = (int64_t)b * rpb;
      const float nb = (float)(min(r0 + rpb, M) - r0);
      chan_merge(n, m, q, nb, pmean[(int64_t)b * C + ch], pm2[(int64_t)b * C + ch]);
    }
  }
  sn[threadIdx.x] = n;
  sm[threadIdx.x] = m;
  sq[threadIdx.x] = q;
  __syncthreads();
  for (int s = 16; s > 0; s >>= 1) {
    if (lane < s) {
      const int o = threadIdx.x + s * 8;
      float nn = sn[threadIdx.x], mm = sm[threadIdx.x], qq = sq[threadIdx.x];
      chan_merge(nn, mm, qq, sn[o], sm[o], sq[o]);
      sn[threadIdx.x] = nn;
      sm[threadIdx.x] = mm;
      sq[threadIdx.x] = qq;
    }
    __syncthreads();
  }
  if (lane == 0 && ch < C) {
    const float N = sn[threadIdx.x], mean = sm[threadIdx.x], M2 = sq[threadIdx.x];
    const float var = M2 / N;
    const float invstd = rsqrtf(var + eps);
    save_mean[ch] = mean;
    save_invstd[ch] = invstd;
    if (running_mean) {
      running_mean[ch] = (1.f - momentum) * running_mean[ch] + momentum * mean;
      const float unbiased = N > 1.f ? M2 / (N - 1.f) : var;
      running_var[ch] = (1.f - momentum) * running_var[ch] + momentum * unbiased;
    }
    const float g = gamma_f ? gamma_f[ch] : (gamma_b ? bf2f(gamma_b[ch]) : 1.f);
    const float b = beta_f ? beta_f[ch] : (beta_b ? bf2f(beta_b[ch]) : 0.f);
    scale[ch] = g * invstd;
    shift[ch] = b - mean * g * invstd;
  }
}

// Eval mode: affine from running statistics.
__global__ void bn_eval_affine_kernel(int C, float eps, const float* __restrict__ gamma_f,
                                      const bf16_t* __restrict__ gamma_b, const float* __restrict__ beta_f,
                                      const bf16_t* __restrict__ beta_b, const float* __restrict__ running_mean,
                                      const float* __restrict__ running_var, float* __restrict__ scale,
                                      float* __restrict__ shift) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= C) return;
  const float invstd = rsqrtf(running_var[ch] + eps);
  const float g = gamma_f ? gamma_f[ch] : (gamma_b ? bf2f(gamma_b[ch]) : 1.f);
  const float b = beta_f ? beta_f[ch] : (beta_b ? bf2f(beta_b[ch]) : 0.f);
  scale[ch] = g * invstd;
  shift[ch] = b - running_mean[ch] * g * invstd;
}

// ---------------------------------------------------------------- forward apply
template <bool RES, bool RELU>
__global__ void __launch_bounds__(kThreads) bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                            int64_t nvec, int cv) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % cv) * 8;
    float a[8], sc[8], sh[8];
    load8(x + v * 8, a);
    load8(scale + c0, sc);
    load8(shift + c0, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = a[j] * sc[j] + sh[j];
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
// partial layout: [nrb][C] sum(dz), [nrb][C] sum(dz * (x - mean))
template <bool RELU>
__global__ void __launch_bounds__(kThreads) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ x,
                                                                 const bf16_t* __restrict__ y,
                                                                 const float* __restrict__ mean, int64_t M, int C,
                                                                 int cols, int rpi, int64_t rpb,
                                                                 float* __restrict__ psum, float* __restrict__ pdot) {
  __shared__ float s_a[kThreads * 8];
  __shared__ float s_b[kThreads * 8];
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
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s_a[threadIdx.x * 8 + j] = sa[j];
    s_b[threadIdx.x * 8 + j] = sb[j];
  }
  __syncthreads();
  if (ty == 0 && vcol * 8 < C) {
    for (int k = 1; k < rpi; ++k) {
      const int t = k * cols + tx;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sa[j] += s_a[t * 8 + j];
        sb[j] += s_b[t * 8 + j];
      }
    }
    store8(psum + (int64_t)blockIdx.x * C + vcol * 8, sa);
    store8(pdot + (int64_t)blockIdx.x * C + vcol * 8, sb);
  }
}

// dgamma = invstd * sum(dz (x-mean)), dbeta = sum(dz);  dx = A*dz + B*x + Cc
__global__ void __launch_bounds__(kThreads) bn_bwd_finalize_kernel(
    const float* __restrict__ psum, const float* __restrict__ pdot, int nrb, int64_t M, int C,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ gamma_f,
    const bf16_t* __restrict__ gamma_b, float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ coA,
    float* __restrict__ coB, float* __restrict__ coC) {
  __shared__ float s1[kThreads], s2[kThreads];
  const int ch = blockIdx.x * 8 + (threadIdx.x & 7);
  const int lane = threadIdx.x >> 3;
  float a = 0.f, b = 0.f;
  if (ch < C) {
    for (int k = lane; k < nrb; k += 32) {
      a += psum[(int64_t)k * C + ch];
      b += pdot[(int64_t)k * C + ch];
    }
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int s = 16; s > 0; s >>= 1) {
    if (lane < s) {
      s1[threadIdx.x] += s1[threadIdx.x + s * 8];
      s2[threadIdx.x] += s2[threadIdx.x + s * 8];
    }
    __syncthreads();
  }
  if (lane == 0 && ch < C) {
    const float sdz = s1[threadIdx.x], sdx = s2[threadIdx.x];
    const float is = invstd[ch], mu = mean[ch];
    const float g = gamma_f ? gamma_f[ch] : (gamma_b ? bf2f(gamma_b[ch]) : 1.f);
    const float dg = sdx * is;
    dgamma[ch] = dg;
    dbeta[ch] = sdz;
    const float A = g * is;
    const float B = -A * is * dg / (float)M;
    coA[ch] = A;
    coB[ch] = B;
    coC[ch] = -A * sdz / (float)M - B * mu;
  }
}

template <bool RELU, bool DRES>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                                const bf16_t* __restrict__ x,
                                                                const bf16_t* __restrict__ y,
                                                                const float* __restrict__ coA,
                                                                const float* __restrict__ coB,
                                                                const float* __restrict__ coC,
                                                                bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
                                                                int64_t nvec, int cv) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % cv) * 8;
    float g[8], xv[8], A[8], B[8], Cc[8];
    load8(dy + v * 8, g);
    load8(x + v * 8, xv);
    if (RELU) {
      u16x8 yr = *reinterpret_cast<const u16x8*>(y + v * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = bf2f(yr[j]) > 0.f ? g[j] : 0.f;
    }
    if (DRES) store8(dres + v * 8, g);
    load8(coA + c0, A);
    load8(coB + c0, B);
    load8(coC + c0, Cc);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = A[j] * g[j] + B[j] * xv[j] + Cc[j];
    store8(dx + v * 8, xv);
  }
}

inline int ew_grid(int64_t nvec) {
  int64_t g = (nvec + kThreads - 1) / kThreads;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

int64_t bn_workspace_floats(int64_t M, int64_t C) {
  BnGeom g = bn_geom(M, C);
  return 2 * (int64_t)g.nrb * C + 8 * C;
}

// Workspace: [2*nrb*C partial slabs][scale C][shift C] ... (see bn_workspace_floats)
hipError_t bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                        const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, float* running_mean,
                        float* running_var, float momentum, float eps, bool relu, float* save_mean,
                        float* save_invstd, float* ws, hipStream_t st) {
  BnGeom g = bn_geom(M, C);
  float* pmean = ws;
  float* pm2 = ws + (int64_t)g.nrb * C;
  float* scale = ws + 2 * (int64_t)g.nrb * C;
  float* shift = scale + C;
  bn_stats_kernel<<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(x, M, (int)C, g.cols, g.rpi, g.rpb, pmean, pm2);
  bn_stats_finalize_kernel<<<(unsigned)((C + 7) / 8), kThreads, 0, st>>>(
      pmean, pm2, g.nrb, g.rpb, M, (int)C, eps, momentum, gamma_f, gamma_b, beta_f, beta_b, running_mean, running_var,
      save_mean, save_invstd, scale, shift);
  const int64_t nvec = M * C / 8;
  const int cv = (int)(C / 8);
  const int grid = ew_grid(nvec);
  if (res && relu) bn_apply_kernel<true, true><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  else if (res) bn_apply_kernel<true, false><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  else if (relu) bn_apply_kernel<false, true><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  else bn_apply_kernel<false, false><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  return hipGetLastError();
}

hipError_t bn_fwd_eval(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                       const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, const float* running_mean,
                       const float* running_var, float eps, bool relu, float* ws, hipStream_t st) {
  float* scale = ws;
  float* shift = ws + C;
  bn_eval_affine_kernel<<<(unsigned)((C + 255) / 256), 256, 0, st>>>((int)C, eps, gamma_f, gamma_b, beta_f, beta_b,
                                                                     running_mean, running_var, scale, shift);
  const int64_t nvec = M * C / 8;
  const int cv = (int)(C / 8);
  const int grid = ew_grid(nvec);
  if (res && relu) bn_apply_kernel<true, true><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  else if (res) bn_apply_kernel<true, false><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  else if (relu) bn_apply_kernel<false, true><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  else bn_apply_kernel<false, false><<<grid, kThreads, 0, st>>>(x, res, scale, shift, y, nvec, cv);
  return hipGetLastError();
}

hipError_t bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, int64_t M, int64_t C, const float* save_mean,
                  const float* save_invstd, const float* gamma_f, const bf16_t* gamma_b, bool relu, bf16_t* dx,
                  bf16_t* dres, float* dgamma, float* dbeta, float* ws, hipStream_t st) {
  BnGeom g = bn_geom(M, C);
  float* psum = ws;
  float* pdot = ws + (int64_t)g.nrb * C;
  float* coA = ws + 2 * (int64_t)g.nrb * C;
  float* coB = coA + C;
  float* coC = coB + C;
  if (relu)
    bn_bwd_reduce_kernel<true><<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(dy, x, y, save_mean, M, (int)C, g.cols, g.rpi,
                                                                       g.rpb, psum, pdot);
  else
    bn_bwd_reduce_kernel<false><<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(dy, x, y, save_mean, M, (int)C, g.cols,
                                                                        g.rpi, g.rpb, psum, pdot);
  bn_bwd_finalize_kernel<<<(unsigned)((C + 7) / 8), kThreads, 0, st>>>(psum, pdot, g.nrb, M, (int)C, save_mean,
                                                                       save_invstd, gamma_f, gamma_b, dgamma, dbeta,
                                                                       coA, coB, coC);
  const int64_t nvec = M * C / 8;
  const int cv = (int)(C / 8);
  const int grid = ew_grid(nvec);
  if (relu && dres)
    bn_bwd_apply_kernel<true, true><<<grid, kThreads, 0, st>>>(dy, x, y, coA, coB, coC, dx, dres, nvec, cv);
  else if (relu)
    bn_bwd_apply_kernel<true, false><<<grid, kThreads, 0, st>>>(dy, x, y, coA, coB, coC, dx, dres, nvec, cv);
  else if (dres)
    bn_bwd_apply_kernel<false, true><<<grid, kThreads, 0, st>>>(dy, x, y, coA, coB, coC, dx, dres, nvec, cv);
  else
    bn_bwd_apply_kernel<false, false><<<grid, kThreads, 0, st>>>(dy, x, y, coA, coB, coC, dx, dres, nvec, cv);
  return hipGetLastError();
}

}  // namespace pda
