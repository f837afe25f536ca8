// Cross-entropy forward / backward.
//
// Reference call sites: `F.cross_entropy(output, ys)` with FLOAT probability targets (`PY1:40`,
// ys = rand(1) at `PY1:60`) and `nn.CrossEntropyLoss()(outputs, one_hot)` (`NB03:382,389`), i.e. the
// probability-target path; the BASELINE configs use class indices (MNIST / ImageNet / LM heads).
// Both are served here.  One workgroup per row; the forward is a single pass with an online
// log-sum-exp (running max + rescaled sum per lane, merged across the block), the backward
// recomputes softmax from the saved LSE and writes dlogits directly (no [M,C] probability tensor).
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// Block-wide merge of per-thread (max, scaled-sum) pairs plus two plain sums. Result on all threads.
__device__ __forceinline__ void block_lse(float& m, float& s, float& a, float& b) {
  __shared__ float sm[16], ss[16], sa[16], sb[16];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
    sa[wid] = a;
    sb[wid] = b;
  }
  __syncthreads();
  m = sm[0];
  s = ss[0];
  a = sa[0];
  b = sb[0];
  for (int i = 1; i < nw; ++i) {
    lse_merge(m, s, sm[i], ss[i]);
    a += sa[i];
    b += sb[i];
  }
}

// Forward. Class-index targets: loss = (1-eps)(lse - x_t) + eps(lse - mean_c x_c), 0 for ignored rows.
// Probability targets:        loss = lse * sum_c p_c - sum_c p_c x_c.
template <typename T>
__global__ void __launch_bounds__(kThreads) ce_fwd_kernel(const T* __restrict__ logits, int64_t C, int64_t Cv,
                                                          const int64_t* __restrict__ tidx,
                                                          const float* __restrict__ tprob, int64_t ignore_index,
                                                          float smoothing, float* __restrict__ loss,
                                                          float* __restrict__ lse_out) {
  const int64_t r = blockIdx.x;
  const T* row = logits + r * C;
  float m = -INFINITY, s = 0.f, a = 0.f, b = 0.f;  // a: sum x (or sum p x), b: sum p
  if (tprob) {
    const float* prow = tprob + r * C;
    for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
      const float v = Elem<T>::load(row, c), p = prow[c];
      lse_merge(m, s, v, 1.f);
      a += p * v;
      b += p;
    }
  } else if (C % 8 == 0) {
    for (int64_t c = (int64_t)threadIdx.x * 8; c < Cv; c += (int64_t)blockDim.x * 8) {
      float v[8];
      load8(row + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c + j >= Cv) v[j] = -INFINITY;  // vocabulary padding
      float lm = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ls += __expf(v[j] - lm);
        a += (c + j < Cv) ? v[j] : 0.f;
      }
      lse_merge(m, s, lm, ls);
    }
  } else {
    for (int64_t c = threadIdx.x; c < Cv; c += blockDim.x) {
      const float v = Elem<T>::load(row, c);
      lse_merge(m, s, v, 1.f);
      a += v;
    }
  }
  block_lse(m, s, a, b);
  if (threadIdx.x == 0) {
    const float lse = m + __logf(s);
    lse_out[r] = lse;
    float l;
    if (tprob) {
      l = lse * b - a;
    } else {
      const int64_t t = tidx[r];
      if (t == ignore_index || t < 0 || t >= Cv) {
        l = 0.f;
      } else {
        const float xt = Elem<T>::load(row, t);
        l = (1.f - smoothing) * (lse - xt) + smoothing * (lse - a / (float)Cv);
      }
    }
    loss[r] = l;
  }
}

// Backward: d x_c = g * (softmax_c * S - target_c), S = sum_c p_c for probability targets (1 for
// class indices), target_c = (1-eps)[c==t] + eps/C for class indices.
template <typename T, typename D>
__global__ void __launch_bounds__(kThreads) ce_bwd_kernel(const T* __restrict__ logits, int64_t C, int64_t Cv,
                                                          const int64_t* __restrict__ tidx,
                                                          const float* __restrict__ tprob, int64_t ignore_index,
                                                          float smoothing, const float* __restrict__ lse,
                                                          const float* __restrict__ gscale_ptr, float gscale,
                                                          D* __restrict__ dlogits) {
  __shared__ float scratch[16];
  const int64_t r = blockIdx.x;
  const T* row = logits + r * C;
  D* drow = dlogits + r * C;
  const float g = gscale * (gscale_ptr ? gscale_ptr[0] : 1.f);
  const float L = lse[r];
  if (tprob) {
    const float* prow = tprob + r * C;
    float ps = 0.f;
    for (int64_t c = threadIdx.x; c < C; c += blockDim.x) ps += prow[c];
    ps = block_sum(ps, scratch);
    for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
      const float sm = __expf(Elem<T>::load(row, c) - L);
      Elem<D>::store(drow, c, g * (sm * ps - prow[c]));
    }
    return;
  }
  const int64_t t = tidx[r];
  const float gr = (t == ignore_index) ? 0.f : g;
  const float off = smoothing / (float)Cv, hit = 1.f - smoothing;
  if (C % 8 == 0) {
    for (int64_t c = (int64_t)threadIdx.x * 8; c < C; c += (int64_t)blockDim.x * 8) {
      float v[8];
      load8(row + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = (c + j < Cv) ? gr * (__expf(v[j] - L) - ((c + j == t ? hit : 0.f) + off)) : 0.f;
      store8(drow + c, v);
    }
  } else {
    for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
      const float sm = __expf(Elem<T>::load(row, c) - L);
      Elem<D>::store(drow, c, c < Cv ? gr * (sm - ((c == t ? hit : 0.f) + off)) : 0.f);
    }
  }
}

}  // namespace

hipError_t cross_entropy_fwd(const void* logits, bool logits_bf16, int64_t M, int64_t C, int64_t Cv,
                             const int64_t* target_idx,
                             const float* target_prob, int64_t ignore_index, float smoothing, float* loss, float* lse,
                             hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (logits_bf16)
    ce_fwd_kernel<bf16_t><<<(unsigned)M, kThreads, 0, st>>>((const bf16_t*)logits, C, Cv, target_idx, target_prob,
                                                            ignore_index, smoothing, loss, lse);
  else
    ce_fwd_kernel<float><<<(unsigned)M, kThreads, 0, st>>>((const float*)logits, C, Cv, target_idx, target_prob,
                                                           ignore_index, smoothing, loss, lse);
  return hipGetLastError();
}

hipError_t cross_entropy_bwd(const void* logits, bool logits_bf16, int64_t M, int64_t C, int64_t Cv,
                             const int64_t* target_idx,
                             const float* target_prob, int64_t ignore_index, float smoothing, const float* lse,
                             const float* gscale_ptr, float gscale, void* dlogits, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (logits_bf16)
    ce_bwd_kernel<bf16_t, bf16_t><<<(unsigned)M, kThreads, 0, st>>>((const bf16_t*)logits, C, Cv, target_idx,
                                                                    target_prob, ignore_index, smoothing, lse,
                                                                    gscale_ptr, gscale, (bf16_t*)dlogits);
  else
    ce_bwd_kernel<float, float><<<(unsigned)M, kThreads, 0, st>>>((const float*)logits, C, Cv, target_idx, target_prob,
                                                                  ignore_index, smoothing, lse, gscale_ptr, gscale,
                                                                  (float*)dlogits);
  return hipGetLastError();
}

}  // namespace pda
