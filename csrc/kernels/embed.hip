// Token embedding lookup / gradient and a standalone rotary-embedding pass.
//
// Embedding forward: row gather, 16-B vector per lane.  Backward: each token's gradient row is added
// into an fp32 accumulator of the table with float atomics (no sort); rows are 2-8 KB so every wave
// instruction adds 1 KB of contiguous bytes (the full-rate atomic shape, guide §6 G12), and only
// repeated tokens contend.  The fp32 accumulator is cast to the parameter dtype afterwards.
// (PDA_DETERMINISTIC=1: a sorted, atomic-free variant.)
// RoPE (rotate-half convention) is normally fused into the attention kernels; `rope_apply` is the
// standalone form (e.g. for KV-cache writes / tests).
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads) embedding_fwd_kernel(const int64_t* __restrict__ idx,
                                                                 const bf16_t* __restrict__ table,
                                                                 bf16_t* __restrict__ out, int64_t n, int64_t D) {
  const int64_t cv = D / 8;
  const int64_t total = n * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t tok = t / cv, c = t % cv;
    const int64_t row = idx[tok];
    *reinterpret_cast<u16x8*>(out + tok * D + c * 8) = *reinterpret_cast<const u16x8*>(table + row * D + c * 8);
  }
}

__global__ void __launch_bounds__(kThreads) embedding_bwd_kernel(const int64_t* __restrict__ idx,
                                                                 const bf16_t* __restrict__ dy,
                                                                 float* __restrict__ acc, int64_t n, int64_t D) {
  const int64_t cv = D / 8;
  const int64_t total = n * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t tok = t / cv, c = t % cv;
    const int64_t row = idx[tok];
    float g[8];
    load8(dy + tok * D + c * 8, g);
    float* dst = acc + row * D + c * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(dst + j, g[j]);
  }
}

// PDA_DETERMINISTIC=1: the same gradient without atomics.  The tokens come sorted by id (stable sort:
// `sidx`, with `order` mapping a sorted position back to its token); the lane at the first position of a
// run of equal ids sums the run's dy rows in token order and stores the table row once.
__global__ void __launch_bounds__(kThreads) embedding_bwd_sorted_kernel(const int64_t* __restrict__ sidx,
                                                                        const int64_t* __restrict__ order,
                                                                        const bf16_t* __restrict__ dy,
                                                                        float* __restrict__ acc, int64_t n, int64_t D) {
  const int64_t cv = D / 8;
  const int64_t total = n * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t j = t / cv, c = t % cv;
    const int64_t row = sidx[j];
    if (j > 0 && sidx[j - 1] == row) continue;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t k = j; k < n && sidx[k] == row; ++k) {
      float g[8];
      load8(dy + order[k] * D + c * 8, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += g[e];
    }
    float* dst = acc + row * D + c * 8;
    *reinterpret_cast<float4*>(dst) = make_float4(s[0], s[1], s[2], s[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(s[4], s[5], s[6], s[7]);
  }
}

__global__ void __launch_bounds__(kThreads) rope_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                        const float* __restrict__ cs, const float* __restrict__ sn,
                                                        int B, int T, int H, int D, int64_t sb, int64_t st_,
                                                        int64_t sh, int64_t yb, int64_t yt, int64_t yh, float sign) {
  const int half = D / 2, hv = half / 8;
  const int64_t total = (int64_t)B * T * H * hv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c = (int)(t % hv);
    int64_t r = t / hv;
    const int h = (int)(r % H);
    r /= H;
    const int pos = (int)(r % T);
    const int b = (int)(r / T);
    const int64_t base = b * sb + pos * st_ + h * sh + c * 8;
    const int64_t ybase = b * yb + pos * yt + h * yh + c * 8;
    float a[8], bb[8];
    load8(x + base, a);
    load8(x + base + half, bb);
    const float* cr = cs + (int64_t)pos * half + c * 8;
    const float* sr = sn + (int64_t)pos * half + c * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sign * sr[j];
      const float x1 = a[j], x2 = bb[j];
      a[j] = x1 * cr[j] - x2 * s;
      bb[j] = x2 * cr[j] + x1 * s;
    }
    store8(y + ybase, a);
    store8(y + ybase + half, bb);
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

hipError_t embedding_fwd(const int64_t* idx, const bf16_t* table, bf16_t* out, int64_t n, int64_t D, hipStream_t st) {
  embedding_fwd_kernel<<<grid_for(n * D / 8), kThreads, 0, st>>>(idx, table, out, n, D);
  return hipGetLastError();
}

hipError_t embedding_bwd(const int64_t* idx, const bf16_t* dy, float* acc, int64_t n, int64_t D, hipStream_t st) {
  embedding_bwd_kernel<<<grid_for(n * D / 8), kThreads, 0, st>>>(idx, dy, acc, n, D);
  return hipGetLastError();
}

hipError_t embedding_bwd_sorted(const int64_t* sidx, const int64_t* order, const bf16_t* dy, float* acc, int64_t n,
                                int64_t D, hipStream_t st) {
  embedding_bwd_sorted_kernel<<<grid_for(n * D / 8), kThreads, 0, st>>>(sidx, order, dy, acc, n, D);
  return hipGetLastError();
}

hipError_t rope_apply(const bf16_t* x, bf16_t* y, const float* cos, const float* sin, int B, int T, int H, int D,
                      int64_t sb, int64_t st_, int64_t sh, int64_t yb, int64_t yt, int64_t yh, bool inverse,
                      hipStream_t st) {
  rope_kernel<<<grid_for((int64_t)B * T * H * (D / 16)), kThreads, 0, st>>>(x, y, cos, sin, B, T, H, D, sb, st_, sh,
                                                                            yb, yt, yh, inverse ? -1.f : 1.f);
  return hipGetLastError();
}

}  // namespace pda
