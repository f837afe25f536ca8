// Pooling over channels-last activations (SURVEY §2.5 K06 MaxPool2d 3x3/s2/p1 `NB03:333`,
// K07 AdaptiveAvgPool2d(1) `NB03:341`).
//
// MaxPool saves the in-window argmax as one byte per output element (the window is at most 255
// positions), so the backward is a gather over the <= ceil(k/s)^2 windows that cover each input
// pixel: no atomics, no [N,H,W,C] index tensor.  Each lane owns 8 channels (16-B accesses).
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kThreads = 256;

inline int ew_grid(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  if (g > 16384) g = 16384;
  return g < 1 ? 1 : (int)g;
}

// BN: the pooled tensor is relu(x * ss[c] + ss[C + c]) computed on the fly from the BatchNorm input
// (stem conv -> BN -> ReLU -> maxpool: the BN+ReLU output is never stored)
template <bool BN>
__global__ void __launch_bounds__(kThreads) maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                               uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                               int P, int Q, int k, int s, int pad,
                                                               const float* __restrict__ ss) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * P * Q * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c8 = (int)(t % cv);
    int64_t pix = t / cv;
    const int q = (int)(pix % Q);
    pix /= Q;
    const int p = (int)(pix % P);
    const int n = (int)(pix / P);
    float best[8], sc[8], sh[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    if constexpr (BN) {
      load8(ss + c8 * 8, sc);
      load8(ss + C + c8 * 8, sh);
    }
    for (int kh = 0; kh < k; ++kh) {
      const int h = p * s - pad + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = q * s - pad + kw;
        if (w < 0 || w >= W) continue;
        float v[8];
        load8(x + (((int64_t)n * H + h) * W + w) * C + c8 * 8, v);
        if constexpr (BN) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f)));  // as stored
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best[j] || (v[j] != v[j])) {  // NaN propagates like torch
            best[j] = v[j];
            bi[j] = (uint8_t)(kh * k + kw);
          }
      }
    }
    store8(y + t * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= (uint64_t)bi[j] << (8 * j);
    *reinterpret_cast<uint64_t*>(idx + t * 8) = packed;
  }
}

__global__ void __launch_bounds__(kThreads) maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                               int P, int Q, int k, int s, int pad) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c8 = (int)(t % cv);
    int64_t pix = t / cv;
    const int w = (int)(pix % W);
    pix /= W;
    const int h = (int)(pix % H);
    const int n = (int)(pix / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // outputs p with p*s - pad <= h <= p*s - pad + k - 1
    const int p_lo = max(0, (h + pad - k + s) / s), p_hi = min(P - 1, (h + pad) / s);
    const int q_lo = max(0, (w + pad - k + s) / s), q_hi = min(Q - 1, (w + pad) / s);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int kh = h - (p * s - pad);
      if (kh < 0 || kh >= k) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int kw = w - (q * s - pad);
        if (kw < 0 || kw >= k) continue;
        const int64_t o = (((int64_t)n * P + p) * Q + q) * C + c8 * 8;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        float g[8];
        load8(dy + o, g);
        const uint8_t me = (uint8_t)(kh * k + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((uint8_t)(packed >> (8 * j)) == me) acc[j] += g[j];
      }
    }
    store8(dx + t * 8, acc);
  }
}

// 3x3 / stride 2 / pad 1 (the ResNet stem pool): one thread per 2x2 input block (2p..2p+1, 2q..2q+1)
// and 8 channels.  Exactly the outputs (p..p+1, q..q+1) cover the block, so each dy / argmax vector
// is read once per block instead of once per covering input pixel (4x fewer L2 reads than the
// generic gather above), and all index math is 32-bit (no 64-bit div/mod per vector).
//   dx(2p,   2q)   = [i(p,q)=4] g(p,q)
//   dx(2p,   2q+1) = [i(p,q)=5] g(p,q)   + [i(p,q+1)=3] g(p,q+1)
//   dx(2p+1, 2q)   = [i(p,q)=7] g(p,q)   + [i(p+1,q)=1] g(p+1,q)
//   dx(2p+1, 2q+1) = [i(p,q)=8] g(p,q) + [i(p,q+1)=6] g(p,q+1) + [i(p+1,q)=2] g(p+1,q) + [i(p+1,q+1)=0] g(p+1,q+1)
__global__ void __launch_bounds__(kThreads) maxpool3s2_bwd_kernel(const bf16_t* __restrict__ dy,
                                                                  const uint8_t* __restrict__ idx,
                                                                  bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                                  int P, int Q) {
  const int cv = C >> 3;
  const int Hb = (H + 1) >> 1, Wb = (W + 1) >> 1;
  const int total = N * Hb * Wb * cv;
  const int stride = gridDim.x * blockDim.x;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c8 = t % cv;
    int pix = t / cv;
    const int q = pix % Wb;
    pix /= Wb;
    const int p = pix % Hb;
    const int n = pix / Hb;
    float g[4][8];
    uint64_t id[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int pp = p + (o >> 1), qq = q + (o & 1);
      if (pp < P && qq < Q) {
        const int64_t off = (((int64_t)n * P + pp) * Q + qq) * C + c8 * 8;
        id[o] = *reinterpret_cast<const uint64_t*>(idx + off);
        load8(dy + off, g[o]);
      } else {
        id[o] = ~0ull;  // no tap matches 0xFF
#pragma unroll
        for (int j = 0; j < 8; ++j) g[o][j] = 0.f;
      }
    }
    float d00[8], d01[8], d10[8], d11[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i0 = (uint32_t)(id[0] >> (8 * j)) & 0xFF, i1 = (uint32_t)(id[1] >> (8 * j)) & 0xFF;
      const uint32_t i2 = (uint32_t)(id[2] >> (8 * j)) & 0xFF, i3 = (uint32_t)(id[3] >> (8 * j)) & 0xFF;
      d00[j] = i0 == 4 ? g[0][j] : 0.f;
      d01[j] = (i0 == 5 ? g[0][j] : 0.f) + (i1 == 3 ? g[1][j] : 0.f);
      d10[j] = (i0 == 7 ? g[0][j] : 0.f) + (i2 == 1 ? g[2][j] : 0.f);
      d11[j] = ((i0 == 8 ? g[0][j] : 0.f) + (i1 == 6 ? g[1][j] : 0.f)) + ((i2 == 2 ? g[2][j] : 0.f) + (i3 == 0 ? g[3][j] : 0.f));
    }
    const int h = 2 * p, w = 2 * q;
    bf16_t* base = dx + (((int64_t)n * H + h) * W + w) * C + c8 * 8;
    store8(base, d00);
    if (w + 1 < W) store8(base + C, d01);
    if (h + 1 < H) {
      store8(base + (int64_t)W * C, d10);
      if (w + 1 < W) store8(base + (int64_t)W * C + C, d11);
    }
  }
}

// Global average pool: x [N, HW, C] -> y [N, C]
template <typename O>
__global__ void __launch_bounds__(kThreads) avgpool_fwd_kernel(const bf16_t* __restrict__ x, O* __restrict__ y, int N,
                                                               int HW, int C) {
  const int cv = C / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * cv) return;
  const int n = (int)(t / cv), c8 = (int)(t % cv);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const bf16_t* base = x + (int64_t)n * HW * C + c8 * 8;
  for (int i = 0; i < HW; ++i) {
    float v[8];
    load8(base + (int64_t)i * C, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  const float r = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= r;
  store8(y + (int64_t)n * C + c8 * 8, acc);
}

template <typename G>
__global__ void __launch_bounds__(kThreads) avgpool_bwd_kernel(const G* __restrict__ dy, bf16_t* __restrict__ dx,
                                                               int N, int HW, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * HW * cv;
  const float r = 1.f / (float)HW;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c8 = (int)(t % cv);
    const int n = (int)(t / cv / HW);
    float g[8];
    load8(dy + (int64_t)n * C + c8 * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= r;
    store8(dx + t * 8, g);
  }
}

}  // namespace

hipError_t maxpool2d_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int k,
                         int s, int pad, hipStream_t st) {
  const int64_t total = (int64_t)N * P * Q * (C / 8);
  maxpool_fwd_kernel<false><<<ew_grid(total), kThreads, 0, st>>>(x, y, idx, N, H, W, C, P, Q, k, s, pad, nullptr);
  return hipGetLastError();
}

hipError_t maxpool2d_bn_fwd(const bf16_t* x, const float* ss, bf16_t* y, uint8_t* idx, int N, int H, int W, int C,
                            int P, int Q, int k, int s, int pad, hipStream_t st) {
  const int64_t total = (int64_t)N * P * Q * (C / 8);
  maxpool_fwd_kernel<true><<<ew_grid(total), kThreads, 0, st>>>(x, y, idx, N, H, W, C, P, Q, k, s, pad, ss);
  return hipGetLastError();
}

hipError_t maxpool2d_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int P, int Q,
                         int k, int s, int pad, hipStream_t st) {
  const int64_t blocks = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  if (k == 3 && s == 2 && pad == 1 && P == (H - 1) / 2 + 1 && Q == (W - 1) / 2 + 1 && blocks < (1ll << 31) - 2048 * 256) {
    maxpool3s2_bwd_kernel<<<ew_grid(blocks), kThreads, 0, st>>>(dy, idx, dx, N, H, W, C, P, Q);
    return hipGetLastError();
  }
  const int64_t total = (int64_t)N * H * W * (C / 8);
  maxpool_bwd_kernel<<<ew_grid(total), kThreads, 0, st>>>(dy, idx, dx, N, H, W, C, P, Q, k, s, pad);
  return hipGetLastError();
}

hipError_t avgpool_global_fwd(const bf16_t* x, void* y, bool y_bf16, int N, int HW, int C, hipStream_t st) {
  const int64_t total = (int64_t)N * (C / 8);
  const int grid = (int)((total + kThreads - 1) / kThreads);
  if (y_bf16) avgpool_fwd_kernel<bf16_t><<<grid, kThreads, 0, st>>>(x, (bf16_t*)y, N, HW, C);
  else avgpool_fwd_kernel<float><<<grid, kThreads, 0, st>>>(x, (float*)y, N, HW, C);
  return hipGetLastError();
}

hipError_t avgpool_global_bwd(const void* dy, bool dy_bf16, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  const int64_t total = (int64_t)N * HW * (C / 8);
  if (dy_bf16) avgpool_bwd_kernel<bf16_t><<<ew_grid(total), kThreads, 0, st>>>((const bf16_t*)dy, dx, N, HW, C);
  else avgpool_bwd_kernel<float><<<ew_grid(total), kThreads, 0, st>>>((const float*)dy, dx, N, HW, C);
  return hipGetLastError();
}

// ------------------------------------------------------------------ stem space-to-depth
// y[n, u, v, (i*2 + j)*C + c] = x[n, 2u + i - pad, 2v + j - pad, c] (0 outside), channels padded with
// zeros to Cy (16): the 7x7/2 stem conv becomes a 4x4/1 conv with 16-B channel vectors (see
// models/resnet.py:space_to_depth_stem).  One thread per output pixel: 4 x C input loads (x's pixel
// stride Cx may exceed C — device-side channel padding is skipped), two 16-B stores.
__global__ void __launch_bounds__(256) stem_s2d_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N,
                                                       int H, int W, int Cx, int C, int U, int V, int pad) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)N * U * V;
  if (t >= total) return;
  const int v = (int)(t % V);
  const int64_t r = t / V;
  const int u = (int)(r % U);
  const int n = (int)(r / U);
  u16x8 o0, o1;
#pragma unroll
  for (int q = 0; q < 8; ++q) o0[q] = o1[q] = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int h = 2 * u + i - pad, w = 2 * v + j - pad;
      if ((unsigned)h >= (unsigned)H || (unsigned)w >= (unsigned)W) continue;
      const bf16_t* px = x + (((int64_t)n * H + h) * W + w) * Cx;
      // slot (i, j, c) = (i*2 + j)*C + c; unrolled over c < 4 so every vector index is a constant
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c >= C) break;
        const bf16_t val = px[c];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          if (k != (i * 2 + j) * C + c) continue;
          if (k < 8) o0[k] = val;
          else o1[k - 8] = val;
        }
      }
    }
  u16x8* dst = reinterpret_cast<u16x8*>(y + t * 16);
  dst[0] = o0;
  dst[1] = o1;
}

hipError_t stem_space_to_depth(const bf16_t* x, bf16_t* y, int N, int H, int W, int Cx, int C, int U, int V, int pad,
                               hipStream_t st) {
  if (C < 1 || 4 * C > 16) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * U * V;
  stem_s2d_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(x, y, N, H, W, Cx, C, U, V, pad);
  return hipGetLastError();
}

}  // namespace pda
