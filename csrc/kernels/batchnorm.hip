// Training-mode BatchNorm over channels-last (NHWC) activations, with fused residual-add + ReLU
// (SURVEY §2.5 K05, K03).
//
// The reference's ResNet-50 (`NB03:314`, Bottleneck BN x53, `model.train()` at `NB03:381`) runs
// torch's BN followed by separate ReLU / add kernels.  Here every BN is viewed as an [M = N*H*W, C]
// matrix (C contiguous, a multiple of 8) and handled in two memory-bound passes per direction:
//   forward : stats    — per-channel shifted sums (x - K_c), (x - K_c)^2 with pivot K_c = x[0, c]
//                        (cancellation-safe when |mean| >> std), block-reduced in LDS, written as
//                        per-workgroup partial slabs [nrb][C] (plain stores: no same-address atomics,
//                        which serialise at the memory side when hundreds of workgroups hit 2C words);
//             finalize — 64 channels x 16 row-lanes per workgroup sum the slabs (coalesced, unrolled),
//                        produce mean / invstd / running stats and the per-channel scale, shift;
//             apply    — y = relu(x * scale + shift [+ residual]), scale/shift staged in LDS.
//   backward: reduce   — sum(dz), sum(dz * (x - mean)) with dz = dy * [y > 0] recomputed from the
//                        saved output, same slab scheme; finalize -> dgamma / dbeta (parameter dtype)
//                        and per-channel (A, B, C); apply -> dx = A*dz + B*x + C, dz for the residual.
// Each lane owns 8 consecutive channels (16-B loads); workgroups tile rows x channel groups.
#include "pda_common.h"
#include "pda_kernels.h"

#include <cstdlib>

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
  // ~1024 row blocks (4 workgroups per CU, 8 outstanding 16-B loads per lane).  Measured on the
  // ResNet-50 shapes with HBM-cold buffers (tools/bnlab): 512 -> 1024 blocks lifts the backward
  // reductions from ~4.9 to ~6.1 TB/s (3.7 -> 5.6 with the ReLU bit mask) and the statistics pass
  // slightly; the finalize pass keeps up by summing the slab rows 8 loads deep per lane.  Small
  // blocks (>= 8 row iterations of the widest layers) keep C = 2048 at ~800 blocks, not 196.
  const int target = 1024 / g.gy > 0 ? 1024 / g.gy : 1;
  int64_t rpb = (M + target - 1) / target;
  const int64_t min_rpb = (int64_t)g.rpi * 8 > 16 ? (int64_t)g.rpi * 8 : 16;
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

// Reduce per-thread 8-channel partials (a, b) over the `rpi` row-threads of a column and store one
// partial per channel per workgroup: slab_a[blockIdx.x][c], slab_b[blockIdx.x][c].
__device__ __forceinline__ void block_col_reduce_store(float (&a)[8], float (&b)[8], int tx, int ty, int cols,
                                                       int rpi, int vcol, int C, float* slab_a, float* slab_b) {
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
    store8(slab_a + (int64_t)blockIdx.x * C + vcol * 8, a);
    store8(slab_b + (int64_t)blockIdx.x * C + vcol * 8, b);
  }
}

// Sum the [nrb][C] slabs for 64 channels per workgroup: kFinThreads = 64 channels x 16 row-lanes.
constexpr int kStemBlocks = 2048;  // stem pool+BN backward grid (slab rows of its reduce phase)
constexpr int kFinThreads = 1024;
// Rows are `ld` floats apart (C for the [nrb][C] slabs, 2C for a conv epilogue's [R][2][C] table).
// CLEAR: zero every entry after reading it (the epilogue table must be zero for its next conv).
template <bool CLEAR = false>
__device__ __forceinline__ void slab_sum(float* __restrict__ pa, float* __restrict__ pb, int nrb, int64_t ld,
                                         int C, int c, float& sa, float& sb) {
  __shared__ float red_a[kFinThreads], red_b[kFinThreads];
  const int l = threadIdx.x >> 6;  // 0..15
  float a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = b[u] = 0.f;
  if (c < C) {
    // 8 independent loads per slab in flight per lane: the slab rows were just written (L2/MALL
    // hits), so this pass is latency-bound — depth, not bandwidth, sets its time
    int r = l;
    for (; r + 7 * 16 < nrb; r += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] += pa[(int64_t)(r + 16 * u) * ld + c];
        b[u] += pb[(int64_t)(r + 16 * u) * ld + c];
      }
    }
    for (; r < nrb; r += 16) {
      a[0] += pa[(int64_t)r * ld + c];
      b[0] += pb[(int64_t)r * ld + c];
    }
    if (CLEAR)
      for (r = l; r < nrb; r += 16) pa[(int64_t)r * ld + c] = pb[(int64_t)r * ld + c] = 0.f;
  }
  const float a0 = (a[0] + a[1]) + (a[2] + a[3]), a1 = (a[4] + a[5]) + (a[6] + a[7]);
  const float b0 = (b[0] + b[1]) + (b[2] + b[3]), b1 = (b[4] + b[5]) + (b[6] + b[7]);
  red_a[threadIdx.x] = a0 + a1;
  red_b[threadIdx.x] = b0 + b1;
  __syncthreads();
  const int ch = threadIdx.x & 63;
  sa = sb = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    sa += red_a[k * 64 + ch];
    sb += red_b[k * 64 + ch];
  }
}

// ---------------------------------------------------------------- forward statistics
__global__ void __launch_bounds__(kThreads) bn_stats_kernel(const bf16_t* __restrict__ x, int64_t M, int C, int cols,
                                                            int rpi, int64_t rpb, float* __restrict__ slab) {
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
    int64_t r = r0 + ty;
    for (; r + 7 * rpi < r1; r += 8 * rpi) {  // 8 independent 16-B loads in flight per lane
      float v[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) load8(x + (r + u * rpi) * C + vcol * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[u][j] - piv[j];
          s1[j] += d;
          s2[j] += d * d;
        }
    }
    for (; r < r1; r += rpi) {
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
  block_col_reduce_store(s1, s2, tx, ty, cols, rpi, vcol, C, slab, slab + (int64_t)gridDim.x * C);
}

__device__ __forceinline__ float param_at(const float* f, const bf16_t* b, int c, float dflt) {
  return f ? f[c] : (b ? bf2f(b[c]) : dflt);
}

// ---------------------------------------------------------------- forward finalize
// TRAIN: statistics from the slabs; eval: from the running statistics.  Writes scale/shift [C].
template <bool TRAIN, bool TABLE = false>
__global__ void __launch_bounds__(kFinThreads) bn_finalize_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ pivot, float* __restrict__ slab, int nrb,
    int64_t M, int C, const float* __restrict__ gamma_f, const bf16_t* __restrict__ gamma_b, const float* __restrict__ beta_f,
    const bf16_t* __restrict__ beta_b, float* __restrict__ running_mean, float* __restrict__ running_var,
    float momentum, float eps, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ scale, float* __restrict__ shift, int64_t* __restrict__ num_batches) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  // the module's num_batches_tracked += 1 rides on this launch (one fewer kernel per BN layer)
  if (TRAIN && num_batches && blockIdx.x == 0 && threadIdx.x == 0) *num_batches += 1;
  float s1 = 0.f, s2 = 0.f;
  if (TRAIN) {
    if (TABLE) slab_sum<true>(slab, slab + C, nrb, 2 * (int64_t)C, C, c, s1, s2);  // conv epilogue table
    else slab_sum(slab, slab + (int64_t)nrb * C, nrb, C, C, c, s1, s2);
  }
  if (threadIdx.x >= 64 || c >= C) return;
  float mean, invstd;
  if (TRAIN) {
    const float invM = 1.f / (float)M;
    const float m1 = s1 * invM;
    const float var = fmaxf(s2 * invM - m1 * m1, 0.f);
    mean = (pivot ? pivot[c] : bf2f(x[c])) + m1;
    invstd = rsqrtf(var + eps);
    save_mean[c] = mean;
    save_invstd[c] = invstd;
    if (running_mean) {
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
    }
  } else {
    mean = running_mean[c];
    invstd = rsqrtf(running_var[c] + eps);
  }
  const float g = param_at(gamma_f, gamma_b, c, 1.f), b = param_at(beta_f, beta_b, c, 0.f);
  scale[c] = g * invstd;
  shift[c] = b - mean * g * invstd;
}

// ---------------------------------------------------------------- forward apply
// LDS tables are sized by C (dynamic shared memory): a fixed kMaxC table (16-40 KB) capped residency
// at 4 workgroups per CU for the backward apply, too few bytes in flight for HBM3E.
template <bool RES, bool RELU>
__device__ __forceinline__ void bn_apply_vec(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                             bf16_t* __restrict__ y, uint8_t* __restrict__ bits, int64_t v, int c0,
                                             const float* s_scale, const float* s_shift, const float (&a_in)[8],
                                             const float (&r)[8]) {
  float a[8];
  const f32x4 sc0 = *reinterpret_cast<const f32x4*>(s_scale + c0), sc1 = *reinterpret_cast<const f32x4*>(s_scale + c0 + 4);
  const f32x4 sh0 = *reinterpret_cast<const f32x4*>(s_shift + c0), sh1 = *reinterpret_cast<const f32x4*>(s_shift + c0 + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] = a_in[j] * sc0[j] + sh0[j];
    a[j + 4] = a_in[j + 4] * sc1[j] + sh1[j];
  }
  if (RES) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += r[j];
  }
  if (RELU) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m |= (a[j] > 0.f ? 1u : 0u) << j;
      a[j] = fmaxf(a[j], 0.f);
    }
    if (bits) bits[v] = (uint8_t)m;  // one byte per 8 channels: the backward's ReLU mask
  }
  store8(y + v * 8, a);
}

template <bool RES, bool RELU>
__global__ void __launch_bounds__(kThreads) bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                            bf16_t* __restrict__ y, int64_t M, int C,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            uint8_t* __restrict__ bits) {
  extern __shared__ __attribute__((aligned(16))) float s_tab[];  // [2][C]
  float* s_scale = s_tab;
  float* s_shift = s_tab + C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    s_scale[c] = scale[c];
    s_shift[c] = shift[c];
  }
  __syncthreads();
  const int cv = C / 8;
  const int64_t nvec = M * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; v + stride < nvec; v += 2 * stride) {  // two vectors (2-3 loads each) in flight per lane
    float a0[8], a1[8], r0[8], r1[8];
    load8(x + v * 8, a0);
    load8(x + (v + stride) * 8, a1);
    if (RES) {
      load8(res + v * 8, r0);
      load8(res + (v + stride) * 8, r1);
    }
    bn_apply_vec<RES, RELU>(x, res, y, bits, v, (int)(v % cv) * 8, s_scale, s_shift, a0, r0);
    bn_apply_vec<RES, RELU>(x, res, y, bits, v + stride, (int)((v + stride) % cv) * 8, s_scale, s_shift, a1, r1);
  }
  if (v < nvec) {
    float a0[8], r0[8];
    load8(x + v * 8, a0);
    if (RES) load8(res + v * 8, r0);
    bn_apply_vec<RES, RELU>(x, res, y, bits, v, (int)(v % cv) * 8, s_scale, s_shift, a0, r0);
  }
}

// Wave-contiguous register-coefficient variant (every ResNet shape).  One wave iteration covers 256
// consecutive 8-channel vectors: four coalesced 1-KB instructions per tensor, and the 256 ReLU-mask
// bytes of the iteration leave as ONE 4-byte store per lane (regrouped with four shuffles) instead of
// 256 one-byte stores — the byte stores cost the BN+residual+ReLU apply 15-20 % of its time on the
// ResNet-50 bs512 shapes (4.3-4.7 -> 5.3-5.6 TB/s, tools/bnlab/apply_lab.hip).  Outputs are written
// with nontemporal stores (they are next read by another kernel, not this one: +2-3 %).  A lane's
// coefficients live in registers: its channel group is fixed when 64 % cv == 0 and cycles through
// NS = cv / 64 groups when cv is a multiple of 64 (up to 4: C = 2048).
constexpr int kWaveVec = 256;  // vectors per wave iteration

inline int wave_sets(int cv) {
  if (cv <= 0) return 0;  // C < 8: no register-table path (and no division by zero)
  if (cv <= 64) return 64 % cv == 0 ? 1 : 0;
  return (cv % 64 == 0 && cv / 64 <= 4) ? cv / 64 : 0;
}
inline int wave_grid(int64_t nvec) {
  int64_t g = (nvec + kWaveVec * (kThreads / 64) - 1) / (kWaveVec * (kThreads / 64));
  if (g > 2048) g = 2048;
  return g < 1 ? 1 : (int)g;
}

__device__ __forceinline__ void store8_nt(bf16_t* p, const float (&v)[8]) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
  __builtin_nontemporal_store(r, reinterpret_cast<u16x8*>(p));
}

// mask bytes m_u of vectors base + 64u + lane (u < 4, packed w = m_0 | m_1 << 8 | ...) -> the 4-byte
// word of vectors base + 4 lane .. 4 lane + 3 (lane l reads byte l >> 4 of lanes 4l .. 4l + 3 mod 64)
__device__ __forceinline__ uint32_t mask_words_out(uint32_t w, int lane) {
  uint32_t out = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t t = (uint32_t)__shfl((int)w, (4 * lane + k) & 63, 64);
    out |= ((t >> (8 * (lane >> 4))) & 0xFFu) << (8 * k);
  }
  return out;
}
// inverse: lane l holds the word of vectors base + 4l .. 4l + 3; returns byte u of vector 64u + lane
__device__ __forceinline__ uint32_t mask_words_in(uint32_t word, int lane) {
  uint32_t w = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t t = (uint32_t)__shfl((int)word, 16 * u + (lane >> 2), 64);
    w |= ((t >> (8 * (lane & 3))) & 0xFFu) << (8 * u);
  }
  return w;
}

template <bool RES, bool RELU>
__device__ __forceinline__ uint32_t bn_apply8(float (&a)[8], const float (&xv)[8], const float (&rv)[8],
                                              const float (&sc)[8], const float (&sh)[8]) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = fmaf(xv[j], sc[j], sh[j]) + (RES ? rv[j] : 0.f);
    if (RELU) {
      m |= (a[j] > 0.f ? 1u : 0u) << j;
      a[j] = fmaxf(a[j], 0.f);
    }
  }
  return m;
}

// RBN: the residual is itself a batch-normalised tensor, res * scale2 + shift2 (a bottleneck's
// downsample branch applied inside the block's output kernel: its BN output is never stored).
template <bool RES, bool RELU, int NS, bool RBN = false>
__global__ void __launch_bounds__(kThreads) bn_apply_wave_kernel(const bf16_t* __restrict__ x,
                                                                 const bf16_t* __restrict__ res,
                                                                 bf16_t* __restrict__ y, int64_t M, int C,
                                                                 const float* __restrict__ scale,
                                                                 const float* __restrict__ shift,
                                                                 uint8_t* __restrict__ bits,
                                                                 const float* __restrict__ scale2,
                                                                 const float* __restrict__ shift2) {
  const int cv = C / 8, lane = threadIdx.x & 63;
  const int64_t nvec = M * cv;
  const int64_t tw = (int64_t)gridDim.x * (kThreads / 64);
  constexpr int NS2 = RBN ? NS : 1;
  float sc[NS][8], sh[NS][8], sc2[NS2][8], sh2[NS2][8];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c0 = ((64 * s + lane) % cv) * 8;
    load8(scale + c0, sc[s]);
    load8(shift + c0, sh[s]);
    if constexpr (RBN) {
      load8(scale2 + c0, sc2[s]);
      load8(shift2 + c0, sh2[s]);
    }
  }
  int64_t base = ((int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * kWaveVec;
  for (; base + kWaveVec <= nvec; base += tw * kWaveVec) {
    u16x8 xa[4], ra[4];  // loads kept packed until used (register budget: 4 vectors x 2 tensors in flight)
#pragma unroll
    for (int u = 0; u < 4; ++u) xa[u] = *reinterpret_cast<const u16x8*>(x + (base + 64 * u + lane) * 8);
    if (RES) {
#pragma unroll
      for (int u = 0; u < 4; ++u) ra[u] = *reinterpret_cast<const u16x8*>(res + (base + 64 * u + lane) * 8);
    }
    uint32_t w = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float o[8], a[8], r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = bf2f(xa[u][j]);
        if constexpr (RBN) r[j] = fmaf(bf2f(ra[u][j]), sc2[u % NS][j], sh2[u % NS][j]);
        else r[j] = RES ? bf2f(ra[u][j]) : 0.f;
      }
      w |= bn_apply8<RES, RELU>(o, a, r, sc[u % NS], sh[u % NS]) << (8 * u);
      store8_nt(y + (base + 64 * u + lane) * 8, o);
    }
    if (RELU && bits) {
      const uint32_t out = mask_words_out(w, lane);
      __builtin_nontemporal_store(out, reinterpret_cast<uint32_t*>(bits + base) + lane);
    }
  }
  // the last partial iteration (nvec % 256 vectors, one wave): a byte per vector
  for (int64_t v = base + lane; base < nvec && v < nvec; v += 64) {
    const int c0 = (int)(v % cv) * 8;
    float s1[8], h1[8], a[8], r[8], o[8];
    load8(scale + c0, s1);
    load8(shift + c0, h1);
    load8(x + v * 8, a);
    if (RES) load8(res + v * 8, r);
    if constexpr (RBN) {
      float s2[8], h2[8];
      load8(scale2 + c0, s2);
      load8(shift2 + c0, h2);
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = fmaf(r[j], s2[j], h2[j]);
    }
    const uint32_t m = bn_apply8<RES, RELU>(o, a, r, s1, h1);
    if (RELU && bits) bits[v] = (uint8_t)m;
    store8(y + v * 8, o);
  }
}

// ---------------------------------------------------------------- backward reduction
// MASK: 0 no ReLU; 1 ReLU mask from the saved output y; 2 ReLU mask recomputed from x and the
// forward's per-channel scale/shift (BN+ReLU without residual: y is never saved or re-read);
// 3 ReLU mask from the bit mask written by the forward apply (BN+residual+ReLU: 1 bit instead of
// re-reading the 16-bit output, in both backward passes).
template <int MASK>
__device__ __forceinline__ void relu_mask(float (&g)[8], const bf16_t* __restrict__ y, const float (&xv)[8],
                                          const float* __restrict__ sc, const float* __restrict__ sh, int64_t off,
                                          int c0) {
  if constexpr (MASK == 3) {
    const uint32_t m = reinterpret_cast<const uint8_t*>(y)[off >> 3];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (m >> j) & 1u ? g[j] : 0.f;
  } else if constexpr (MASK == 1) {
    const u16x8 yr = *reinterpret_cast<const u16x8*>(y + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = bf2f(yr[j]) > 0.f ? g[j] : 0.f;
  } else if constexpr (MASK == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = xv[j] * sc[c0 + j] + sh[c0 + j] > 0.f ? g[j] : 0.f;
  }
}

// In-launch finalize of the backward reduce (replaces bn_bwd_finalize_kernel's separate launch).
//
// Why: a wide wgrad GEMM workgroup on the side stream holds 144 KB of LDS and ~470 of a SIMD's 512
// VGPRs, so a critical-path kernel launched beside it waits for a whole CU to drain; the finalize's
// 1024-thread workgroups waited longest (9 us alone, ~145 us per call beside the wgrads at bs 640).
// How: every reduce block adds its per-channel partials into a small persistent table [R][2][C] with
// no-return float atomics (executed at the memory side, so coherent across the 8 XCDs without
// fences), drains them (vmcnt(0)) and draws a ticket; the block that draws the last ticket reads AND
// re-zeroes the table with atomic exchanges (also memory-side: no stale L2 copy can be read), sums
// the R rows, writes dgamma / dbeta / the apply coefficients and resets the ticket.  The table and
// ticket are zero on entry (allocated zeroed; every call leaves them zero).
struct BwdFin {
  float* table;   // [R][2][C] fp32, zero on entry and exit
  unsigned* ticket;
  int R;
  const float* invstd;
  const float* gamma_f;
  const bf16_t* gamma_b;
  float* dgamma_f;
  bf16_t* dgamma_b;
  float* dbeta_f;
  bf16_t* dbeta_b;
  float* coef;
};

__device__ __forceinline__ void bwd_fused_finish(float (&a)[8], float (&b)[8], int tx, int ty, int cols, int rpi,
                                                 int vcol, int C, int64_t M, const float* __restrict__ mean,
                                                 const BwdFin& f) {
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
    float* ra = f.table + (int64_t)(blockIdx.x % f.R) * 2 * C + vcol * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __hip_atomic_fetch_add(ra + j, a[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(ra + C + j, b[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every adding wave: its adds are performed
  __syncthreads();
  unsigned* s_flag = reinterpret_cast<unsigned*>(s_a);
  if (threadIdx.x == 0)
    s_flag[0] = __hip_atomic_fetch_add(f.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                gridDim.x * gridDim.y - 1;
  __syncthreads();
  if (!s_flag[0]) return;
  __syncthreads();  // everyone has read the flag before s_a is reused below
  // last block: thread t sums channel vector (t % cv) over table rows t / cv, t / cv + rpt, ...
  const int cv = C / 8;
  const int rpt = kThreads / cv;  // >= 1 (C <= 2048)
  const int v = threadIdx.x % cv, r0 = threadIdx.x / cv;
  float sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.f;
  if (r0 < rpt) {
    for (int r = r0; r < f.R; r += rpt) {
      float* ra = f.table + (int64_t)r * 2 * C + v * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sa[j] += __hip_atomic_exchange(ra + j, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sb[j] += __hip_atomic_exchange(ra + C + j, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s_a[threadIdx.x * 8 + j] = sa[j];
    s_b[threadIdx.x * 8 + j] = sb[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(f.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x >= cv) return;
  for (int k = 1; k < rpt; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[j] += s_a[(k * cv + v) * 8 + j];
      sb[j] += s_b[(k * cv + v) * 8 + j];
    }
  }
  const float invM = 1.f / (float)M;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = v * 8 + j;
    const float is = f.invstd[c], mu = mean[c];
    const float g = param_at(f.gamma_f, f.gamma_b, c, 1.f);
    const float sdz = sa[j], dg = sb[j] * is;
    if (f.dgamma_f) f.dgamma_f[c] = dg;
    if (f.dgamma_b) f.dgamma_b[c] = f2bf(dg);
    if (f.dbeta_f) f.dbeta_f[c] = sdz;
    if (f.dbeta_b) f.dbeta_b[c] = f2bf(sdz);
    const float A = g * is;
    const float B = -A * is * dg * invM;
    f.coef[c] = A;
    f.coef[C + c] = B;
    f.coef[2 * C + c] = -A * sdz * invM - B * mu;
  }
}

template <int MASK, bool FUSED>
__global__ void __launch_bounds__(kThreads) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ x,
                                                                 const bf16_t* __restrict__ y,
                                                                 const float* __restrict__ ss,
                                                                 const float* __restrict__ mean, int64_t M, int C,
                                                                 int cols, int rpi, int64_t rpb,
                                                                 float* __restrict__ slab, BwdFin fin) {
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(r0 + rpb, M);
  const int c0 = vcol * 8;
  float sa[8], sb[8], mu[8], rsc[8], rsh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.f;
  if (active) {
    load8(mean + c0, mu);
    // a lane's channel group never changes: the MASK 2 scale/shift live in registers, not in
    // per-element global loads
    if constexpr (MASK == 2) {
      load8(ss + c0, rsc);
      load8(ss + C + c0, rsh);
    }
    int64_t r = r0 + ty;
    for (; r + 3 * rpi < r1; r += 4 * rpi) {  // 4 rows x 2 tensors = 8 loads in flight per lane
      float g[4][8], xv[4][8];
      uint32_t mb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t off = (r + u * rpi) * C + c0;
        load8(dy + off, g[u]);
        load8(x + off, xv[u]);
        if constexpr (MASK == 3) mb[u] = reinterpret_cast<const uint8_t*>(y)[off >> 3];  // in flight with dy/x
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (MASK == 3) {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[u][j] = (mb[u] >> j) & 1u ? g[u][j] : 0.f;
        } else if constexpr (MASK == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[u][j] = fmaf(xv[u][j], rsc[j], rsh[j]) > 0.f ? g[u][j] : 0.f;
        } else {
          relu_mask<MASK>(g[u], y, xv[u], ss, ss + C, (r + u * rpi) * C + c0, c0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sa[j] += g[u][j];
          sb[j] += g[u][j] * (xv[u][j] - mu[j]);
        }
      }
    }
    for (; r < r1; r += rpi) {
      const int64_t off = r * C + c0;
      float g[8], xv[8];
      load8(dy + off, g);
      load8(x + off, xv);
      relu_mask<MASK>(g, y, xv, ss, ss + C, off, c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sa[j] += g[j];
        sb[j] += g[j] * (xv[j] - mu[j]);
      }
    }
  }
  if constexpr (FUSED) bwd_fused_finish(sa, sb, tx, ty, cols, rpi, vcol, C, M, mean, fin);
  else block_col_reduce_store(sa, sb, tx, ty, cols, rpi, vcol, C, slab, slab + (int64_t)gridDim.x * C);
}

// Two BNs fed by one masked gradient (a downsample bottleneck's relu(bn(x) + bn2(x2)), MASK 3): one
// pass over dy, the bit mask, x and x2.  sum(dz) is shared; sum(dz (x - mean)) per input.
__global__ void __launch_bounds__(kThreads) bn_bwd_reduce_dual_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
    const uint8_t* __restrict__ bits, const float* __restrict__ mean, const float* __restrict__ mean2, int64_t M,
    int C, int cols, int rpi, int64_t rpb, float* __restrict__ slab, float* __restrict__ slab2) {
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(r0 + rpb, M);
  const int c0 = vcol * 8;
  float sa[8], sb[8], sb2[8], mu[8], mu2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = sb2[j] = 0.f;
  if (active) {
    load8(mean + c0, mu);
    load8(mean2 + c0, mu2);
    int64_t r = r0 + ty;
    for (; r + 3 * rpi < r1; r += 4 * rpi) {  // 4 rows x 3 tensors in flight per lane
      u16x8 ga[4], xa[4], x2a[4];
      uint32_t mb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t off = (r + u * rpi) * C + c0;
        ga[u] = *reinterpret_cast<const u16x8*>(dy + off);
        xa[u] = *reinterpret_cast<const u16x8*>(x + off);
        x2a[u] = *reinterpret_cast<const u16x8*>(x2 + off);
        mb[u] = bits[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = (mb[u] >> j) & 1u ? bf2f(ga[u][j]) : 0.f;
          sa[j] += g;
          sb[j] += g * (bf2f(xa[u][j]) - mu[j]);
          sb2[j] += g * (bf2f(x2a[u][j]) - mu2[j]);
        }
      }
    }
    for (; r < r1; r += rpi) {
      const int64_t off = r * C + c0;
      float g[8], xv[8], x2v[8];
      load8(dy + off, g);
      load8(x + off, xv);
      load8(x2 + off, x2v);
      const uint32_t m = bits[off >> 3];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gm = (m >> j) & 1u ? g[j] : 0.f;
        sa[j] += gm;
        sb[j] += gm * (xv[j] - mu[j]);
        sb2[j] += gm * (x2v[j] - mu2[j]);
      }
    }
  }
  float sa2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa2[j] = sa[j];  // (the store reduces its arguments in place)
  block_col_reduce_store(sa, sb, tx, ty, cols, rpi, vcol, C, slab, slab + (int64_t)gridDim.x * C);
  __syncthreads();
  block_col_reduce_store(sa2, sb2, tx, ty, cols, rpi, vcol, C, slab2, slab2 + (int64_t)gridDim.x * C);
}

// dgamma = invstd * sum(dz (x-mean)), dbeta = sum(dz);  coefficients for dx = A*dz + B*x + Cc.
// TABLE: the sums come from a dgrad epilogue's [nrb][2][C] table (gemm_epi.h bst_*), re-zeroed here.
template <bool TABLE = false>
__global__ void __launch_bounds__(kFinThreads) bn_bwd_finalize_kernel(
    float* __restrict__ slab, int nrb, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma_f, const bf16_t* __restrict__ gamma_b,
    float* __restrict__ dgamma_f, bf16_t* __restrict__ dgamma_b, float* __restrict__ dbeta_f,
    bf16_t* __restrict__ dbeta_b, float* __restrict__ coef) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float sdz, sdx;
  if (TABLE) slab_sum<true>(slab, slab + C, nrb, 2 * (int64_t)C, C, c, sdz, sdx);
  else slab_sum(slab, slab + (int64_t)nrb * C, nrb, C, C, c, sdz, sdx);
  if (threadIdx.x >= 64 || c >= C) return;
  const float is = invstd[c], mu = mean[c];
  const float g = param_at(gamma_f, gamma_b, c, 1.f);
  const float dg = sdx * is;
  if (dgamma_f) dgamma_f[c] = dg;
  if (dgamma_b) dgamma_b[c] = f2bf(dg);
  if (dbeta_f) dbeta_f[c] = sdz;
  if (dbeta_b) dbeta_b[c] = f2bf(sdz);
  const float invM = 1.f / (float)M;
  const float A = g * is;
  const float B = -A * is * dg * invM;
  coef[c] = A;
  coef[C + c] = B;
  coef[2 * C + c] = -A * sdz * invM - B * mu;
}

template <int MASK, bool DRES>
__device__ __forceinline__ void bn_bwd_apply_vec(const bf16_t* __restrict__ y, const float* s_co, int C, int64_t v,
                                                 int c0, float (&g)[8], float (&xv)[8], bf16_t* __restrict__ dx,
                                                 bf16_t* __restrict__ dres) {
  relu_mask<MASK>(g, y, xv, s_co + 3 * C, s_co + 4 * C, v * 8, c0);
  if (DRES) store8(dres + v * 8, g);
  const float* s_A = s_co;
  const float* s_B = s_co + C;
  const float* s_C = s_co + 2 * C;
#pragma unroll
  for (int j = 0; j < 8; ++j) xv[j] = s_A[c0 + j] * g[j] + s_B[c0 + j] * xv[j] + s_C[c0 + j];
  store8(dx + v * 8, xv);
}

template <int MASK, bool DRES>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                                const bf16_t* __restrict__ x,
                                                                const bf16_t* __restrict__ y,
                                                                const float* __restrict__ ss, int64_t M, int C,
                                                                const float* __restrict__ coef,
                                                                bf16_t* __restrict__ dx, bf16_t* __restrict__ dres) {
  extern __shared__ __attribute__((aligned(16))) float s_co[];  // [5][C]: A, B, Cc, scale, shift
  for (int c = threadIdx.x; c < 3 * C; c += blockDim.x) s_co[c] = coef[c];
  if (MASK == 2)
    for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) s_co[3 * C + c] = ss[c];
  __syncthreads();
  const int cv = C / 8;
  const int64_t nvec = M * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; v + stride < nvec; v += 2 * stride) {  // two vectors in flight per lane
    float g0[8], x0[8], g1[8], x1[8];
    load8(dy + v * 8, g0);
    load8(x + v * 8, x0);
    load8(dy + (v + stride) * 8, g1);
    load8(x + (v + stride) * 8, x1);
    bn_bwd_apply_vec<MASK, DRES>(y, s_co, C, v, (int)(v % cv) * 8, g0, x0, dx, dres);
    bn_bwd_apply_vec<MASK, DRES>(y, s_co, C, v + stride, (int)((v + stride) % cv) * 8, g1, x1, dx, dres);
  }
  if (v < nvec) {
    float g0[8], x0[8];
    load8(dy + v * 8, g0);
    load8(x + v * 8, x0);
    bn_bwd_apply_vec<MASK, DRES>(y, s_co, C, v, (int)(v % cv) * 8, g0, x0, dx, dres);
  }
}

// Wave-contiguous register-coefficient backward apply (layout and mask words as bn_apply_wave_kernel:
// the 256 mask bytes of an iteration arrive as one 4-byte load per lane; dx / dres are written with
// nontemporal stores).
template <int MASK, bool DRES, int NS>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_wave_kernel(const bf16_t* __restrict__ dy,
                                                                     const bf16_t* __restrict__ x,
                                                                     const bf16_t* __restrict__ y,
                                                                     const float* __restrict__ ss, int64_t M, int C,
                                                                     const float* __restrict__ coef,
                                                                     bf16_t* __restrict__ dx,
                                                                     bf16_t* __restrict__ dres) {
  const int cv = C / 8, lane = threadIdx.x & 63;
  const int64_t nvec = M * cv;
  const int64_t tw = (int64_t)gridDim.x * (kThreads / 64);
  const uint8_t* mbytes = reinterpret_cast<const uint8_t*>(y);  // MASK 3: the bit mask
  float cA[NS][8], cB[NS][8], cC[NS][8], sc[NS][8], sh[NS][8];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c0 = ((64 * s + lane) % cv) * 8;
    load8(coef + c0, cA[s]);
    load8(coef + C + c0, cB[s]);
    load8(coef + 2 * C + c0, cC[s]);
    if constexpr (MASK == 2) {
      load8(ss + c0, sc[s]);
      load8(ss + C + c0, sh[s]);
    }
  }
  auto one = [&](float (&g)[8], float (&xv)[8], uint32_t mb, const bf16_t* yv, int s, bf16_t* dxp, bf16_t* drp,
                 bool nt) {
    if constexpr (MASK == 3) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (mb >> j) & 1u ? g[j] : 0.f;
    } else if constexpr (MASK == 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(xv[j], sc[s][j], sh[s][j]) > 0.f ? g[j] : 0.f;
    } else if constexpr (MASK == 1) {
      const u16x8 yr = *reinterpret_cast<const u16x8*>(yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = bf2f(yr[j]) > 0.f ? g[j] : 0.f;
    }
    if (DRES) {
      if (nt) store8_nt(drp, g);
      else store8(drp, g);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = fmaf(cA[s][j], g[j], fmaf(cB[s][j], xv[j], cC[s][j]));
    if (nt) store8_nt(dxp, xv);
    else store8(dxp, xv);
  };
  int64_t base = ((int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * kWaveVec;
  for (; base + kWaveVec <= nvec; base += tw * kWaveVec) {
    u16x8 ga[4], xa[4];  // packed until used
    uint32_t word = 0;
    if constexpr (MASK == 3) word = reinterpret_cast<const uint32_t*>(mbytes + base)[lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t v = base + 64 * u + lane;
      ga[u] = *reinterpret_cast<const u16x8*>(dy + v * 8);
      xa[u] = *reinterpret_cast<const u16x8*>(x + v * 8);
    }
    const uint32_t w = MASK == 3 ? mask_words_in(word, lane) : 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t v = base + 64 * u + lane;
      float g[8], xv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g[j] = bf2f(ga[u][j]);
        xv[j] = bf2f(xa[u][j]);
      }
      one(g, xv, w >> (8 * u), y + v * 8, u % NS, dx + v * 8, DRES ? dres + v * 8 : nullptr, true);
    }
  }
  for (int64_t v = base + lane; base < nvec && v < nvec; v += 64) {  // last partial iteration
    // (the channel group of a tail vector is its own: (v % cv) — reload that group's coefficients)
    const int c0 = (int)(v % cv) * 8;
    load8(coef + c0, cA[0]);
    load8(coef + C + c0, cB[0]);
    load8(coef + 2 * C + c0, cC[0]);
    if constexpr (MASK == 2) {
      load8(ss + c0, sc[0]);
      load8(ss + C + c0, sh[0]);
    }
    float g[8], xv[8];
    load8(dy + v * 8, g);
    load8(x + v * 8, xv);
    one(g, xv, MASK == 3 ? (uint32_t)mbytes[v] : 0u, y + v * 8, 0, dx + v * 8, DRES ? dres + v * 8 : nullptr,
        false);
  }
}

// A/B switch read once per process (PDA_BN_LDS_TABLES=1 forces the LDS-table kernels)
inline bool lds_tables_forced() {
  static const bool v = [] {
    const char* e = getenv("PDA_BN_LDS_TABLES");
    return e && e[0] == '1';
  }();
  return v;
}

template <int NS>
void launch_apply_wave(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int C, const float* scale,
                       const float* shift, bool relu, uint8_t* bits, hipStream_t st) {
  const int grid = wave_grid(M * C / 8);
  const float* n = nullptr;
  if (res && relu) bn_apply_wave_kernel<true, true, NS><<<grid, kThreads, 0, st>>>(x, res, y, M, C, scale, shift, bits, n, n);
  else if (res) bn_apply_wave_kernel<true, false, NS><<<grid, kThreads, 0, st>>>(x, res, y, M, C, scale, shift, nullptr, n, n);
  else if (relu) bn_apply_wave_kernel<false, true, NS><<<grid, kThreads, 0, st>>>(x, res, y, M, C, scale, shift, bits, n, n);
  else bn_apply_wave_kernel<false, false, NS><<<grid, kThreads, 0, st>>>(x, res, y, M, C, scale, shift, nullptr, n, n);
}

template <int NS>
void launch_apply_dual_wave(const bf16_t* x, const bf16_t* x2, bf16_t* y, int64_t M, int C, const float* ss,
                            const float* ss2, uint8_t* bits, hipStream_t st) {
  const int grid = wave_grid(M * C / 8);
  bn_apply_wave_kernel<true, true, NS, true><<<grid, kThreads, 0, st>>>(x, x2, y, M, C, ss, ss + C, bits, ss2,
                                                                        ss2 + C);
}

hipError_t launch_apply(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int C, const float* scale,
                        const float* shift, bool relu, uint8_t* bits, hipStream_t st) {
  const int ns = lds_tables_forced() ? 0 : wave_sets(C / 8);
  if (ns == 1) launch_apply_wave<1>(x, res, y, M, C, scale, shift, relu, bits, st);
  else if (ns == 2) launch_apply_wave<2>(x, res, y, M, C, scale, shift, relu, bits, st);
  else if (ns == 4) launch_apply_wave<4>(x, res, y, M, C, scale, shift, relu, bits, st);
  if (ns == 1 || ns == 2 || ns == 4) return hipGetLastError();
  const int grid = ew_grid(M * C / 8);
  const size_t lds = 2 * (size_t)C * sizeof(float);
  if (res && relu) bn_apply_kernel<true, true><<<grid, kThreads, lds, st>>>(x, res, y, M, C, scale, shift, bits);
  else if (res) bn_apply_kernel<true, false><<<grid, kThreads, lds, st>>>(x, res, y, M, C, scale, shift, nullptr);
  else if (relu) bn_apply_kernel<false, true><<<grid, kThreads, lds, st>>>(x, res, y, M, C, scale, shift, bits);
  else bn_apply_kernel<false, false><<<grid, kThreads, lds, st>>>(x, res, y, M, C, scale, shift, nullptr);
  return hipGetLastError();
}

// Dual backward apply (MASK 3): dx = A g + B x + Cc and dx2 = A2 g + B2 x2 + C2 from one read of dy
// and the mask; register coefficient tables for both BNs (NS <= 2).
template <int NS>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_dual_wave_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
    const uint8_t* __restrict__ bits, int64_t M, int C, const float* __restrict__ coef,
    const float* __restrict__ coef2, bf16_t* __restrict__ dx, bf16_t* __restrict__ dx2) {
  const int cv = C / 8, lane = threadIdx.x & 63;
  const int64_t nvec = M * cv;
  const int64_t tw = (int64_t)gridDim.x * (kThreads / 64);
  float cA[NS][8], cB[NS][8], cC[NS][8], dA[NS][8], dB[NS][8], dC[NS][8];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c0 = ((64 * s + lane) % cv) * 8;
    load8(coef + c0, cA[s]);
    load8(coef + C + c0, cB[s]);
    load8(coef + 2 * C + c0, cC[s]);
    load8(coef2 + c0, dA[s]);
    load8(coef2 + C + c0, dB[s]);
    load8(coef2 + 2 * C + c0, dC[s]);
  }
  int64_t base = ((int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * kWaveVec;
  for (; base + kWaveVec <= nvec; base += tw * kWaveVec) {
    u16x8 ga[4], xa[4], x2a[4];
    const uint32_t word = reinterpret_cast<const uint32_t*>(bits + base)[lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t v = base + 64 * u + lane;
      ga[u] = *reinterpret_cast<const u16x8*>(dy + v * 8);
      xa[u] = *reinterpret_cast<const u16x8*>(x + v * 8);
      x2a[u] = *reinterpret_cast<const u16x8*>(x2 + v * 8);
    }
    const uint32_t w = mask_words_in(word, lane);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t v = base + 64 * u + lane;
      const int s = u % NS;
      const uint32_t mb = w >> (8 * u);
      float o[8], o2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = (mb >> j) & 1u ? bf2f(ga[u][j]) : 0.f;
        o[j] = fmaf(cA[s][j], g, fmaf(cB[s][j], bf2f(xa[u][j]), cC[s][j]));
        o2[j] = fmaf(dA[s][j], g, fmaf(dB[s][j], bf2f(x2a[u][j]), dC[s][j]));
      }
      store8_nt(dx + v * 8, o);
      store8_nt(dx2 + v * 8, o2);
    }
  }
  for (int64_t v = base + lane; base < nvec && v < nvec; v += 64) {  // last partial iteration
    const int c0 = (int)(v % cv) * 8;
    float a[8], b[8], c[8], a2[8], b2[8], c2[8], g[8], xv[8], x2v[8], o[8], o2[8];
    load8(coef + c0, a);
    load8(coef + C + c0, b);
    load8(coef + 2 * C + c0, c);
    load8(coef2 + c0, a2);
    load8(coef2 + C + c0, b2);
    load8(coef2 + 2 * C + c0, c2);
    load8(dy + v * 8, g);
    load8(x + v * 8, xv);
    load8(x2 + v * 8, x2v);
    const uint32_t mb = bits[v];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gm = (mb >> j) & 1u ? g[j] : 0.f;
      o[j] = fmaf(a[j], gm, fmaf(b[j], xv[j], c[j]));
      o2[j] = fmaf(a2[j], gm, fmaf(b2[j], x2v[j], c2[j]));
    }
    store8(dx + v * 8, o);
    store8(dx2 + v * 8, o2);
  }
}

// ---------------------------------------------------------------- stem: maxpool(3, 2, 1) + BN + ReLU backward
// The pooled input gradient da of an input pixel is gathered from the (up to 4) windows whose argmax
// byte picked it (as maxpool3s2_bwd_kernel: one thread = a 2x2 input block x 8 channels) and used in
// registers: PHASE 0 reduces sum(g), sum(g (z - mean)) with g = da * relu_mask(z * sc + sh) into
// per-block slabs; PHASE 1 writes dz = A g + B z + Cc.  da is never stored.
template <int PHASE>
__global__ void __launch_bounds__(kThreads) stem_pool_bn_bwd_kernel(
    const bf16_t* __restrict__ dp, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ z,
    const float* __restrict__ ss, const float* __restrict__ mean, const float* __restrict__ coef, int N, int H, int W,
    int C, int P, int Q, float* __restrict__ slab, bf16_t* __restrict__ dz) {
  const int cv = C >> 3;
  const int Hb = (H + 1) >> 1, Wb = (W + 1) >> 1;
  const int total = N * Hb * Wb * cv;
  const int stride = gridDim.x * blockDim.x;  // a multiple of cv (host-checked): c8 is fixed per thread
  const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = t0 % cv;
  float sc[8], sh[8], mu[8], cA[8], cB[8], cC[8], sa[8], sb[8];
  load8(ss + c8 * 8, sc);
  load8(ss + C + c8 * 8, sh);
  if (PHASE == 0) {
    load8(mean + c8 * 8, mu);
  } else {
    load8(coef + c8 * 8, cA);
    load8(coef + C + c8 * 8, cB);
    load8(coef + 2 * C + c8 * 8, cC);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.f;
  for (int t = t0; t < total; t += stride) {
    int pix = t / cv;
    const int q = pix % Wb;
    pix /= Wb;
    const int p = pix % Hb;
    const int n = pix / Hb;
    const int h = 2 * p, w = 2 * q;
    // the block's 4 z vectors are loaded up front, beside the pooled gradients: their addresses do not
    // depend on the argmax bytes, and in phase 1 a z load issued after the previous pixel's dz store
    // cannot be hoisted above it (the compiler cannot rule out aliasing), which serialised 4 memory
    // latencies per block
    u16x8 zr[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int hh = h + (e >> 1), ww = w + (e & 1);
      const bool ok = hh < H && ww < W;
      const int64_t off = ok ? (((int64_t)n * H + hh) * W + ww) * C + c8 * 8 : (int64_t)c8 * 8;
      zr[e] = *reinterpret_cast<const u16x8*>(z + off);
    }
    float g[4][8];
    uint64_t id[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int pp = p + (o >> 1), qq = q + (o & 1);
      if (pp < P && qq < Q) {
        const int64_t off = (((int64_t)n * P + pp) * Q + qq) * C + c8 * 8;
        id[o] = *reinterpret_cast<const uint64_t*>(idx + off);
        load8(dp + off, g[o]);
      } else {
        id[o] = ~0ull;
#pragma unroll
        for (int j = 0; j < 8; ++j) g[o][j] = 0.f;
      }
    }
    float d[4][8];  // 2x2 block: (0,0) (0,1) (1,0) (1,1)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i0 = (uint32_t)(id[0] >> (8 * j)) & 0xFF, i1 = (uint32_t)(id[1] >> (8 * j)) & 0xFF;
      const uint32_t i2 = (uint32_t)(id[2] >> (8 * j)) & 0xFF, i3 = (uint32_t)(id[3] >> (8 * j)) & 0xFF;
      d[0][j] = i0 == 4 ? g[0][j] : 0.f;
      d[1][j] = (i0 == 5 ? g[0][j] : 0.f) + (i1 == 3 ? g[1][j] : 0.f);
      d[2][j] = (i0 == 7 ? g[0][j] : 0.f) + (i2 == 1 ? g[2][j] : 0.f);
      d[3][j] = ((i0 == 8 ? g[0][j] : 0.f) + (i1 == 6 ? g[1][j] : 0.f)) + ((i2 == 2 ? g[2][j] : 0.f) + (i3 == 0 ? g[3][j] : 0.f));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int hh = h + (e >> 1), ww = w + (e & 1);
      if (hh >= H || ww >= W) continue;
      const int64_t off = (((int64_t)n * H + hh) * W + ww) * C + c8 * 8;
      float zv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) zv[j] = bf2f(zr[e][j]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gm = fmaf(zv[j], sc[j], sh[j]) > 0.f ? d[e][j] : 0.f;
        if (PHASE == 0) {
          sa[j] += gm;
          sb[j] += gm * (zv[j] - mu[j]);
        } else {
          zv[j] = fmaf(cA[j], gm, fmaf(cB[j], zv[j], cC[j]));
        }
      }
      if (PHASE == 1) store8(dz + off, zv);
    }
  }
  if (PHASE == 0) {
    __shared__ float s_a[kThreads * 8];
    __shared__ float s_b[kThreads * 8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s_a[threadIdx.x * 8 + j] = sa[j];
      s_b[threadIdx.x * 8 + j] = sb[j];
    }
    __syncthreads();
    if ((int)threadIdx.x < cv) {  // thread c sums the threads c, c + cv, ... (same channel group)
      for (int k = threadIdx.x + cv; k < kThreads; k += cv) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sa[j] += s_a[k * 8 + j];
          sb[j] += s_b[k * 8 + j];
        }
      }
      store8(slab + (int64_t)blockIdx.x * C + c8 * 8, sa);
      store8(slab + (int64_t)gridDim.x * C + (int64_t)blockIdx.x * C + c8 * 8, sb);
    }
  }
}

}  // namespace

// rows of the fused-finalize table for C channels: enough rows that the ~1024 reduce blocks' atomic
// adds do not pile onto a few hundred bytes (8 K floats per slab), few enough that the last block's
// exchange sweep stays short
int bn_bwd_table_rows(int64_t C) {
  int r = (int)(8192 / (C > 0 ? C : 1));
  return r < 8 ? 8 : (r > 128 ? 128 : r);
}

// workspace: 2 partial slabs [nrb][C] + 3 per-channel tables [C]
int64_t bn_workspace_floats(int64_t M, int64_t C) {
  BnGeom g = bn_geom(M, C);
  return 2 * (int64_t)g.nrb * C + 3 * C;
}

hipError_t bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                        const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, float* running_mean,
                        float* running_var, float momentum, float eps, bool relu, float* save_mean,
                        float* save_invstd, float* save_ss, float* ws, uint8_t* relu_bits, int64_t* num_batches,
                        hipStream_t st) {
  if (C > kMaxC || C % 8) return hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C);
  float* scale = save_ss ? save_ss : ws + 2 * (int64_t)g.nrb * C;
  float* shift = scale + C;
  bn_stats_kernel<<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(x, M, (int)C, g.cols, g.rpi, g.rpb, ws);
  PDA_CHECK_HIP(hipGetLastError());
  bn_finalize_kernel<true><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
      x, nullptr, ws, g.nrb, M, (int)C, gamma_f, gamma_b, beta_f, beta_b, running_mean, running_var, momentum, eps, save_mean,
      save_invstd, scale, shift, num_batches);
  PDA_CHECK_HIP(hipGetLastError());
  return launch_apply(x, res, y, M, (int)C, scale, shift, relu, relu_bits, st);
}

hipError_t bn_fwd_train_sums(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, float* table,
                             int table_rows, const float* shift, const float* gamma_f, const bf16_t* gamma_b,
                             const float* beta_f, const bf16_t* beta_b, float* running_mean, float* running_var,
                             float momentum, float eps, bool relu, float* save_mean, float* save_invstd,
                             float* save_ss, uint8_t* relu_bits, int64_t* num_batches, hipStream_t st) {
  if (C > kMaxC || C % 8 || table_rows < 1) return hipErrorInvalidValue;
  float* scale = save_ss;
  float* shift_out = save_ss + C;
  bn_finalize_kernel<true, true><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
      x, shift, table, table_rows, M, (int)C, gamma_f, gamma_b, beta_f, beta_b, running_mean, running_var, momentum,
      eps, save_mean, save_invstd, scale, shift_out, num_batches);
  PDA_CHECK_HIP(hipGetLastError());
  return launch_apply(x, res, y, M, (int)C, scale, shift_out, relu, relu_bits, st);
}

// Bottleneck output with a downsample shortcut: y = relu(bn(x) + bn2(x2)), both BNs finalized from
// their conv-epilogue statistics tables; one pass reads x and x2 and writes y + the 1-bit ReLU mask
// (the shortcut's normalised tensor is never stored, nor its gradient in the backward: both BN
// backwards read dy and the mask).  C must take the register-table path (bn_dual_ok).
hipError_t bn_finalize_sums(const bf16_t* x, int64_t M, int64_t C, const BnSumsArgs& p, float momentum, float eps,
                            hipStream_t st) {
  if (C > kMaxC || C % 8 || p.table_rows < 1) return hipErrorInvalidValue;
  bn_finalize_kernel<true, true><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
      x, p.shift, p.table, p.table_rows, M, (int)C, p.gamma_f, p.gamma_b, p.beta_f, p.beta_b, p.running_mean,
      p.running_var, momentum, eps, p.save_mean, p.save_invstd, p.save_ss, p.save_ss + C, p.num_batches);
  return hipGetLastError();
}

bool bn_dual_ok(int64_t C) {
  if (C % 8 || C > kMaxC || lds_tables_forced()) return false;
  const int ns = wave_sets((int)(C / 8));  // register tables with 1, 2 or 4 sets per lane (not 3: C = 1536)
  return ns == 1 || ns == 2 || ns == 4;
}

hipError_t bn_fwd_train_sums_dual(const bf16_t* x, const bf16_t* x2, bf16_t* y, int64_t M, int64_t C,
                                  const BnSumsArgs& a, const BnSumsArgs& b, float momentum, float eps,
                                  uint8_t* relu_bits, hipStream_t st) {
  if (!bn_dual_ok(C) || a.table_rows < 1 || b.table_rows < 1) return hipErrorInvalidValue;
  const BnSumsArgs* ab[2] = {&a, &b};
  const bf16_t* xs[2] = {x, x2};
  for (int i = 0; i < 2; ++i) {
    const BnSumsArgs& p = *ab[i];
    bn_finalize_kernel<true, true><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
        xs[i], p.shift, p.table, p.table_rows, M, (int)C, p.gamma_f, p.gamma_b, p.beta_f, p.beta_b, p.running_mean,
        p.running_var, momentum, eps, p.save_mean, p.save_invstd, p.save_ss, p.save_ss + C, p.num_batches);
    PDA_CHECK_HIP(hipGetLastError());
  }
  const int ns = wave_sets((int)(C / 8));
  if (ns == 1) launch_apply_dual_wave<1>(x, x2, y, M, (int)C, a.save_ss, b.save_ss, relu_bits, st);
  else if (ns == 2) launch_apply_dual_wave<2>(x, x2, y, M, (int)C, a.save_ss, b.save_ss, relu_bits, st);
  else launch_apply_dual_wave<4>(x, x2, y, M, (int)C, a.save_ss, b.save_ss, relu_bits, st);
  return hipGetLastError();
}

hipError_t bn_fwd_eval(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                       const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, const float* running_mean,
                       const float* running_var, float eps, bool relu, float* ws, hipStream_t st) {
  if (C > kMaxC || C % 8) return hipErrorInvalidValue;
  float* scale = ws;
  float* shift = ws + C;
  bn_finalize_kernel<false><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
      x, nullptr, nullptr, 0, M, (int)C, gamma_f, gamma_b, beta_f, beta_b, const_cast<float*>(running_mean),
      const_cast<float*>(running_var), 0.f, eps, nullptr, nullptr, scale, shift, nullptr);
  PDA_CHECK_HIP(hipGetLastError());
  return launch_apply(x, res, y, M, (int)C, scale, shift, relu, nullptr, st);
}

hipError_t bwd_apply(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* ss, int64_t M, int64_t C,
                     const float* coef, bf16_t* dx, bf16_t* dres, int mask, hipStream_t st);

hipError_t bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const uint8_t* relu_bits, const float* ss,
                  int64_t M, int64_t C,
                  const float* save_mean, const float* save_invstd, const float* gamma_f, const bf16_t* gamma_b,
                  bool relu, bf16_t* dx, bf16_t* dres, float* dgamma_f, bf16_t* dgamma_b, float* dbeta_f,
                  bf16_t* dbeta_b, float* ws, float* fin_table, unsigned* fin_ticket, int fin_rows, hipStream_t st) {
  if (C > kMaxC || C % 8) return hipErrorInvalidValue;
  if (relu && !y && !ss && !relu_bits) return hipErrorInvalidValue;
  if (fin_table && (fin_rows < 1 || !fin_ticket)) return hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C);
  // fused finalize: ws holds only the 3 coefficient tables (no slabs)
  float* coef = fin_table ? ws : ws + 2 * (int64_t)g.nrb * C;
  if (fin_table && g.gy != 1) return hipErrorInvalidValue;
  const int mask = !relu ? 0 : (relu_bits ? 3 : (y ? 1 : 2));
  if (mask == 3) y = reinterpret_cast<const bf16_t*>(relu_bits);  // the mask kernels index it as bytes
  const dim3 rg(g.nrb, g.gy);
  BwdFin fin{fin_table, fin_ticket, fin_rows, save_invstd, gamma_f, gamma_b, dgamma_f, dgamma_b, dbeta_f, dbeta_b, coef};
  const bool fused = fin_table != nullptr;
#define BWD_REDUCE(MK)                                                                                       \
  do {                                                                                                       \
    if (fused)                                                                                               \
      bn_bwd_reduce_kernel<MK, true><<<rg, kThreads, 0, st>>>(dy, x, y, ss, save_mean, M, (int)C, g.cols, g.rpi, \
                                                             g.rpb, ws, fin);                                \
    else                                                                                                     \
      bn_bwd_reduce_kernel<MK, false><<<rg, kThreads, 0, st>>>(dy, x, y, ss, save_mean, M, (int)C, g.cols,     \
                                                              g.rpi, g.rpb, ws, fin);                        \
  } while (0)
  if (mask == 0) BWD_REDUCE(0);
  else if (mask == 1) BWD_REDUCE(1);
  else if (mask == 2) BWD_REDUCE(2);
  else BWD_REDUCE(3);
#undef BWD_REDUCE
  PDA_CHECK_HIP(hipGetLastError());
  if (!fused) {
    bn_bwd_finalize_kernel<false><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(ws, g.nrb, M, (int)C, save_mean,
                                                                           save_invstd, gamma_f, gamma_b, dgamma_f,
                                                                           dgamma_b, dbeta_f, dbeta_b, coef);
    PDA_CHECK_HIP(hipGetLastError());
  }
  return bwd_apply(dy, x, y, ss, M, C, coef, dx, dres, mask, st);
}

// the BN backward apply pass: dx = A dz + B x + Cc (dz = dy * ReLU mask), optionally dres = dz
hipError_t bwd_apply(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* ss, int64_t M, int64_t C,
                     const float* coef, bf16_t* dx, bf16_t* dres, int mask, hipStream_t st) {
  int ns = lds_tables_forced() ? 0 : wave_sets((int)(C / 8));
  if (ns == 3 || ns > 4) ns = 0;
  const int grid = ns ? wave_grid(M * C / 8) : ew_grid(M * C / 8);
  const size_t lds = 5 * (size_t)C * sizeof(float);
#define BWD_APPLY(MK, DR)                                                                                        \
  do {                                                                                                           \
    if (ns == 1) bn_bwd_apply_wave_kernel<MK, DR, 1><<<grid, kThreads, 0, st>>>(dy, x, y, ss, M, (int)C, coef, dx, dres); \
    else if (ns == 2) bn_bwd_apply_wave_kernel<MK, DR, 2><<<grid, kThreads, 0, st>>>(dy, x, y, ss, M, (int)C, coef, dx, dres); \
    else if (ns == 4) bn_bwd_apply_wave_kernel<MK, DR, 4><<<grid, kThreads, 0, st>>>(dy, x, y, ss, M, (int)C, coef, dx, dres); \
    else bn_bwd_apply_kernel<MK, DR><<<grid, kThreads, lds, st>>>(dy, x, y, ss, M, (int)C, coef, dx, dres);     \
  } while (0)
  if (mask == 0) { if (dres) BWD_APPLY(0, true); else BWD_APPLY(0, false); }
  else if (mask == 1) { if (dres) BWD_APPLY(1, true); else BWD_APPLY(1, false); }
  else if (mask == 2) { if (dres) BWD_APPLY(2, true); else BWD_APPLY(2, false); }
  else { if (dres) BWD_APPLY(3, true); else BWD_APPLY(3, false); }
#undef BWD_APPLY
  return hipGetLastError();
}

hipError_t bn_bwd_table(const bf16_t* dy, const bf16_t* x, const uint8_t* relu_bits, const float* ss, int64_t M,
                        int64_t C, const float* save_mean, const float* save_invstd, const float* gamma_f,
                        const bf16_t* gamma_b, bool relu, bf16_t* dx, bf16_t* dres, float* dgamma_f, bf16_t* dgamma_b,
                        float* dbeta_f, bf16_t* dbeta_b, float* table, int rows, float* coef, hipStream_t st) {
  if (C > kMaxC || C % 8 || rows < 1 || !table) return hipErrorInvalidValue;
  if (relu && !ss && !relu_bits) return hipErrorInvalidValue;
  bn_bwd_finalize_kernel<true><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
      table, rows, M, (int)C, save_mean, save_invstd, gamma_f, gamma_b, dgamma_f, dgamma_b, dbeta_f, dbeta_b, coef);
  PDA_CHECK_HIP(hipGetLastError());
  const int mask = !relu ? 0 : (relu_bits ? 3 : 2);
  const bf16_t* y = mask == 3 ? reinterpret_cast<const bf16_t*>(relu_bits) : nullptr;
  return bwd_apply(dy, x, y, ss, M, C, coef, dx, dres, mask, st);
}

bool bn_bwd_dual_ok(int64_t C) {
  if (C % 8 || C > kMaxC || lds_tables_forced()) return false;
  const int ns = wave_sets((int)(C / 8));
  return ns == 1 || ns == 2;
}

hipError_t bn_bwd_dual(const bf16_t* dy, const uint8_t* relu_bits, int64_t M, int64_t C, const BnBwdSide& a,
                       const BnBwdSide& b, hipStream_t st) {
  if (!bn_bwd_dual_ok(C) || !relu_bits) return hipErrorInvalidValue;
  BnGeom g = bn_geom(M, C);
  float* coef = a.ws + 2 * (int64_t)g.nrb * C;
  float* coef2 = b.ws + 2 * (int64_t)g.nrb * C;
  // both sums from a dgrad epilogue (BnBwdStats z / z2): no reduce pass, finalize from the tables
  const bool tables = a.table && b.table;
  if ((a.table != nullptr) != (b.table != nullptr) || (tables && (a.rows < 1 || b.rows < 1))) return hipErrorInvalidValue;
  if (!tables) {
    bn_bwd_reduce_dual_kernel<<<dim3(g.nrb, g.gy), kThreads, 0, st>>>(dy, a.x, b.x, relu_bits, a.mean, b.mean, M,
                                                                     (int)C, g.cols, g.rpi, g.rpb, a.ws, b.ws);
    PDA_CHECK_HIP(hipGetLastError());
  }
  const BnBwdSide* sides[2] = {&a, &b};
  float* coefs[2] = {coef, coef2};
  for (int i = 0; i < 2; ++i) {
    const BnBwdSide& p = *sides[i];
    if (tables)
      bn_bwd_finalize_kernel<true><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
          p.table, p.rows, M, (int)C, p.mean, p.invstd, p.gamma_f, p.gamma_b, p.dgamma_f, p.dgamma_b, p.dbeta_f,
          p.dbeta_b, coefs[i]);
    else
      bn_bwd_finalize_kernel<false><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(
          p.ws, g.nrb, M, (int)C, p.mean, p.invstd, p.gamma_f, p.gamma_b, p.dgamma_f, p.dgamma_b, p.dbeta_f,
          p.dbeta_b, coefs[i]);
    PDA_CHECK_HIP(hipGetLastError());
  }
  const int grid = wave_grid(M * C / 8);
  if (wave_sets((int)(C / 8)) == 1)
    bn_bwd_apply_dual_wave_kernel<1><<<grid, kThreads, 0, st>>>(dy, a.x, b.x, relu_bits, M, (int)C, coef, coef2, a.dx,
                                                                 b.dx);
  else
    bn_bwd_apply_dual_wave_kernel<2><<<grid, kThreads, 0, st>>>(dy, a.x, b.x, relu_bits, M, (int)C, coef, coef2, a.dx,
                                                                 b.dx);
  return hipGetLastError();
}

bool stem_pool_bn_bwd_ok(int H, int W, int C, int P, int Q, int k, int s, int pad) {
  return k == 3 && s == 2 && pad == 1 && P == (H - 1) / 2 + 1 && Q == (W - 1) / 2 + 1 && C % 8 == 0 && C <= kMaxC &&
         kThreads % (C / 8) == 0;
}

int64_t stem_pool_bn_bwd_ws_floats(int64_t C) { return 2 * (int64_t)kStemBlocks * C + 3 * C; }

hipError_t stem_pool_bn_bwd(const bf16_t* dp, const uint8_t* idx, const bf16_t* z, const float* ss,
                            const float* mean, const float* invstd, const float* gamma_f, const bf16_t* gamma_b,
                            int N, int H, int W, int C, int P, int Q, bf16_t* dz, float* dgamma_f, bf16_t* dgamma_b,
                            float* dbeta_f, bf16_t* dbeta_b, float* ws, hipStream_t st) {
  if (!stem_pool_bn_bwd_ok(H, W, C, P, Q, 3, 2, 1)) return hipErrorInvalidValue;
  float* coef = ws + 2 * (int64_t)kStemBlocks * C;
  const int64_t M = (int64_t)N * H * W;
  stem_pool_bn_bwd_kernel<0><<<kStemBlocks, kThreads, 0, st>>>(dp, idx, z, ss, mean, nullptr, N, H, W, C, P, Q, ws,
                                                              nullptr);
  PDA_CHECK_HIP(hipGetLastError());
  bn_bwd_finalize_kernel<false><<<(unsigned)((C + 63) / 64), kFinThreads, 0, st>>>(ws, kStemBlocks, M, C, mean, invstd,
                                                                           gamma_f, gamma_b, dgamma_f, dgamma_b,
                                                                           dbeta_f, dbeta_b, coef);
  PDA_CHECK_HIP(hipGetLastError());
  stem_pool_bn_bwd_kernel<1><<<kStemBlocks, kThreads, 0, st>>>(dp, idx, z, ss, mean, coef, N, H, W, C, P, Q, nullptr,
                                                              dz);
  return hipGetLastError();
}

}  // namespace pda
