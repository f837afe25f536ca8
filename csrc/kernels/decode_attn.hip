// Decode attention (serving: one new query token per sequence against a bf16 KV cache), GQA-aware,
// split over the sequence ("flash decoding"): SURVEY §2.4 W8 (the reference's Llama auto-placement
// inference, `03 模型并行/03_model_parallel.ipynb` raw lines 85-89) on the MI355X serving path.
//
// Why not MFMA: at one query row per head the op is ~G/2 FLOP per cache byte (G = query heads per KV
// head), i.e. purely HBM-bound — the job is to stream K and V exactly once at full bandwidth.
// CDNA4 layout, no LDS in the main loop:
//   * a workgroup = one (batch, KV head, sequence split), 4 waves; the G query heads that share the KV
//     head are processed together, so every K/V byte is read once for all of them;
//   * a wave reads KPI = 64 / (D/8) cache rows per instruction: lane = (row kk, 16-B chunk c), so every
//     load is a coalesced 16 B per lane (1 KB per wave); the lane keeps q[g][chunk c] (pre-scaled by
//     softmax_scale·log2 e) in registers for all G heads;
//   * QK: 8 FMAs per head per lane, then a DPP/xor butterfly across the D/8 chunk lanes of a row gives
//     every lane of the row its score; the same lanes then own that row's softmax weight, so PV needs no
//     data exchange: acc[g][8] += p[g] · v[chunk];
//   * every wave keeps its own running max / sum (online softmax over its key range); waves, then
//     splits, are merged once at the end (LDS, then a tiny combine kernel when split).
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int kDecThreads = 256;
constexpr int kDecWaves = kDecThreads / 64;
constexpr int kMaxSteps = 8;  // row-steps per wave tile (loads in flight per lane)

__device__ __forceinline__ float xor_sum(float v, int lo, int hi) {
  for (int o = lo; o < hi; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float xor_max(float v, int lo, int hi) {
  for (int o = lo; o < hi; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int D, int G>
__global__ void __launch_bounds__(kDecThreads) decode_attn_kernel(DecodeAttnParams p) {
  constexpr int DCH = D / 8;        // 16-B chunks per row
  constexpr int KPI = 64 / DCH;     // rows per wave instruction
  constexpr int kSteps = G >= 8 ? 4 : kMaxSteps;  // G = 8: fewer rows in flight keeps 1 wave/SIMD spill-free
  constexpr int TILE = KPI * kSteps;  // rows per wave tile
  const int split = blockIdx.x, hkv = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kk = lane / DCH, c = lane % DCH;
  // graph-replayable decode: the length comes from device memory (pos + 1 of this step)
  const int L = p.L_dev != nullptr ? *p.L_dev + 1 : p.L;
  const int chunk = p.L_dev != nullptr ? (L + p.splits - 1) / p.splits : p.chunk;
  const int k0 = split * chunk;
  const int k1 = min(L, k0 + chunk);

  // q (pre-scaled into the exp2 domain) for this lane's chunk, all G heads
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16_t* qp = p.q + (int64_t)b * p.q_sb + (int64_t)(hkv * G + g) * p.q_sh + c * 8;
    load8(qp, q[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) q[g][j] *= p.scale_log2;
  }
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -1e30f;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }
  const bf16_t* kb = p.k + (int64_t)b * p.k_sb + (int64_t)hkv * p.k_sh + c * 8;
  const bf16_t* vb = p.v + (int64_t)b * p.v_sb + (int64_t)hkv * p.v_sh + c * 8;

  for (int t0 = k0 + wave * TILE; t0 < k1; t0 += kDecWaves * TILE) {
    u16x8 kr[kSteps];
    int rows[kSteps];
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      const int r = t0 + s * KPI + kk;
      rows[s] = r;
      const int rc = r < k1 ? r : k1 - 1;  // clamp: masked rows read a valid (written) row
      kr[s] = *reinterpret_cast<const u16x8*>(kb + (int64_t)rc * p.k_st);
    }
    float sc[kSteps][G];
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      float kf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[j] = bf2f(kr[s][j]);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d = fmaf(q[g][j], kf[j], d);
        sc[s][g] = xor_sum(d, 1, DCH);
      }
    }
    // issue the V loads before the softmax math so they overlap it
    u16x8 vr[kSteps];
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      const int rc = rows[s] < k1 ? rows[s] : k1 - 1;
      vr[s] = *reinterpret_cast<const u16x8*>(vb + (int64_t)rc * p.v_st);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float tmax = -INFINITY;
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        if (rows[s] >= k1) sc[s][g] = -INFINITY;
        tmax = fmaxf(tmax, sc[s][g]);
      }
      tmax = xor_max(tmax, DCH, 64);
      const float mn = fmaxf(m[g], tmax);
      const float alpha = __builtin_amdgcn_exp2f(m[g] - mn);
      m[g] = mn;
      float ps = 0.f;
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        sc[s][g] = __builtin_amdgcn_exp2f(sc[s][g] - mn);
        ps += sc[s][g];
      }
      l[g] = l[g] * alpha + xor_sum(ps, DCH, 64);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] *= alpha;
    }
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      float vf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) vf[j] = bf2f(vr[s][j]);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] = fmaf(sc[s][g], vf[j], acc[g][j]);
    }
  }
  // rows of a wave -> one partial per wave (same running max across its lanes)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = xor_sum(acc[g][j], DCH, 64);

  __shared__ float s_ml[kDecWaves][G][2];
  __shared__ float s_acc[kDecWaves][G][D];
  if (lane < DCH) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_acc[wave][g][c * 8 + j] = acc[g][j];
      if (c == 0) {
        s_ml[wave][g][0] = m[g];
        s_ml[wave][g][1] = l[g];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += kDecThreads) {
    const int g = i / D, d = i % D;
    float mx = -1e30f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) mx = fmaxf(mx, s_ml[w][g][0]);
    float ls = 0.f, o = 0.f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) {
      const float f = __builtin_amdgcn_exp2f(s_ml[w][g][0] - mx);
      ls += s_ml[w][g][1] * f;
      o += s_acc[w][g][d] * f;
    }
    const int hq = hkv * G + g;
    if (p.splits == 1) {
      p.o[((int64_t)b * p.Hq + hq) * D + d] = f2bf(ls > 0.f ? o / ls : 0.f);
    } else {
      const int64_t row = ((int64_t)b * p.Hq + hq) * p.splits + split;
      p.ws_acc[row * D + d] = o;
      if (d == 0) {
        p.ws_ml[row * 2] = mx;
        p.ws_ml[row * 2 + 1] = ls;
      }
    }
  }
}

// one workgroup per (batch, query head): merge the split partials
template <int D>
__global__ void __launch_bounds__(D) decode_combine_kernel(DecodeAttnParams p) {
  const int64_t bh = blockIdx.x;
  const int d = threadIdx.x;
  const float* ml = p.ws_ml + bh * p.splits * 2;
  float mx = -1e30f;
  for (int s = 0; s < p.splits; ++s) mx = fmaxf(mx, ml[2 * s]);
  float ls = 0.f, o = 0.f;
  for (int s = 0; s < p.splits; ++s) {
    const float f = __builtin_amdgcn_exp2f(ml[2 * s] - mx);
    ls += ml[2 * s + 1] * f;
    o += p.ws_acc[(bh * p.splits + s) * D + d] * f;
  }
  p.o[bh * D + d] = f2bf(ls > 0.f ? o / ls : 0.f);
}

// New token of a decode step, graph-replayable (position read from device memory): q rotated into
// q_out, k rotated into k_cache[:, pos], v copied into v_cache[:, pos].  One wave per (batch, head),
// lane i owns the rotate-half pairs (i, i + D/2) (D = 128: one pair, D = 64: lanes 0..31).
__global__ void __launch_bounds__(64) kv_append_rope_kernel(KvAppendParams p) {
  const int b = blockIdx.y, h = blockIdx.x, i = threadIdx.x;
  const int half = p.D / 2;
  if (i >= half) return;
  const int pos = *p.pos;
  const bf16_t* x = p.qkv + (int64_t)b * p.x_sb + (int64_t)h * p.x_sh;
  const float x1 = bf2f(x[i]), x2 = bf2f(x[i + half]);
  if (h >= p.Hq + p.Hkv) {  // V: plain copy
    bf16_t* dst = p.v_cache + (int64_t)b * p.v_sb + (int64_t)pos * p.v_st + (int64_t)(h - p.Hq - p.Hkv) * p.v_sh;
    dst[i] = x[i];
    dst[i + half] = x[i + half];
    return;
  }
  float y1 = x1, y2 = x2;
  if (p.cos != nullptr) {
    const float cs = p.cos[(int64_t)pos * half + i], sn = p.sin[(int64_t)pos * half + i];
    y1 = x1 * cs - x2 * sn;
    y2 = x2 * cs + x1 * sn;
  }
  bf16_t* dst = h < p.Hq ? p.q_out + ((int64_t)b * p.Hq + h) * p.D
                         : p.k_cache + (int64_t)b * p.k_sb + (int64_t)pos * p.k_st + (int64_t)(h - p.Hq) * p.k_sh;
  dst[i] = f2bf(y1);
  dst[i + half] = f2bf(y2);
}

template <int D, int G>
hipError_t launch_decode(const DecodeAttnParams& p, hipStream_t st) {
  dim3 grid((unsigned)p.splits, (unsigned)p.Hkv, (unsigned)p.B);
  decode_attn_kernel<D, G><<<grid, kDecThreads, 0, st>>>(p);
  PDA_CHECK_HIP(hipGetLastError());
  if (p.splits > 1) decode_combine_kernel<D><<<(unsigned)(p.B * p.Hq), D, 0, st>>>(p);
  return hipGetLastError();
}

template <int D>
hipError_t dispatch_g(const DecodeAttnParams& p, hipStream_t st) {
  switch (p.Hq / p.Hkv) {
    case 1: return launch_decode<D, 1>(p, st);
    case 2: return launch_decode<D, 2>(p, st);
    case 4: return launch_decode<D, 4>(p, st);
    case 8: return launch_decode<D, 8>(p, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int decode_attn_splits(int B, int Hkv, int L, int D) {
  // enough workgroups to cover the 256 CUs twice, but every split keeps >= one full pass of its 4 waves
  const int rows_per_pass = kDecWaves * (64 / (D / 8)) * kMaxSteps;
  const int max_splits = (L + rows_per_pass - 1) / rows_per_pass;
  int s = (512 + B * Hkv - 1) / (B * Hkv);
  if (s > max_splits) s = max_splits;
  if (s > 64) s = 64;
  return s < 1 ? 1 : s;
}

hipError_t kv_append_rope(const KvAppendParams& p, hipStream_t st) {
  if (p.D % 2 || p.D / 2 > 64) return hipErrorInvalidValue;
  dim3 grid((unsigned)(p.Hq + 2 * p.Hkv), (unsigned)p.B);
  kv_append_rope_kernel<<<grid, 64, 0, st>>>(p);
  return hipGetLastError();
}

hipError_t decode_attention(DecodeAttnParams p, hipStream_t st) {
  if ((p.L_dev == nullptr && p.L < 1) || p.Hkv < 1 || p.Hq % p.Hkv || p.splits < 1) return hipErrorInvalidValue;
  p.chunk = p.L_dev != nullptr ? 0 : (p.L + p.splits - 1) / p.splits;
  if (p.D == 64) return dispatch_g<64>(p, st);
  if (p.D == 128) return dispatch_g<128>(p, st);
  return hipErrorInvalidValue;
}

}  // namespace pda
