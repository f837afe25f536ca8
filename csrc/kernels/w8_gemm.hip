// Weight-only int8 GEMM for serving decode steps: y[M, N] = x[M, K] · (Wq[N, K] · s[N])^T, M <= 64
// (tokens of one decode step), bf16 activations, int8 weights with one fp32 scale per output row.
// SURVEY §2.5 K17 / §2.3 N15 (the reference loads its Llama with bitsandbytes LLM.int8,
// `03 模型并行/03_model_parallel.ipynb` raw line 86): a decode step streams every weight once, so
// halving the weight bytes is what moves tokens/s — the MI355X-native version of that idea.
//
// CDNA4 structure:
//  * v_mfma_f32_16x16x32_bf16 with the dequantised weight rows as the A operand (int8 -> bf16 is exact
//    for |q| <= 127) and the activation rows as B: a lane owns one token column (lane & 15) and four
//    consecutive output rows, so the per-row scale is applied once to the fp32 accumulator;
//  * each lane streams 16 contiguous int8 (one 16-B load) per n-block per 64-k step and uses them for
//    two MFMAs (k sub-steps 0-7 / 8-15 of its 16-element group; the activation fragment uses the same
//    permutation, so the dot products are unchanged);
//  * large N: a wave owns 64 output rows (4 n-blocks), so each activation fragment feeds 8 MFMAs
//    (activation bytes per weight byte = M/32, read from L2); small N (< 256 such tiles): 16-row tiles,
//    4x the workgroups; in both the workgroup's 4 waves split K and reduce through LDS;
//  * optional inter-workgroup split-K (S > 1): fp32 partial slabs + an atomic ticket, the last
//    workgroup of a tile sums them — one launch, graph-capturable, but measured slower than S = 1 on
//    every Llama shape (publishing a slab across XCDs costs an L2 write-back), so S = 1 by default.
//    (v1 used fp32 atomic adds into one buffer: 3-10x slower still.)
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

typedef __bf16 mbf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int kW8Threads = 256;

__device__ __forceinline__ mbf16x8 i8_to_bf16x8(uint32_t lo, uint32_t hi) {
  mbf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (__bf16)(float)(int8_t)(lo >> (8 * j));
    r[j + 4] = (__bf16)(float)(int8_t)(hi >> (8 * j));
  }
  return r;
}

// NB = n-blocks of 16 output rows per workgroup (every wave covers the same rows, the 4 waves split K)
template <int MB, int kNB>
__global__ void __launch_bounds__(kW8Threads) w8_gemm_kernel(W8GemmParams p) {
  constexpr int kW8Rows = 16 * kNB;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r16 = lane & 15, kg = lane >> 4;
  const int ntile = blockIdx.x, split = blockIdx.y;
  const int kper = p.K / (4 * p.S);
  const int64_t kbeg = (int64_t)(split * 4 + wave) * kper + kg * 16;
  const int8_t* wr = p.w + (int64_t)(ntile * kW8Rows + r16) * p.K + kbeg;
  const bf16_t* xr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = min(mb * 16 + r16, p.M - 1);  // padded token rows re-read row M-1, never stored
    xr[mb] = p.x + (int64_t)m * p.ldx + kbeg;
  }
  f32x4 acc[kNB][MB];
#pragma unroll
  for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 4
  for (int k = 0; k < kper; k += 64) {
    i32x4 q[kNB];
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb) q[nb] = *reinterpret_cast<const i32x4*>(wr + (int64_t)nb * 16 * p.K + k);
    mbf16x8 xa[MB], xb[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      xa[mb] = *reinterpret_cast<const mbf16x8*>(xr[mb] + k);
      xb[mb] = *reinterpret_cast<const mbf16x8*>(xr[mb] + k + 8);
    }
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb) {
      const mbf16x8 a = i8_to_bf16x8((uint32_t)q[nb][0], (uint32_t)q[nb][1]);
      const mbf16x8 b = i8_to_bf16x8((uint32_t)q[nb][2], (uint32_t)q[nb][3]);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xa[mb], acc[nb][mb], 0, 0, 0);
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, xb[mb], acc[nb][mb], 0, 0, 0);
      }
    }
  }
  // reduce the 4 K-slices of the workgroup into wave 0
  __shared__ f32x4 red[3][kNB][MB][64];
  if (wave > 0) {
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) red[wave - 1][nb][mb][lane] = acc[nb][mb];
  }
  __syncthreads();
  __shared__ int s_last;
  if (wave == 0) {
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        f32x4 v = acc[nb][mb];
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          const f32x4 t = red[w][nb][mb][lane];
          v[0] += t[0]; v[1] += t[1]; v[2] += t[2]; v[3] += t[3];
        }
        const int m = mb * 16 + r16;
        const int n0 = ntile * kW8Rows + nb * 16 + kg * 4;
        if (m < p.M) {
          if (p.S == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) p.y[(int64_t)m * p.ldy + n0 + i] = f2bf(v[i] * p.scale[n0 + i]);
          } else {  // this split's partial tile -> its fp32 slab (plain stores)
            *reinterpret_cast<f32x4*>(p.ws + ((int64_t)split * p.M + m) * p.N + n0) = v;
          }
        }
      }
  }
  if (p.S == 1) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(p.tickets + ntile, 1) == p.S - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  // last workgroup of the tile: sum the S slabs (L2-coherent loads) and write the bf16 result
  for (int e = threadIdx.x; e < p.M * (kW8Rows / 4); e += kW8Threads) {
    const int m = e / (kW8Rows / 4), n = ntile * kW8Rows + (e % (kW8Rows / 4)) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < p.S; ++sp) {
      const f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p.ws + ((int64_t)sp * p.M + m) * p.N + n));
      v[0] += t[0]; v[1] += t[1]; v[2] += t[2]; v[3] += t[3];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) p.y[(int64_t)m * p.ldy + n + i] = f2bf(v[i] * p.scale[n + i]);
  }
  if (threadIdx.x == 0) p.tickets[ntile] = 0;
}

}  // namespace

int w8_gemm_rows() { return 16; }

int w8_gemm_splits(int N, int K) {
  // Measured (profiles/r1_w8_gemm_splits.jsonl, M = 32): inter-workgroup split-K loses on every Llama
  // shape — the agent-scope release that publishes a slab to another XCD writes back L2 — so the
  // parallelism comes from narrower row tiles (NB = 1 -> N/16 workgroups) instead.
  (void)N;
  (void)K;
  return 1;
}

template <int NB>
static hipError_t launch_w8(const W8GemmParams& p, hipStream_t st) {
  dim3 grid((unsigned)(p.N / (16 * NB)), (unsigned)p.S);
  if (p.M <= 16) w8_gemm_kernel<1, NB><<<grid, kW8Threads, 0, st>>>(p);
  else if (p.M <= 32) w8_gemm_kernel<2, NB><<<grid, kW8Threads, 0, st>>>(p);
  else w8_gemm_kernel<4, NB><<<grid, kW8Threads, 0, st>>>(p);
  return hipGetLastError();
}

hipError_t w8_gemm(const W8GemmParams& p, hipStream_t st) {
  if (p.M < 1 || p.M > 64 || p.N % 16 || p.S < 1 || p.S > 8 || p.K % (64 * 4 * p.S)) return hipErrorInvalidValue;
  // 64-row tiles (activation fragment reused by 8 MFMAs) while they still give >= 256 workgroups;
  // 16-row tiles otherwise (4x the workgroups; activations re-read from L2 instead)
  if (p.N % 64 == 0 && (p.N / 64) * p.S >= 256) return launch_w8<4>(p, st);
  return launch_w8<1>(p, st);
}

}  // namespace pda
