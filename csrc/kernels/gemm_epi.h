// Shared GEMM epilogue of the 256 x 256 tiles (gemm_conv.hip wide kernel, gemm_pp.hip pipelined
// kernel): the Epi descriptor (bias / ReLU / addend / GELU / BN statistics / fp32 and split-K slab
// outputs / dgrad row remap) and the tile epilogue for the 8-wave (2 x 4) accumulator layout
//   acc[i][j][r] = C[m0 + wr*128 + 16 i + (lane & 15)][n0 + wc*64 + 16 j + 4 (lane >> 4) + r].
#pragma once
#ifndef PDA_BSTG
#define PDA_BSTG 8
#endif
#include "pda_common.h"

namespace pda {

struct Epi {
  void* C;           // output base
  int64_t ldc;
  int c_f32;         // 1: fp32 output, 0: bf16 output
  const void* bias;  // per-column bias or null
  int bias_f32;
  int relu;
  float* slab;       // split-K fp32 partial slabs [splits][M][N] (overrides C when non-null)
  // row remap (dgrad phase launches): row m = (n, hh, ww) of a [N, Hh, Wh] phase grid is written to
  // C row (n*H + hh*st + ph)*W + ww*st + pw
  int rm_on, rm_Hh, rm_Wh, rm_st, rm_ph, rm_pw, rm_H, rm_W;
  // optional bf16 addend with C's layout (gradient accumulation fused into the store: conv1's dgrad
  // adds the residual-branch gradient of a bottleneck instead of a separate add kernel)
  const bf16_t* addend;
  // optional ReLU bit mask of the addend (bit j of byte v masks element 8v + j of C's layout): the
  // addend is then dz * mask, i.e. a bottleneck's residual gradient read straight from the block's
  // output gradient and the BN's forward bit mask, never materialised by the BN backward
  const uint8_t* addend_bits;
  // optional BatchNorm statistics of the (bf16-rounded) output: per-tile column sums of (y - K) and
  // (y - K)^2 (K = stats_shift, e.g. the running mean) are atomically added to row (tile_m % stats_rows)
  // of a zero-initialised stats[stats_rows][2][N] table, which the BN finalize reads and re-zeroes.
  float* stats;
  const float* stats_shift;
  int stats_rows;
  // optional fused activation of a bf16 output (staged epilogues; no split-K): 1 = GELU-tanh forward,
  // the pre-activation written to act_aux (C's layout) for the backward; 2 = GELU-tanh backward,
  // C = (A B) * gelu'(act_aux) with act_aux the forward's pre-activation (the MLP's fc2 dgrad fused
  // with the activation backward: no separate elementwise pass over two [tokens, 4d] tensors)
  int act;
  bf16_t* act_aux;
  // optional row sums of operand A over this launch's K range (only the pipelined kernel, gemm_pp.hip,
  // computes them): a Linear weight gradient dW = dY^T X has A = dY^T, so its row sums are the bias
  // gradient (db folded into the dW GEMM).  mode 1: fp32 store, 2: bf16 store, 3: fp32
  // atomic add (split-K launches; the caller zeroes the buffer)
  void* rowsum;
  int rowsum_mode;  // 1 fp32 store, 2 bf16 store, 3 fp32 atomic add, 4 fp32 store at [split][M]
  // mode 4 + rowsum_out: the split-K reduce launch also sums the [split][M] row sums into rowsum_out (its
  // last ceil(M / 256) workgroups; bf16 when rowsum_out_bf16) — no separate cast launch
  void* rowsum_out;
  int rowsum_out_bf16;
  int nt_store;     // bf16 C rows written with nontemporal stores (streamed past the caches)
  // optional BatchNorm-BACKWARD statistics of the produced gradient (the data gradient of the
  // conv that consumed relu(bn(z)) IS that BN's dy).  With bst_z set, the stats path above accumulates
  // instead g = C masked by the BN's ReLU — recomputed from z and the BN's per-channel scale / shift
  // bst_ss [2][N], or read from the forward's 1-bit mask bst_bits — as sum(g) and sum(g (z - K)), K =
  // stats_shift = the saved batch mean: exactly the sums of the separate backward reduce pass, which
  // would re-read dy and z from HBM right after this epilogue had dy in registers.
  const bf16_t* bst_z;
  const float* bst_ss;
  const uint8_t* bst_bits;
  // second BN fed by the same masked gradient (a downsample bottleneck's relu(bn(z) + bn2(z2))): its sums
  // sum(g) and sum(g (z2 - mean2)) go to bst_table2 (same row layout)
  const bf16_t* bst_z2;
  const float* bst_mean2;
  float* bst_table2;
  // in-kernel split-K fix-up (pipelined tile, splitk_fixup below): one zeroed arrival counter per tile of
  // the launch (indexed by blockIdx.x); the last split of a tile sums the slabs and runs the epilogue, so no
  // separate reduce launch follows.  Null: the caller reduces the slabs (splitk_reduce_kernel).
  int* tickets;
};

// The pipelined 256 x 256 GEMM (gemm_pp.hip); gemm_conv.hip routes plain GEMMs to it.
hipError_t gemm_pp(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                   int64_t M, int64_t N, int64_t K, const Epi& epi, int splits, int variant, hipStream_t st,
                   int* used_splits);
int pp_default_variant();
// Streaming short-K (64 / 128) 1x1 stride-1 dgrad with the BN-backward sums (dgrad_stream.hip)
bool dgrad_stream_ok(int64_t M, int64_t N, int64_t K, const Epi& epi);
hipError_t dgrad_stream(const bf16_t* dy, const bf16_t* w, int64_t M, int64_t N, int64_t K, const Epi& epi,
                        hipStream_t st);
// Streaming short-K (64 / 128 / 256) 1x1 stride-1 forward with the forward BN statistics (fwd_stream.hip)
bool fwd_stream_ok(int64_t M, int64_t N, int64_t K, const Epi& epi);
hipError_t fwd_stream(const bf16_t* x, const bf16_t* w, int64_t M, int64_t N, int64_t K, const Epi& epi,
                      hipStream_t st);
hipError_t gemm_pp_wgrad(const bf16_t* dy, const bf16_t* x, int Nimg, int H, int W, int C, int Cout, int R, int S,
                         int P, int Q, int stride, int pad, int dil, const Epi& epi, int splits, hipStream_t stream,
                         int* used_splits);
hipError_t gemm_pp_gather(const bf16_t* src, int Nimg, int H, int W, int C, int P, int Q, int S, int K, int st,
                          int o_r, int o_c, int tr, int ts, const bf16_t* w, int Cout, const Epi& epi, hipStream_t stream);

namespace {


__device__ __forceinline__ void epi_act8(const Epi& e, int64_t crow, int64_t n, u16x8& v) {
  if (e.act == 1) {
    *reinterpret_cast<u16x8*>(e.act_aux + crow * e.ldc + n) = v;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = f2bf(gelu_tanh(bf2f(v[q])));
  } else if (e.act == 2) {
    const u16x8 h = *reinterpret_cast<const u16x8*>(e.act_aux + crow * e.ldc + n);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = f2bf(bf2f(v[q]) * gelu_tanh_grad(bf2f(h[q])));
  }
}

// One workgroup's column partials (8 consecutive columns per thread, `cpr` column chunks per row,
// `nt` threads): fold the lanes of a wave that share a chunk, then the waves through `red` (nt/64 x
// 8*cpr x 2 floats of LDS that nothing else uses), then one atomic add per column and statistic.
// The only barrier is LDS-only (lgkmcnt + s_barrier): a __syncthreads() here would also wait for the
// tile's global stores to be acknowledged (vmcnt(0)) — measured at ~16 us per wide-tile conv, since a
// 1-workgroup-per-CU kernel exposes every epilogue cycle.
__device__ __forceinline__ void epi_stats_flush(const Epi& epi, float (&st1)[8], float (&st2)[8], float* red, int cpr,
                                                int nt, int tm, int64_t n0, int64_t N, float* table = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, ncol = cpr * 8;
  for (int off = cpr; off < 64; off <<= 1)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      st1[q] += __shfl_xor(st1[q], off, 64);
      st2[q] += __shfl_xor(st2[q], off, 64);
    }
  if (lane < cpr) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[(wid * ncol + lane * 8 + q) * 2] = st1[q];
      red[(wid * ncol + lane * 8 + q) * 2 + 1] = st2[q];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (tid < ncol && n0 + tid < N) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < nt / 64; ++w) {
      a += red[(w * ncol + tid) * 2];
      b += red[(w * ncol + tid) * 2 + 1];
    }
    float* row = (table ? table : epi.stats) + (int64_t)(tm % epi.stats_rows) * 2 * N;
    unsafeAtomicAdd(row + n0 + tid, a);
    unsafeAtomicAdd(row + N + n0 + tid, b);
  }
}

// Per-thread constants of the statistics path for the column chunk n .. n + 7 (fixed per thread in every
// staged epilogue): the shift K, and for the backward sums with a recomputed ReLU mask the BN's scale /
// shift.
struct EpiStatCols {
  float k[8];
};
__device__ __forceinline__ void epi_stat_cols(const Epi& e, bool want, int64_t n, int64_t N, EpiStatCols& c) {
#pragma unroll
  for (int q = 0; q < 8; ++q) c.k[q] = (want && n + q < N) ? e.stats_shift[n + q] : 0.f;
}

// accumulate the forward statistics of the 8 stored (bf16-rounded) values v at (crow, n): sums of (v - K)
// and (v - K)^2 (the BN-backward sums take epi_bst_chunks)
__device__ __forceinline__ void epi_stats8(const Epi& e, const EpiStatCols& c, int64_t crow, int64_t n, const u16x8& v,
                                           float (&st1)[8], float (&st2)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float d = bf2f(v[q]) - c.k[q];
    st1[q] += d;
    st2[q] = fmaf(d, d, st2[q]);
  }
}

__device__ __forceinline__ int64_t epi_row(const Epi& e, int64_t m) {
  if (!e.rm_on) return m;
  // 32-bit divisions (a phase GEMM's rows and the phase grid fit easily; the int64 divide is a ~100-instruction
  // software sequence, paid per 16-B chunk of every strided-dgrad epilogue)
  const uint32_t mm = (uint32_t)m, wh = (uint32_t)e.rm_Wh, hh_ = (uint32_t)e.rm_Hh;
  const uint32_t t = mm / wh;
  const int ww = (int)(mm - t * wh);
  const uint32_t n = t / hh_;
  const int hh = (int)(t - n * hh_);
  return ((int64_t)n * e.rm_H + (int64_t)hh * e.rm_st + e.rm_ph) * e.rm_W + (int64_t)ww * e.rm_st + e.rm_pw;
}

// The staged-chunk loop of a bf16 epilogue WITH BN-backward statistics (bst_z set; no act / nontemporal
// stores there — dgrad launches).  Every chunk needs z (and the bit masks / the addend) from HBM, and the
// plain loop's loads wait a full memory latency per 16-B chunk (the stores before them may alias, so they
// are not hoisted): measured +4.4 ms on the ResNet-50 step against the 3.9 ms of reduce passes it
// replaced.  Here G chunks' loads are issued back to back, from always-valid addresses (element 0 for
// out-of-range chunks; the flags and pointers are selected once, not per load: a per-element "load or not"
// branch would wait vmcnt(0) per element), and then the G chunks are finished and stored.
//   stg_read(r, ch): the staged bf16 values of tile row r, column chunk ch.
//   GMAX: chunks per load group (a 64-column tile takes 2: its kernel then stays within 168 VGPRs, three
//   workgroups per CU)
//   LEAN: the launch has no addend, no second BN and no bit mask (the caller checked): only z is loaded
//   (the generic path loads z2 / addend / mask bytes from always-valid aliases of z when they are absent)
template <int ROWS, int CPR, int NT, class StgRead, int GMAX = 4, bool LEAN = false>
__device__ __forceinline__ void epi_bst_chunks(const Epi& e, const EpiStatCols& sc, StgRead stg_read, int64_t m0,
                                               int64_t n0, int64_t M, int64_t N, float (&st1)[8], float (&st2)[8],
                                               float (&st3)[8]) {
  constexpr int ITERS = ROWS * CPR / NT;
  constexpr int G = ITERS < GMAX ? ITERS : GMAX;  // (8 pushed the gathered wide-tile kernels into scratch)
  static_assert(ITERS % G == 0, "groups cover the tile");
  const int tid = threadIdx.x;
  const bool has_add = !LEAN && e.addend != nullptr, use_bits = !LEAN && e.bst_bits != nullptr;
  const bf16_t* adp = has_add ? e.addend : e.bst_z;
  const uint8_t* abp = e.addend_bits ? e.addend_bits : reinterpret_cast<const uint8_t*>(e.bst_z);
  const uint32_t ab_or = e.addend_bits ? 0u : 0xFFu;
  const uint8_t* zbp = use_bits ? e.bst_bits : reinterpret_cast<const uint8_t*>(e.bst_z);
  const bool dual = !LEAN && e.bst_z2 != nullptr;
  const bf16_t* z2p = dual ? e.bst_z2 : e.bst_z;
  float mu2[8];
  {
    const int64_t n = n0 + (tid % CPR) * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) mu2[q] = (dual && n + q < N) ? e.bst_mean2[n + q] : 0.f;
  }
  float scl[8], shf[8];  // the BN's scale / shift of this thread's (fixed) column chunk: the recomputed mask
  {
    const int64_t n = n0 + (tid % CPR) * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool ok = e.bst_ss && n + q < N;
      scl[q] = ok ? e.bst_ss[n + q] : 0.f;
      shf[q] = ok ? e.bst_ss[N + n + q] : 0.f;
    }
  }
#pragma unroll 1
  for (int c0 = tid; c0 < ROWS * CPR; c0 += G * NT) {
    u16x8 z[G], a[G], z2[G];
    uint32_t ab[G], zb[G];
    int64_t off[G];
    bool ok[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int c = c0 + u * NT;
      const int r = c / CPR, ch = c % CPR;
      const int64_t m = m0 + r, n = n0 + ch * 8;
      ok[u] = m < M && n < N;
      off[u] = ok[u] ? epi_row(e, m) * e.ldc + n : 0;
      z[u] = *reinterpret_cast<const u16x8*>(e.bst_z + off[u]);
      if constexpr (LEAN) {
        z2[u] = a[u] = z[u];
        ab[u] = zb[u] = 0u;
      } else {
        z2[u] = *reinterpret_cast<const u16x8*>(z2p + off[u]);
        a[u] = *reinterpret_cast<const u16x8*>(adp + off[u]);
        ab[u] = (uint32_t)abp[off[u] >> 3] | ab_or;
        zb[u] = zbp[off[u] >> 3];
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (!ok[u]) continue;
      const int c = c0 + u * NT;
      u16x8 o = stg_read(c / CPR, c % CPR);
      if (has_add) {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(bf2f(o[q]) + ((ab[u] >> q) & 1u ? bf2f(a[u][q]) : 0.f));
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float zf = bf2f(z[u][q]);
        const bool keep = use_bits ? ((zb[u] >> q) & 1u) != 0u : fmaf(zf, scl[q], shf[q]) > 0.f;
        const float g = keep ? bf2f(o[q]) : 0.f;
        st1[q] += g;
        st2[q] = fmaf(g, zf - sc.k[q], st2[q]);
        if (!LEAN) st3[q] = fmaf(g, bf2f(z2[u][q]) - mu2[q], st3[q]);
      }
      *reinterpret_cast<u16x8*>((bf16_t*)e.C + off[u]) = o;
    }
  }
}

// flush of a tile's statistics; with a second BN (bst_z2) also (sum g, sum g (z2 - mean2)) into bst_table2
// (st1 is reduced in place by a flush, so the second one gets a copy; an LDS-only barrier separates the
// two uses of the scratch)
__device__ __forceinline__ void epi_stats_flush_all(const Epi& epi, float (&st1)[8], float (&st2)[8], float (&st3)[8],
                                                    float* red, int cpr, int nt, int tm, int64_t n0, int64_t N) {
  float g1[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) g1[q] = st1[q];
  epi_stats_flush(epi, st1, st2, red, cpr, nt, tm, n0, N);
  if (epi.bst_z2) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    epi_stats_flush(epi, g1, st3, red, cpr, nt, tm, n0, N, epi.bst_table2);
  }
}

// addend (optionally bit-masked) of the 8 (or 4) consecutive elements at (crow, n), n 8- (4-) aligned
__device__ __forceinline__ void epi_addend8(const Epi& e, int64_t crow, int64_t n, float (&a)[8]) {
  const int64_t off = crow * e.ldc + n;
  const u16x8 v = *reinterpret_cast<const u16x8*>(e.addend + off);
  const uint32_t mb = e.addend_bits ? e.addend_bits[off >> 3] : 0xFFu;
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = (mb >> q) & 1u ? bf2f(v[q]) : 0.f;
}
__device__ __forceinline__ void epi_addend4(const Epi& e, int64_t crow, int64_t n, float (&a)[4]) {
  const int64_t off = crow * e.ldc + n;
  const u16x4 v = *reinterpret_cast<const u16x4*>(e.addend + off);
  const uint32_t mb = e.addend_bits ? (uint32_t)e.addend_bits[off >> 3] >> (off & 7) : 0xFu;
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = (mb >> q) & 1u ? bf2f(v[q]) : 0.f;
}


constexpr int WT_NT = 512;          // threads of a 256 x 256 tile workgroup
constexpr int WT_SROW = 256 + 8;    // epilogue staging row (bf16 elements)
constexpr int WT_STAGE_BYTES = 256 * WT_SROW * 2;
constexpr int WT_STATS_BYTES = (WT_NT / 64) * 256 * 2 * 4;  // BN-statistics scratch

// the wave's bias values, loaded once per tile: column n0 + wc*(16*JT) + 16*j + 4*(lane>>4) + q -> bv[j][q]
// (zero past N or without a bias): 4*JT loads a thread instead of one per accumulator element.
template <int JT = 4>
__device__ __forceinline__ void epi_bias_cols(const Epi& epi, int64_t n0, int64_t N, int wc, int lane,
                                              float (&bv)[JT][4]) {
#pragma unroll
  for (int j = 0; j < JT; ++j) {
    const int64_t n = n0 + wc * 16 * JT + 16 * j + 4 * (lane >> 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) bv[j][q] = 0.f;
    if (!epi.bias) continue;
    // element loads: a bias may be a view into a flat parameter buffer at any element offset
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (n + q < N)
        bv[j][q] = epi.bias_f32 ? ((const float*)epi.bias)[n + q] : bf2f(((const bf16_t*)epi.bias)[n + q]);
  }
}

// Shared epilogue of the 256 x 256 tiles.  WCOLS = wave columns: 4 (8 waves of 128 x 64, acc[8][4]: the
// wide kernel of gemm_conv.hip and gemm_pp.hip) or 2 (4 waves of 128 x 128, acc[8][8]: gemm_pp4.hip).
// acc[i][j][q] is C(row wr*128 + 16 i + (lane & 15), col wc*(16*JT) + 16 j + 4 (lane >> 4) + q).
// BST: compile the BN-backward statistics path (epi_bst_chunks).  Off for the kernels that never produce a
// BN's dy (gathered forward / weight-gradient loaders of the wide kernel): the extra epilogue code pushed
// their main loops into scratch spills.  BSTG: chunks per load group of the BN-backward sums (each group
// is one exposed z-load latency; a short-K tile — the 56^2 1x1 dgrads, K = 64 — has nothing else to hide
// it behind).
template <int WCOLS = 4, bool BST = true, int BSTG = PDA_BSTG>
__device__ __forceinline__ void wide_tile_epilogue(const f32x4 (&acc)[8][16 / WCOLS], char* smem, int stats_off,
                                                   const Epi& epi, int64_t m0, int64_t n0, int64_t M, int64_t N, int tm,
                                                   int split, bool reduced = false) {
  constexpr int JT = 16 / WCOLS, NT = 128 * WCOLS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WCOLS, wc = wid % WCOLS;
  const bool to_slab = epi.slab && !reduced;  // reduced: acc is the split-K total (splitk_fixup)
  if (to_slab || epi.c_f32) {
    // fp32 output (split-K slab partials or an fp32 C): 16-B stores straight from the accumulators
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t m = m0 + wr * 128 + 16 * i + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < JT; ++j) {
        const int64_t n = n0 + wc * 16 * JT + 16 * j + 4 * (lane >> 4);
        if (n >= N) continue;
        f32x4 v = acc[i][j];
        if (to_slab) {
          *reinterpret_cast<f32x4*>(epi.slab + (int64_t)split * M * N + m * N + n) = v;
          continue;
        }
        const int64_t crow = epi_row(epi, m);
        if (epi.bias) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[q] += epi.bias_f32 ? ((const float*)epi.bias)[n + q] : bf2f(((const bf16_t*)epi.bias)[n + q]);
        }
        if (epi.relu) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
        }
        if (epi.addend) {
          float a[4];
          epi_addend4(epi, crow, n, a);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += a[q];
        }
        *reinterpret_cast<f32x4*>((float*)epi.C + crow * epi.ldc + n) = v;
      }
    }
    return;
  }

  // epilogue (bf16 output): bias / relu in registers, stage through LDS, coalesced 16-B row stores
  bf16_t* stg = reinterpret_cast<bf16_t*>(smem);
  float bv[JT][4];
  epi_bias_cols<JT>(epi, n0, N, wc, lane, bv);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = wr * 128 + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int cc = wc * 16 * JT + 16 * j + 4 * (lane >> 4);
      f32x4 v = acc[i][j];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += bv[j][q];
      if (epi.relu) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
      }
      u16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
      *reinterpret_cast<u16x4*>(stg + r * WT_SROW + cc) = o;
    }
  }
  __syncthreads();
  constexpr int CPR = 256 / 8;
  static_assert(NT % CPR == 0, "a thread keeps one column chunk");
  const bool want_stats = epi.stats != nullptr;
  float st1[8], st2[8];
  EpiStatCols scol;
  epi_stat_cols(epi, want_stats, n0 + (tid % CPR) * 8, N, scol);
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = 0.f;
  float st3[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) st3[q] = 0.f;
  if (BST && epi.bst_z) {
    auto rd = [&](int r, int ch) { return *reinterpret_cast<const u16x8*>(stg + r * WT_SROW + ch * 8); };
    epi_bst_chunks<256, CPR, NT, decltype(rd), BSTG>(epi, scol, rd, m0, n0, M, N, st1, st2, st3);
  } else
  for (int c = tid; c < 256 * CPR; c += NT) {
    const int r = c / CPR, ch = c % CPR;
    const int64_t m = m0 + r, n = n0 + ch * 8;
    if (m >= M || n >= N) continue;
    const int64_t crow = epi_row(epi, m);
    u16x8 v = *reinterpret_cast<const u16x8*>(stg + r * WT_SROW + ch * 8);
    if (epi.addend) {
      float a[8];
      epi_addend8(epi, crow, n, a);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = f2bf(bf2f(v[q]) + a[q]);
    }
    if (epi.act) epi_act8(epi, crow, n, v);
    if (want_stats) epi_stats8(epi, scol, crow, n, v, st1, st2);
    u16x8* dst = reinterpret_cast<u16x8*>((bf16_t*)epi.C + crow * epi.ldc + n);
    if (epi.nt_store) __builtin_nontemporal_store(v, dst);
    else *dst = v;
  }
  if (want_stats) {
    if (BST) epi_stats_flush_all(epi, st1, st2, st3, reinterpret_cast<float*>(smem + stats_off), CPR, NT, tm, n0, N);
    else epi_stats_flush(epi, st1, st2, reinterpret_cast<float*>(smem + stats_off), CPR, NT, tm, n0, N);
  }
}

// In-kernel split-K fix-up (Epi::tickets): every split stores its fp32 partial tile to its slab and takes
// a ticket; the tile's last arrival sums the S slabs in split order 0..S-1 (its own read back, so the
// total is the same whichever split arrives last: bitwise run-to-run deterministic) into acc, sums the
// [split][M] row sums of A into rowsum_out (tile column 0: the bias gradient), re-zeroes the ticket and
// returns true; the caller then runs the ordinary epilogue on acc (wide_tile_epilogue with reduced =
// true).  Each XCD has its own L2: the release fence before the ticket writes this split's slab back, the
// acquire fence after it keeps the last arrival from reading stale lines.  Replaces the separate
// splitk_reduce_kernel launch, which could only start once the whole GEMM had drained.
template <int WCOLS = 4>
__device__ __forceinline__ bool splitk_fixup(f32x4 (&acc)[8][16 / WCOLS], char* smem, const Epi& epi, int64_t m0,
                                             int64_t n0, int64_t M, int64_t N) {
  constexpr int JT = 16 / WCOLS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WCOLS, wc = wid % WCOLS;
  const int split = blockIdx.y, splits = gridDim.y, ticket = blockIdx.x;
  float* own = epi.slab + (int64_t)split * M * N;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t m = m0 + wr * 128 + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int64_t n = n0 + wc * 16 * JT + 16 * j + 4 * (lane >> 4);
      if (m < M && n < N) *reinterpret_cast<f32x4*>(own + m * N + n) = acc[i][j];
    }
  }
  int* flag = reinterpret_cast<int*>(smem);
  __threadfence();
  __syncthreads();
  if (tid == 0) *flag = atomicAdd(epi.tickets + ticket, 1) == splits - 1 ? 1 : 0;
  __syncthreads();
  const bool last = *flag != 0;
  if (!last) return false;
  __threadfence();
  for (int s = 0; s < splits; ++s) {
    const float* src = epi.slab + (int64_t)s * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t m = m0 + wr * 128 + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < JT; ++j) {
        const int64_t n = n0 + wc * 16 * JT + 16 * j + 4 * (lane >> 4);
        if (m >= M || n >= N) continue;
        const f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + m * N + n));
        acc[i][j] = s == 0 ? t : acc[i][j] + t;
      }
    }
  }
  if (epi.rowsum_out && epi.rowsum_mode == 4 && n0 == 0) {
    const float* rs = (const float*)epi.rowsum;
    for (int r = tid; r < 256; r += blockDim.x) {
      const int64_t m = m0 + r;
      if (m >= M) continue;
      float v = 0.f;
      for (int s = 0; s < splits; ++s) v += __builtin_nontemporal_load(rs + (int64_t)s * M + m);
      if (epi.rowsum_out_bf16) ((bf16_t*)epi.rowsum_out)[m] = f2bf(v);
      else ((float*)epi.rowsum_out)[m] = v;
    }
  }
  if (tid == 0) epi.tickets[ticket] = 0;
  __syncthreads();  // every thread has read the flag before the staged epilogue reuses the LDS
  return true;
}

// Persistent-kernel variant of the bf16 epilogue (gemm_pp.hip): the next tile's operand DMAs are in
// flight, so (1) no barrier may wait on vmcnt (LDS-only barriers: lgkmcnt(0) + s_barrier), and (2) only
// 32 KB of LDS beside the operand ring is free: the tile is staged in four 64-row bands through
// `stage` ([64][256] bf16, 16-B chunks XOR-swizzled by row so both the 8-B fragment writes and the
// 16-B row reads are bank-conflict free).  The BN-statistics scratch reuses `stage` after the bands.
// fp32 / slab outputs go straight from the accumulators (wide_tile_epilogue's path, no LDS).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int band_off(int r, int c) { return r * 256 + (c ^ ((r & 15) << 3)); }

__device__ __forceinline__ void wide_tile_epilogue_banded(const f32x4 (&acc)[8][4], char* stage, const Epi& epi,
                                                          int64_t m0, int64_t n0, int64_t M, int64_t N, int tm) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  if (epi.slab || epi.c_f32) {
    wide_tile_epilogue<4, false>(acc, stage, 0, epi, m0, n0, M, N, tm, 0);  // register path only (no LDS, no barrier)
    return;
  }
  bf16_t* stg = reinterpret_cast<bf16_t*>(stage);
  float bv[4][4];
  epi_bias_cols(epi, n0, N, wc, lane, bv);
  constexpr int CPR = 256 / 8;
  const bool want_stats = epi.stats != nullptr;
  float st1[8], st2[8];
  EpiStatCols scol;
  epi_stat_cols(epi, want_stats, n0 + (tid % CPR) * 8, N, scol);
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = 0.f;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    if (wr == (b >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = (b & 1) * 4 + ii;
        const int r = 16 * ii + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cc = wc * 64 + 16 * j + 4 * (lane >> 4);
          f32x4 v = acc[i][j];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += bv[j][q];
          if (epi.relu) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
          }
          u16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
          *reinterpret_cast<u16x4*>(stg + band_off(r, cc)) = o;
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int c = tid; c < 64 * CPR; c += WT_NT) {
      const int r = c / CPR, ch = c % CPR;
      const int64_t m = m0 + b * 64 + r, n = n0 + ch * 8;
      if (m >= M || n >= N) continue;
      const int64_t crow = epi_row(epi, m);
      u16x8 v = *reinterpret_cast<const u16x8*>(stg + band_off(r, ch * 8));
      if (epi.addend) {
        float a[8];
        epi_addend8(epi, crow, n, a);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = f2bf(bf2f(v[q]) + a[q]);
      }
      if (epi.act) epi_act8(epi, crow, n, v);
      if (want_stats) epi_stats8(epi, scol, crow, n, v, st1, st2);
      *reinterpret_cast<u16x8*>((bf16_t*)epi.C + crow * epi.ldc + n) = v;
    }
    lds_barrier();
  }
  if (want_stats) {
    epi_stats_flush(epi, st1, st2, reinterpret_cast<float*>(stage), CPR, WT_NT, tm, n0, N);
    lds_barrier();  // the scratch is the next tile's staging band
  }
}

}  // namespace
}  // namespace pda
