// Streaming data gradient of a short-K 1x1 stride-1 convolution with the BN-backward sums in its epilogue
// (VERDICT r5 "next" #1).
//
//   dx[M, N] = dy[M, K] * w[K, N]        (1x1 conv: K = C_out of the conv, N = C_in; K in {64, 128})
//
// plus, per column, sum(g) and sum(g (z - mean)) (and for a downsample block's second BN sum(g (z2 - mean2)))
// with g = dx masked by the BN's ReLU — the epilogue contract of gemm_epi.h:epi_bst_chunks.
//
// Why a kernel of its own: at K = 64 the GEMM is 2 MFMA k-steps per output tile, so the 256 x 256 pipelined
// tile (gemm_pp.hip, one 512-thread workgroup per CU, 256 VGPRs) spends each tile in a chain of exposed
// latencies — operand DMA, MFMA, LDS staging, z loads, stores — with nothing of its own to overlap: the
// 56^2 256<-64 dgrad with sums ran at 0.72 ms (3.2 TB/s) against 0.34 ms plain
// (profiles/r5_short_k_dgrad_tiles.jsonl).  The work is HBM-bound (out + z, and the addend / z2 / mask of a
// block output, against a 1/4-size dy), so this kernel is shaped for bytes in flight, not MFMA reuse:
//   * one wave owns 64 output columns for the whole launch: its B fragments (w, K x 64) live in VGPRs
//     (32 at K = 64, 64 at K = 128) and are loaded once;
//   * a wave walks 16- or 32-row tiles (grid-stride, persistent); the NEXT tile's dy fragments and its z / addend /
//     z2 / mask chunks are loaded into registers before the current tile's MFMAs and epilogue run, so each
//     wave always has one tile of loads in flight behind its own compute and stores;
//   * the 16 x 64 accumulator block is transposed through a wave-private LDS patch (no workgroup barrier)
//     into 16-B row chunks: lane l keeps column chunk l & 7 for the whole launch, so its BN sums stay in
//     registers and are flushed once per wave (lanes sharing a chunk reduced by xor shuffles, then one
//     atomic add per column into the statistics-table row of the workgroup);
//   * register footprint for 2-4 waves per SIMD (K = 64: 104-195 VGPRs; K = 128: 173-226; the dual-BN
//     variant at K = 128, one launch per step, takes 1 wave per SIMD).
// PDA_DGRAD_STREAM=0 falls back to the 256 x 256 tile.
#include "pda_common.h"
#include "pda_kernels.h"
#include "gemm_epi.h"

#include <cstdlib>

namespace pda {
namespace {

typedef __bf16 dsbf16x8 __attribute__((ext_vector_type(8)));

constexpr int DS_NT = 256;     // 4 waves per workgroup (fewer when N < 256)
constexpr int DS_PITCH = 72;   // LDS patch row pitch (bf16): 144 B, 16-B aligned, rows 4 banks apart

struct DSArgs {
  const bf16_t* dy;  // [M][K]
  const bf16_t* w;   // [K][N]: the 1x1 conv's OHWI weight (row k = output channel, N input channels)
  int64_t M;
  int N;
  int64_t ntiles;    // ceil(M / 16)
  Epi epi;           // C = dx (bf16, ldc = N); addend / addend_bits; bst_* / stats / stats_shift / stats_rows
};

// FULL: addend (optionally bit-masked), the BN mask from bst_bits or bst_ss; DUAL (with FULL): the second BN
// (z2) of a downsample block's output; otherwise LEAN: only z and the scale / shift mask (a bn1 / bn2 output: conv2 / conv3 dgrads).
// BST: the BN-backward sums (without: a plain dgrad with an optional addend).
template <int K, bool BST, bool FULL, bool DUAL, int ROWS>
__global__ void __launch_bounds__(DS_NT) dgrad_stream_kernel(DSArgs a) {
  constexpr int KS = K / 32;     // MFMA k-steps
  constexpr int RB = ROWS / 16;  // 16-row MFMA blocks per tile
  constexpr int CH = ROWS / 8;   // 16-B epilogue chunks per lane per tile
  __shared__ __attribute__((aligned(16))) bf16_t patch[DS_NT / 64][ROWS * DS_PITCH];
  const Epi& e = a.epi;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int N = a.N;
  const int cb = (blockIdx.y * nw + wid) * 64;  // this wave's 64 columns
  bf16_t* stg = patch[wid];

  // B fragments, once: first MFMA operand, lane l holds w[k = 32 kk + 8 (l >> 4) + i][n = cb + 16 j + (l & 15)]
  dsbf16x8 bfr[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const bf16_t* p = a.w + (int64_t)(32 * kk + 8 * (lane >> 4)) * N + cb + 16 * j + (lane & 15);
      u16x8 v;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = p[(int64_t)i * N];
      bfr[j][kk] = __builtin_bit_cast(dsbf16x8, v);
    }

  // this lane's epilogue chunk: columns nc .. nc + 7 of rows (lane >> 3) + 8 u of every tile
  const int nc = cb + 8 * (lane & 7);
  // FULL launches take the BN mask from bst_bits (a block output: its residual BN wrote the bits); LEAN ones
  // recompute it from z and the BN's scale / shift
  float kmu[8], scl[8], shf[8], mu2[8];
  constexpr bool dual = DUAL;
  const bool has_add = (FULL || !BST) && e.addend != nullptr;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    kmu[q] = BST ? e.stats_shift[nc + q] : 0.f;
    scl[q] = (BST && !FULL) ? e.bst_ss[nc + q] : 0.f;
    shf[q] = (BST && !FULL) ? e.bst_ss[N + nc + q] : 0.f;
    mu2[q] = dual ? e.bst_mean2[nc + q] : 0.f;
  }
  // absent operands load from always-valid aliases (no per-load branches: each would wait vmcnt(0))
  // (every alias spans [M][N]: z with the sums, else the output itself — dy is only [M][K])
  const bf16_t* zp = BST ? e.bst_z : static_cast<const bf16_t*>(e.C);
  const bf16_t* adp = has_add ? e.addend : zp;
  const uint8_t* abp = (has_add && e.addend_bits) ? e.addend_bits : reinterpret_cast<const uint8_t*>(zp);
  const uint32_t ab_or = (has_add && e.addend_bits) ? 0u : 0xFFu;
  const uint8_t* zbp = FULL ? e.bst_bits : reinterpret_cast<const uint8_t*>(zp);
  const bf16_t* z2p = dual ? e.bst_z2 : zp;

  struct Pre {
    dsbf16x8 af[RB][KS];  // dy fragments: lane l holds dy[row t*ROWS + 16 b + (l & 15)][32 kk + 8 (l >> 4) + i]
    u16x8 z[CH], ad[CH], z2[CH];
    uint32_t zb[CH], ab[CH];
  };
  auto load = [&](int64_t t, Pre& p) {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const int64_t mrow = t * ROWS + 16 * b + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        if (mrow < a.M)
          p.af[b][kk] = *reinterpret_cast<const dsbf16x8*>(a.dy + mrow * K + 32 * kk + 8 * (lane >> 4));
        else
          p.af[b][kk] = dsbf16x8{};
      }
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int64_t m = t * ROWS + (lane >> 3) + 8 * u;
      const int64_t off = m < a.M ? m * N + nc : 0;
      if constexpr (BST) p.z[u] = *reinterpret_cast<const u16x8*>(zp + off);
      if constexpr (FULL || !BST) p.ad[u] = *reinterpret_cast<const u16x8*>(adp + off);
      if constexpr (FULL) {
        if constexpr (DUAL) p.z2[u] = *reinterpret_cast<const u16x8*>(z2p + off);
        p.ab[u] = (uint32_t)abp[off >> 3] | ab_or;
        p.zb[u] = zbp[off >> 3];
      } else if constexpr (!BST) {
        p.ab[u] = (uint32_t)abp[off >> 3] | ab_or;
      }
    }
  };

  float st1[8], st2[8], st3[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = st3[q] = 0.f;

  int64_t t = blockIdx.x;
  Pre cur;
  if (t < a.ntiles) load(t, cur);
  for (; t < a.ntiles; t += gridDim.x) {
    const int64_t tn = t + gridDim.x;
    Pre nxt;
    if (tn < a.ntiles) load(tn, nxt);  // in flight under this tile's MFMAs, epilogue and stores
    f32x4 acc[RB][4];
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], cur.af[b][kk], acc[b][j], 0, 0, 0);
    // acc[b][j][q] = dx[row t*ROWS + 16 b + (lane & 15)][col cb + 16 j + 4 (lane >> 4) + q]: bf16 into the patch
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = f2bf(acc[b][j][q]);
        *reinterpret_cast<u16x4*>(stg + (16 * b + (lane & 15)) * DS_PITCH + 16 * j + 4 * (lane >> 4)) = o;
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int r = (lane >> 3) + 8 * u;
      const int64_t m = t * ROWS + r;
      u16x8 o = *reinterpret_cast<const u16x8*>(stg + r * DS_PITCH + 8 * (lane & 7));
      if (m >= a.M) continue;
      if (has_add) {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(bf2f(o[q]) + ((cur.ab[u] >> q) & 1u ? bf2f(cur.ad[u][q]) : 0.f));
      }
      if constexpr (BST) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float zf = bf2f(cur.z[u][q]);
          bool keep;
          if constexpr (FULL) keep = ((cur.zb[u] >> q) & 1u) != 0u;
          else keep = fmaf(zf, scl[q], shf[q]) > 0.f;
          const float g = keep ? bf2f(o[q]) : 0.f;
          st1[q] += g;
          st2[q] = fmaf(g, zf - kmu[q], st2[q]);
          if constexpr (DUAL) st3[q] = fmaf(g, bf2f(cur.z2[u][q]) - mu2[q], st3[q]);
        }
      }
      *reinterpret_cast<u16x8*>((bf16_t*)e.C + m * N + nc) = o;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the patch is rewritten by the next tile
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    cur = nxt;
  }
  if constexpr (BST) {
    // lanes l, l ^ 8, l ^ 16, ... share column chunk l & 7: reduce, then lanes 0..7 add the wave's 64 columns
#pragma unroll
    for (int off = 8; off < 64; off <<= 1)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        st1[q] += __shfl_xor(st1[q], off, 64);
        st2[q] += __shfl_xor(st2[q], off, 64);
        if constexpr (DUAL) st3[q] += __shfl_xor(st3[q], off, 64);
      }
    if (lane < 8) {
      const int64_t row = (int64_t)(blockIdx.x % (unsigned)e.stats_rows) * 2 * N;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        unsafeAtomicAdd(e.stats + row + nc + q, st1[q]);
        unsafeAtomicAdd(e.stats + row + N + nc + q, st2[q]);
        if constexpr (DUAL) {
          unsafeAtomicAdd(e.bst_table2 + row + nc + q, st1[q]);
          unsafeAtomicAdd(e.bst_table2 + row + N + nc + q, st3[q]);
        }
      }
    }
  }
}

int g_stream_override = -1;  // set_dgrad_stream(): tests / A/Bs switch the path at run time

int stream_mode() {
  static const int m = [] {
    const char* s = getenv("PDA_DGRAD_STREAM");
    return s ? atoi(s) : 1;  // 0 off; 1 measured winners; 3 every BN-sums dgrad; 2 also plain short-K dgrads
  }();
  return g_stream_override >= 0 ? g_stream_override : m;
}

int stream_waves_per_cu() {
  static const int w = [] {
    const char* s = getenv("PDA_DGRAD_STREAM_WAVES");
    const int v = s ? atoi(s) : 12;
    return v > 0 ? v : 12;
  }();
  return w;
}

int stream_rows64() {  // PDA_DGRAD_STREAM_ROWS64: rows per tile at K = 64 (16 or 32)
  static const int r = [] {
    const char* s = getenv("PDA_DGRAD_STREAM_ROWS64");
    return (s && atoi(s) == 16) ? 16 : 32;
  }();
  return r;
}

bool deterministic_env() {
  const char* s = getenv("PDA_DETERMINISTIC");
  return s != nullptr && s[0] == '1';
}

template <int K, int ROWS>
hipError_t launch_k(const DSArgs& a, bool bst, bool full, bool dual, dim3 grid, int nt, hipStream_t st) {
  if (dual) dgrad_stream_kernel<K, true, true, true, ROWS><<<grid, nt, 0, st>>>(a);
  else if (bst && full) dgrad_stream_kernel<K, true, true, false, ROWS><<<grid, nt, 0, st>>>(a);
  else if (bst) dgrad_stream_kernel<K, true, false, false, ROWS><<<grid, nt, 0, st>>>(a);
  else dgrad_stream_kernel<K, false, false, false, ROWS><<<grid, nt, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace

void set_dgrad_stream(int mode) { g_stream_override = mode; }

bool dgrad_stream_ok(int64_t M, int64_t N, int64_t K, const Epi& epi) {
  // mode 1 (default): the launches measured faster than the 256 x 256 tile — K = 64 with the sums, one BN
  // (profiles/r6_dgrad_stream.jsonl); 3: every launch with the sums; 2: also plain short-K dgrads
  const int mode = stream_mode();
  if (mode == 0 || (mode != 2 && !epi.bst_z)) return false;
  if (mode == 1 && (K != 64 || epi.bst_z2)) return false;
  if (K != 64 && K != 128) return false;
  if (N % 64 != 0 || N > 65535 * 256 || M <= 0) return false;
  if (epi.c_f32 || epi.slab || epi.bias || epi.relu || epi.act || epi.rm_on || epi.nt_store || epi.rowsum) return false;
  if (epi.ldc != N) return false;
  if (epi.bst_z && (!epi.stats || !epi.stats_shift || epi.stats_rows < 1)) return false;
  // with the sums: FULL (addend / second BN) launches need the bit mask, LEAN ones the scale / shift
  if (epi.bst_z && (epi.addend || epi.bst_z2) && !epi.bst_bits) return false;
  if (epi.bst_z && !(epi.addend || epi.bst_z2 || epi.bst_bits) && !epi.bst_ss) return false;
  if (!epi.bst_z && epi.stats) return false;  // forward statistics are not this kernel's contract
  return true;
}

hipError_t dgrad_stream(const bf16_t* dy, const bf16_t* w, int64_t M, int64_t N, int64_t K, const Epi& epi,
                        hipStream_t st) {
  if (!dgrad_stream_ok(M, N, K, epi)) return hipErrorInvalidValue;
  // rows per tile: 32 at K = 64 (twice the bytes in flight per wave, still 2 waves per SIMD), 16 at K = 128
  // 32 rows for the FULL K = 64 launches (56^2 256<-64 with addend + bit mask: 0.707 ms vs 0.770 at 16 rows
  // and on the tile); LEAN ones measured faster at 16 (0.49 vs 0.52 ms); dual at 32: 1 wave per SIMD
  const bool full_nodual = epi.bst_z && (epi.addend || epi.bst_bits) && !epi.bst_z2;
  const int rows = (K == 64 && full_nodual) ? stream_rows64() : 16;
  DSArgs a{dy, w, M, (int)N, (M + rows - 1) / rows, epi};
  const int nw = N >= 256 ? 4 : (int)(N / 64);
  const int gy = (int)(N / (64 * nw));
  int64_t gx = (int64_t)256 * stream_waves_per_cu() / (nw * gy);
  if (gx < 1) gx = 1;
  if (gx > a.ntiles) gx = a.ntiles;
  // fixed-order sums: every workgroup adds into a table row of its own — in deterministic mode, and for
  // problems the 256 x 256 tile would cover in at most stats_rows tiles (there each row gets one add, so the
  // sums are reproducible; the random-init whole-model equivalence tests amplify a last-bit difference of
  // an atomic order into O(1) BN-gradient changes, test_side_stream_wgrad_matches_single_stream)
  if (epi.bst_z && (deterministic_env() || M <= (int64_t)256 * epi.stats_rows) && gx > epi.stats_rows)
    gx = epi.stats_rows;
  const bool bst = epi.bst_z != nullptr;
  const bool full = bst && (epi.addend || epi.bst_bits || epi.bst_z2);
  const bool dual = bst && epi.bst_z2 != nullptr;
  const dim3 grid((unsigned)gx, (unsigned)gy);
  if (K == 64) {
    if (rows == 32) return launch_k<64, 32>(a, bst, full, dual, grid, nw * 64, st);
    return launch_k<64, 16>(a, bst, full, dual, grid, nw * 64, st);
  }
  return launch_k<128, 16>(a, bst, full, dual, grid, nw * 64, st);
}

}  // namespace pda
