// Streaming forward of a short-K 1x1 stride-1 convolution with the forward BatchNorm statistics in its
// epilogue (the 1x1 expansions of ResNet-50's bottlenecks).
//
//   y[M, N] = x[M, K] * w[N, K]^T        (1x1 conv: K = C_in in {64, 128, 256}, N = C_out, w = OHWI [C_out][C_in])
//
// plus, per column, sum(y - k) and sum((y - k)^2) of the bf16-rounded output (k = stats_shift), atomically added
// to row (workgroup % stats_rows) of the zero-initialised [stats_rows][2][N] table — the contract of
// gemm_epi.h:epi_stats8 / epi_stats_flush that the BN finalize reads.
//
// The 56^2 64 -> 256, 28^2 128 -> 512 and 14^2 256 -> 1024 expansions are HBM-bound (the output is 4x the
// input) but the 256 x 256 pipelined tile runs them at 3.4-4.1 TB/s (profiles/r6_resnet50_bs640_pmc.md,
// r6_conv_table_bs640.jsonl): one workgroup per CU does load -> 1-4 k-steps -> LDS-staged epilogue -> stores
// with nothing of its own to overlap.  Same shape as dgrad_stream.hip, transposed weight access:
//   * one wave owns 64 output channels for the whole launch; its A fragments (w rows, 64 x K) sit in VGPRs,
//     loaded once as 16-B rows (K-major weight: no gather);
//   * a wave walks 16- or 32-row tiles (grid-stride, persistent) with the NEXT tile's x fragments in flight under the
//     current tile's MFMAs, epilogue and stores;
//   * the 16 x 64 accumulator block goes through a wave-private LDS patch (no workgroup barrier) into 16-B row
//     chunks; lane l keeps column chunk l & 7 for the whole launch, so its statistics stay in registers and are
//     flushed once per wave.
// PDA_FWD_STREAM=0 keeps the 256 x 256 tile.
#include "pda_common.h"
#include "pda_kernels.h"
#include "gemm_epi.h"

#include <cstdlib>

namespace pda {
namespace {

typedef __bf16 fsbf16x8 __attribute__((ext_vector_type(8)));

constexpr int FS_NT = 256;    // 4 waves per workgroup (fewer when N < 256)
constexpr int FS_PITCH = 72;  // LDS patch row pitch (bf16): 144 B, 16-B aligned, rows 4 banks apart

struct FSArgs {
  const bf16_t* x;  // [M][K]
  const bf16_t* w;  // [N][K]
  int64_t M;
  int N;
  int64_t ntiles;   // ceil(M / rows per tile)
  Epi epi;          // C = y (bf16, ldc = N); stats / stats_shift / stats_rows (optional)
};

template <int K, bool STATS, int ROWS>
__global__ void __launch_bounds__(FS_NT) fwd_stream_kernel(FSArgs a) {
  constexpr int KS = K / 32;      // MFMA k-steps
  constexpr int RB = ROWS / 16;   // 16-row MFMA blocks per tile
  constexpr int CH = ROWS / 8;    // 16-B epilogue chunks per lane per tile
  __shared__ __attribute__((aligned(16))) bf16_t patch[FS_NT / 64][ROWS * FS_PITCH];
  const Epi& e = a.epi;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int N = a.N;
  const int cb = (blockIdx.y * nw + wid) * 64;  // this wave's 64 output channels
  bf16_t* stg = patch[wid];

  // A fragments, once: lane l holds w[n = cb + 16 j + (l & 15)][k = 32 kk + 8 (l >> 4) + i]
  fsbf16x8 wf[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
      wf[j][kk] = *reinterpret_cast<const fsbf16x8*>(a.w + (int64_t)(cb + 16 * j + (lane & 15)) * K + 32 * kk +
                                                     8 * (lane >> 4));

  const int nc = cb + 8 * (lane & 7);  // this lane's epilogue chunk: columns nc .. nc + 7
  float kmu[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) kmu[q] = STATS ? e.stats_shift[nc + q] : 0.f;

  // B fragments of one tile: lane l holds x[row t * ROWS + 16 b + (l & 15)][32 kk + 8 (l >> 4) + i]
  auto load = [&](int64_t t, fsbf16x8 (&xf)[RB][KS]) {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const int64_t mrow = t * ROWS + 16 * b + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
        xf[b][kk] = mrow < a.M ? *reinterpret_cast<const fsbf16x8*>(a.x + mrow * K + 32 * kk + 8 * (lane >> 4))
                               : fsbf16x8{};
    }
  };

  float st1[8], st2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = 0.f;

  int64_t t = blockIdx.x;
  fsbf16x8 cur[RB][KS];
  if (t < a.ntiles) load(t, cur);
  for (; t < a.ntiles; t += gridDim.x) {
    const int64_t tn = t + gridDim.x;
    fsbf16x8 nxt[RB][KS];
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
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], cur[b][kk], acc[b][j], 0, 0, 0);
    // acc[b][j][q] = y[row t*ROWS + 16 b + (lane & 15)][col cb + 16 j + 4 (lane >> 4) + q]: bf16 into the patch
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = f2bf(acc[b][j][q]);
        *reinterpret_cast<u16x4*>(stg + (16 * b + (lane & 15)) * FS_PITCH + 16 * j + 4 * (lane >> 4)) = o;
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int r = (lane >> 3) + 8 * u;
      const int64_t m = t * ROWS + r;
      const u16x8 o = *reinterpret_cast<const u16x8*>(stg + r * FS_PITCH + 8 * (lane & 7));
      if (m >= a.M) continue;
      if constexpr (STATS) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float d = bf2f(o[q]) - kmu[q];
          st1[q] += d;
          st2[q] = fmaf(d, d, st2[q]);
        }
      }
      *reinterpret_cast<u16x8*>((bf16_t*)e.C + m * N + nc) = o;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the patch is rewritten by the next tile
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) cur[b][kk] = nxt[b][kk];
  }
  if constexpr (STATS) {
    // lanes l, l ^ 8, l ^ 16, ... share column chunk l & 7: reduce, then lanes 0..7 add the wave's 64 columns
#pragma unroll
    for (int off = 8; off < 64; off <<= 1)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        st1[q] += __shfl_xor(st1[q], off, 64);
        st2[q] += __shfl_xor(st2[q], off, 64);
      }
    if (lane < 8) {
      const int64_t row = (int64_t)(blockIdx.x % (unsigned)e.stats_rows) * 2 * N;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        unsafeAtomicAdd(e.stats + row + nc + q, st1[q]);
        unsafeAtomicAdd(e.stats + row + N + nc + q, st2[q]);
      }
    }
  }
}

int g_fwd_stream_override = -1;  // set_fwd_stream(): tests / A/Bs switch the path at run time

int fwd_stream_mode() {
  static const int m = [] {
    const char* s = getenv("PDA_FWD_STREAM");
    return s ? atoi(s) : 1;  // 0 off; 1 K in {64, 128}; 2 also K = 256
  }();
  return g_fwd_stream_override >= 0 ? g_fwd_stream_override : m;
}

int fwd_stream_waves_per_cu() {
  static const int w = [] {
    const char* s = getenv("PDA_FWD_STREAM_WAVES");
    const int v = s ? atoi(s) : 12;
    return v > 0 ? v : 12;
  }();
  return w;
}

int fwd_stream_rows() {  // PDA_FWD_STREAM_ROWS: output rows per tile (16 or 32)
  static const int r = [] {
    const char* s = getenv("PDA_FWD_STREAM_ROWS");
    return (s && atoi(s) == 32) ? 32 : 16;
  }();
  return r;
}

bool fwd_deterministic_env() {
  const char* s = getenv("PDA_DETERMINISTIC");
  return s != nullptr && s[0] == '1';
}

template <int K, int ROWS>
hipError_t launch_fs(const FSArgs& a, bool stats, dim3 grid, int nt, hipStream_t st) {
  if (stats) fwd_stream_kernel<K, true, ROWS><<<grid, nt, 0, st>>>(a);
  else fwd_stream_kernel<K, false, ROWS><<<grid, nt, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace

void set_fwd_stream(int mode) { g_fwd_stream_override = mode; }

bool fwd_stream_ok(int64_t M, int64_t N, int64_t K, const Epi& epi) {
  const int mode = fwd_stream_mode();
  if (mode == 0) return false;
  if (K != 64 && K != 128 && !(mode == 2 && K == 256)) return false;
  if (N % 64 != 0 || N > 65535 * 256 || M <= 0) return false;
  if (epi.c_f32 || epi.slab || epi.bias || epi.relu || epi.act || epi.rm_on || epi.nt_store || epi.rowsum ||
      epi.addend || epi.bst_z)
    return false;
  if (epi.ldc != N) return false;
  if (epi.stats && (!epi.stats_shift || epi.stats_rows < 1)) return false;
  return true;
}

hipError_t fwd_stream(const bf16_t* x, const bf16_t* w, int64_t M, int64_t N, int64_t K, const Epi& epi,
                      hipStream_t st) {
  if (!fwd_stream_ok(M, N, K, epi)) return hipErrorInvalidValue;
  const int rows = K == 256 ? 16 : fwd_stream_rows();
  FSArgs a{x, w, M, (int)N, (M + rows - 1) / rows, epi};
  const int nw = N >= 256 ? 4 : (int)(N / 64);
  const int gy = (int)(N / (64 * nw));
  int64_t gx = (int64_t)256 * fwd_stream_waves_per_cu() / (nw * gy);
  if (gx < 1) gx = 1;
  if (gx > a.ntiles) gx = a.ntiles;
  // fixed-order sums (one add per statistics-table row) in deterministic mode and for problems the 256 x 256
  // tile would cover in at most stats_rows tiles (as dgrad_stream.hip)
  if (epi.stats && (fwd_deterministic_env() || M <= (int64_t)256 * epi.stats_rows) && gx > epi.stats_rows)
    gx = epi.stats_rows;
  const dim3 grid((unsigned)gx, (unsigned)gy);
  const bool stats = epi.stats != nullptr;
  if (K == 64) return rows == 32 ? launch_fs<64, 32>(a, stats, grid, nw * 64, st) : launch_fs<64, 16>(a, stats, grid, nw * 64, st);
  if (K == 128)
    return rows == 32 ? launch_fs<128, 32>(a, stats, grid, nw * 64, st) : launch_fs<128, 16>(a, stats, grid, nw * 64, st);
  return launch_fs<256, 16>(a, stats, grid, nw * 64, st);
}

}  // namespace pda
