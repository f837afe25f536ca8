// Pipelined 256 x 256 bf16 GEMM for gfx950 (VERDICT r3 "next" #1).
//
// Why a new main loop (profiles/r3_conv_roofline_bs640.md): the 2-stage wide kernel of gemm_conv.hip
// ends every 64-deep K step with `vmcnt(0)` + a workgroup barrier and issues each step's 64 KB of
// LDS-DMA in one burst, in lockstep on all 8 waves, so the matrix pipe idles while both waves of a SIMD
// issue DMAs and while they wait: 53 % MFMA busy at 4096^3.
//
// Structure (cdna_hip_programming.md §5 "256^2 8-phase template", T2/T3/T4/T5):
//   * 512 threads = 8 waves, 2 (M) x 4 (N); each wave owns a 128 x 64 output (acc[8][4], 16x16x32 MFMA),
//     the accumulator layout of the shared 256 x 256 epilogue (gemm_epi.h).
//   * The LDS holds two K-tile slots of four 16 KB "half" images each: Ah0 / Ah1 are the rows
//     {0-63, 128-191} / {64-127, 192-255} of the A tile (every wave's first / second 64-row quadrant
//     row), Bh0 / Bh1 the columns {first / second 32 of every wave's 64 columns}.
//   * A K tile is 4 phases of 16 MFMAs, quadrants (a0,b0) (a0,b1) (a1,b1) (a1,b0).  Each phase reads
//     one operand quadrant into registers, so each half image is released after ONE phase: Bh0 after
//     phase 3 of the previous tile (b0 stays in registers), Ah0 after phase 0, Bh1 after 1, Ah1 after 2.
//     The very next phase refills it with K tile t+2 (2 LDS-DMA per thread), so 7 half images (~1.75 K
//     tiles) stay in flight and every wait in the loop is the same counted `vmcnt(12)` — never 0.
//   * Ping-pong: waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave issues its
//     fragment reads + DMAs (load section) while its partner runs its 16 MFMAs (compute section).
//   * Operands come through buffer descriptors (`buffer_load_dwordx4 ... lds`): one 32-bit offset per
//     lane and DMA; rows past M / N, K past the end and invalid columns read as zero.
//   * K-major operands ([rows][K]) are [128][64] images read with ds_read_b128 (16-B chunks XOR-swizzled
//     by row pair); MN-major operands ([K][rows], the weight gradient's dY^T and X) are [64 k][128]
//     images read with ds_read_b64_tr_b16 (32-B slots XOR-swizzled by k) — no transpose pass.
#include "pda_common.h"
#include "pda_kernels.h"
#include "gemm_epi.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace pda {
namespace {

typedef __bf16 ppbf16x8 __attribute__((ext_vector_type(8)));

constexpr int PP_NT = 512;
constexpr int PP_HALF = 128 * 64 * 2;  // one half image: 128 rows x 64 k, bf16
constexpr int PP_SLOT = 4 * PP_HALF;   // Ah0 Ah1 Bh0 Bh1
constexpr int PP_LDS_LOOP = 2 * PP_SLOT;
constexpr int PP_STATS_OFF = WT_STAGE_BYTES > PP_LDS_LOOP ? WT_STAGE_BYTES : PP_LDS_LOOP;
constexpr int PP_LDS = PP_STATS_OFF + WT_STATS_BYTES;
static_assert(PP_LDS <= 160 * 1024, "LDS budget");
constexpr uint32_t PP_OOB = 0x80000000u;  // an offset past every descriptor's range: reads zero

enum { H_A0 = 0, H_A1 = 1, H_B0 = 2, H_B1 = 3 };

// ---- K-major [128][64] half image: 128-B rows, 16-B chunk XOR ((row >> 1) & 7) (gemm_conv.hip kmaj_off).
// Fragment of the 16 rows from row0 (a multiple of 16), k-substep kk: lane l holds (row0 + (l & 15),
// kk + 8 (l >> 4) + j).  For such rows the XOR key is (l >> 1) & 7 whatever row0 is, so the lane part of
// the address is one of two per-lane offsets (kk = 0 / 32) and row0 folds into the immediate offset.
__device__ __forceinline__ int pp_klane(int lane, int kk) {
  const int key = (lane >> 1) & 7, chunk = (kk >> 3) + (lane >> 4);
  return (lane & 15) * 128 + ((chunk ^ key) << 4);
}
__device__ __forceinline__ ppbf16x8 pp_kfrag(const char* half, int row0, int loff) {
  return *reinterpret_cast<const ppbf16x8*>(half + row0 * 128 + loff);
}

// ---- MN-major [64 k][128] half image: 256-B k-rows, 32-B slots (16 rows) XOR-swizzled by k
// (gemm_conv.hip mn_off<128>).  Thread t of a DMA round fills k-row t / 16 (+ 32 per round), slot t % 16.
__device__ __forceinline__ int pp_mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
__device__ __forceinline__ int pp_mn_col(int t) {  // logical column (multiple of 8) that thread t fetches
  const int p = t & 15, k = t >> 4;
  return ((((p >> 1) ^ pp_mn_swz(k)) & 7) << 4) + (p & 1) * 8;
}
// Fragment (same register layout as the K-major one) by two transposing 8-byte reads: lane l = (g, i)
// reads k-rows kk + 8 g + (i >> 2) (+ 4) at rows row0 + 4 (i & 3) .. + 3.  For row0 a multiple of 16 the
// swizzle key depends on the lane only ((i >> 2) | ((g & 1) << 2)); the row group r = row0 / 16 enters
// as (r ^ key) & 7.
typedef short pp_s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) pp_s16x4 pp_lds_s16x4;
__device__ __forceinline__ ppbf16x8 pp_mfrag(const char* half, int r, int kk, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int key = (i >> 2) | ((g & 1) << 2);
  const int k1 = kk + 8 * g + (i >> 2);
  const int off = k1 * 256 + (((r ^ key) & 7) << 5) + ((i & 3) << 3);
  const pp_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pp_lds_s16x4*)(half + off));
  const pp_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pp_lds_s16x4*)(half + off + 4 * 256));
  return __builtin_bit_cast(ppbf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ void pp_glds(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff = 0) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// The same DMA as inline asm, for kernels that read an MN-major image with ds_read_b64_tr_b16: beside
// a compiler-visible LDS-DMA, hipcc (ROCm 7.2) puts `s_waitcnt vmcnt(0)` in front of every transposing
// LDS read (it cannot tell them apart from the DMA's LDS range), which drains the whole pipeline each
// phase.  Hidden in asm, the DMA is ordered by this kernel's own counted vmcnt waits only (no other
// vector-memory op is in flight in the K loop; the loop drains with vmcnt(0) before the epilogue).
typedef int pp_i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pp_glds_asm(pp_i32x4 r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(r), "s"(lds)
               : "memory", "m0");
}
// ... with a uniform byte offset in soffset (the per-lane offset stays one loop-invariant register)
__device__ __forceinline__ void pp_glds_asm(pp_i32x4 r, uint32_t lds, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(r), "s"(lds), "s"(soff)
               : "memory", "m0");
}

__device__ __forceinline__ void pp_sync() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int QA, int QB, int VAR>
__device__ __forceinline__ void pp_mma(f32x4 (&acc)[8][4], const ppbf16x8 (&a)[8], const ppbf16x8 (&b)[4]) {
  if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[QA * 4 + i][QB * 2 + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[kk * 2 + j], a[kk * 4 + i], acc[QA * 4 + i][QB * 2 + j], 0, 0, 0);
  if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(0);
}

// One operand: element (row, k) = p[row * ld + k] (K-major) or p[k * ld + row] (MN-major); `rows` = M
// (operand A) or N (operand B).
struct PPOp {
  const bf16_t* p;
  int64_t ld, rows;
};

// Operand A as the implicit-GEMM gather of an NHWC tensor [N, H, W, C] with C % 64 == 0 (a 64-deep K
// tile lies inside one tap, so the tap is uniform per K tile):
//   element (m = (n, a, b) of an [N, P, Q] row grid, k = (r, s, c)) = src[n, a*st + o_r + r*tr,
//   b*st + o_c + s*ts, c], zero outside the image.
// Convolution forward (gemm_conv.hip ConvFwdKU): grid = output pixels, st = stride, o = -pad, t = dil.
// Stride-phase data gradient (ConvDgradPhaseKU): src = dy, grid = one phase's dx pixels, st = 1,
// o = the phase's base offsets, t = -tap step, S = taps per row of that phase.
struct PPGather {
  int H, W, C, P, Q, S, st, o_r, o_c, tr, ts;
  uint32_t mC, sC, mS, sS;  // k / C and rs / S as mul-hi + shift (fast_div)
};

// Operand B of a convolution's weight gradient as the gather of its input x [N, H, W, C]: element
// (k = output pixel (n, p, q) of the [N, P, Q] grid, col = (r, s, c)) = x[n, p*st + r*dil - pad,
// q*st + s*dil - pad, c], zero outside the image (gemm_conv.hip ConvWgradMN).  MN-major, so a lane's
// 8 columns (one (r, s) tap, 8 channels) are fixed for the kernel and only its k-rows (pixels) move.
struct PPWg {
  int H, W, C, P, Q, st, pad, dil, S;
  uint32_t mQ, sQ, mP, sP, mC, sC, mS, sS;
};

struct PPArgs {
  PPOp a, b;
  int64_t M, N, K;
  int tiles_n, kt_per_split;
  Epi epi;
  PPGather ga;
  PPWg gb;
  // MN-major operands: the descriptor base advances every 2^rb_shift K tiles, so the per-DMA offsets
  // (t * 64 k-rows * ld) stay 32-bit on K spans of any length (the LM head's weight gradient: ld 50304,
  // K = 32768 tokens is 3.3 GB of k-rows)
  int rb_shift = 30;
  int group_m = 8;  // grouped tile order: tile rows per group (PDA_PP_GROUP, A/B knob)
};

__device__ __forceinline__ uint32_t pp_fdiv(uint32_t n, uint32_t mul, uint32_t shr) {
  return mul ? (__umulhi(n, mul) >> shr) : n;
}
// branch-free form for per-DMA use inside the K loop (mul == 0 encodes d == 1: the n term passes through)
__device__ __forceinline__ uint32_t pp_fdiv_nb(uint32_t n, uint32_t mul, uint32_t shr) {
  return (__umulhi(n, mul) + (n & (mul ? 0u : 0xFFFFFFFFu))) >> shr;
}

// Per-lane DMA source of one operand for this workgroup: a buffer descriptor over its panel (from the
// tile's first row and the split's first K element), the lane's offset for (half 0, round 0), and the
// uniform offsets of half 1 / round 1 / one K tile.
struct PPSrc {
  __amdgpu_buffer_rsrc_t r;
  pp_i32x4 rs;  // the same descriptor as four words (inline-asm DMA)
  // per-lane byte offset v (the only per-lane address register); uniform strides dh (half 1), di (the
  // second DMA of a half), dk (one K tile) travel in soffset.  Validity is explicit per DMA — a lane
  // out of the operand gets PP_OOB — so no element depends on how the hardware range check treats
  // soffset:
  //   K-major: chunk in range for K tile t iff t * 64 < lim; row in range iff rows > h * hr + i * 128
  //   MN-major: column chunk in range iff lim > h * half stride; k-row t * 64 + kr (+32) < rows
  uint32_t v, dh, di, dk;
  int lim, rows;
  int64_t rem;  // bytes from the descriptor base to the operand's end (uncapped)
};

__device__ __forceinline__ pp_i32x4 pp_rsrc_words(const bf16_t* base, int64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  pp_i32x4 w;
  w[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  w[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));  // stride 0
  w[2] = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
  w[3] = 0x00020000;
  return w;
}

template <bool KMAJ, bool IS_A>
__device__ __forceinline__ PPSrc pp_src(const PPOp& op, int64_t r0, int64_t k0, int64_t K, int wid, int lane) {
  PPSrc s;
  const int tid = wid * 64 + lane;
  if constexpr (KMAJ) {
    // image row R = round*64 + wid*8 + lane/8 holds logical chunk (lane & 7) ^ ((R >> 1) & 7); it is
    // tile row (R/64)*128 + h*64 + R%64 (A) or (R/32)*64 + h*32 + R%32 (B)
    const int chunk = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
    const int rr = IS_A ? wid * 8 + (lane >> 3) : (wid >> 2) * 64 + (wid & 3) * 8 + (lane >> 3);
    const bf16_t* base = op.p + r0 * op.ld + k0;
    const int64_t rem = (((op.rows - r0) - 1) * op.ld + (K - k0)) * 2;
    s.r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(rem < 0x7fffffff ? rem : 0x7fffffff),
                                            0x00020000);
    s.rs = pp_rsrc_words(base, rem);
    s.rem = rem;
    s.v = (uint32_t)((rr * op.ld + chunk * 8) * 2);
    s.dh = (uint32_t)((IS_A ? 64 : 32) * op.ld * 2);
    s.di = (uint32_t)(128 * op.ld * 2);
    s.dk = 128u;
    s.lim = (int)(K - k0) - chunk * 8;
    const int64_t rl = op.rows - r0 - rr;  // rows of the operand from the lane's first row
    s.rows = rl > 0x7fffffff ? 0x7fffffff : (int)rl;
  } else {
    // image k-row round*32 + tid/16 holds the 8 logical columns from pp_mn_col(tid): tile row
    // (lc/64)*128 + h*64 + lc%64 (A) or (lc/32)*64 + h*32 + lc%32 (B)
    const int lc = pp_mn_col(tid);
    const int rr = IS_A ? (lc >> 6) * 128 + (lc & 63) : (lc >> 5) * 64 + (lc & 31);
    const int kr = tid >> 4;
    const bf16_t* base = op.p + k0 * op.ld + r0;
    const int64_t rem = (((K - k0) - 1) * op.ld + (op.rows - r0)) * 2;
    s.r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(rem < 0x7fffffff ? rem : 0x7fffffff),
                                            0x00020000);
    s.rs = pp_rsrc_words(base, rem);
    s.rem = rem;
    s.v = (uint32_t)((kr * op.ld + rr) * 2);
    s.dh = (uint32_t)((IS_A ? 64 : 32) * 2);
    s.di = (uint32_t)(32 * op.ld * 2);
    s.dk = (uint32_t)(64 * op.ld * 2);
    const int64_t left = op.rows - r0 - rr;
    s.lim = left > 0x7fffffff ? 0x7fffffff : (int)left;
    const int64_t kl = (K - k0) - kr;  // k-rows from the lane's first
    s.rows = kl > 0x7fffffff ? 0x7fffffff : (int)kl;
  }
  return s;
}

// VAR bits: 1 = s_setprio(1) around each MFMA section, 2 = ping-pong stagger of the two wave groups,
// 4 = a load section issues its refill DMA before its fragment reads, 8 = two 32-MFMA phases per K tile
// Row sums of one 16-row tile of A over a K tile (its two 32-deep k-halves) by MFMA against a ones
// fragment: C = 1 * A^T puts every row's sum in each row of C; lane l (< 16) gets row m = l in c[0].
// The ones operand is rematerialised per call (opaque moves) and C starts at zero, so only the caller's
// running float per quadrant lives across the main loop — the persistent-accumulator form (8 registers
// + 4 for the constant) pushed the MN x MN tile into scratch.
__device__ __forceinline__ float pp_rowsum_pair(const ppbf16x8& f0, const ppbf16x8& f1) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 o;
  asm volatile("v_mov_b32 %0, 0x3f803f80\n\tv_mov_b32 %1, 0x3f803f80\n\tv_mov_b32 %2, 0x3f803f80\n\t"
               "v_mov_b32 %3, 0x3f803f80"
               : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]));
  const ppbf16x8 ones = __builtin_bit_cast(ppbf16x8, o);
  f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, f0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, f1, c, 0, 0, 0);
  return c[0];
}

// row sums of wave WC's row tile of a quadrant (a[kk*4 + i]: k-half kk, row tile i).  WC is a template
// argument: the RS kernels run one copy of the main loop per wave column (a runtime select copies two
// fragments — 8 registers — and a branch splits the loop's scheduling region; either spilled the MN x MN
// loop into scratch)
template <int WC>
__device__ __forceinline__ float pp_rs_tile(const ppbf16x8 (&a)[8]) {
  return pp_rowsum_pair(a[WC], a[WC + 4]);
}
__device__ __forceinline__ float pp_rs_tile(const ppbf16x8 (&a)[8], int wc) {  // runtime-select form
  ppbf16x8 f0 = a[0], f1 = a[4];
  if (wc == 1) { f0 = a[1]; f1 = a[5]; }
  else if (wc == 2) { f0 = a[2]; f1 = a[6]; }
  else if (wc == 3) { f0 = a[3]; f1 = a[7]; }
  return pp_rowsum_pair(f0, f1);
}

template <bool AK, bool BK, int VAR, bool RS = false, int GM = 0>
__global__ void __launch_bounds__(PP_NT, 1) gemm_pp_kernel(PPArgs p) {
  constexpr bool GA = GM == 1;  // A = implicit-GEMM gather (PPGather)
  constexpr bool GB = GM == 2;  // B = weight-gradient gather (PPWg)
  static_assert(!GB || (!AK && !BK), "weight-gradient gather: MN-major operands");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  constexpr bool STAGGER = (VAR & 2) != 0;
  const bool lag = STAGGER && wr == 1;
  constexpr bool EARLY = !AK;  // see ktile
  constexpr bool ASM_DMA = !(AK && BK);  // see pp_glds_asm

  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  grouped_tile(tile, ntiles / p.tiles_n, p.tiles_n, p.group_m, tm, tn);
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int ktiles = (int)((p.K + 63) >> 6);
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int nk = min(ktiles, kt0 + p.kt_per_split) - kt0;  // K tiles of this split
  const int64_t k0 = (int64_t)kt0 * 64;

  const PPSrc sa = pp_src<AK, true>(p.a, m0, k0, p.K, wid, lane);
  const PPSrc sb = pp_src<BK, false>(p.b, n0, k0, p.K, wid, lane);
  // GA: per-lane gather state of the 4 A rows this lane stages (half h, round i: tile row
  // i*128 + h*64 + wid*8 + lane/8): the element offset of its tap-(0, 0) source pixel + chunk, and the
  // pixel's (ih0, iw0) packed in 16 bits each (an invalid row never passes the bounds test)
  int g_pb[4] = {0, 0, 0, 0}, g_hw[4] = {0, 0, 0, 0};
  __amdgpu_buffer_rsrc_t g_r = sa.r;
  if constexpr (GA) {
    const int chunk = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
    const PPGather& g = p.ga;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + (j & 1) * 128 + (j >> 1) * 64 + wid * 8 + (lane >> 3);
      const bool ok = m < p.M;
      const int mm = ok ? (int)m : 0;
      const int q = mm % g.Q, t1 = mm / g.Q;
      const int pp = t1 % g.P, n = t1 / g.P;
      const int ih0 = ok ? pp * g.st + g.o_r : -16384, iw0 = q * g.st + g.o_c;
      g_pb[j] = ((n * g.H + ih0) * g.W + iw0) * g.C + chunk * 8;
      g_hw[j] = (ih0 & 0xFFFF) | (iw0 << 16);
    }
    const int64_t bytes = p.a.rows * 2;  // a.rows carries the tensor's element count for a gather
    g_r = __builtin_amdgcn_make_buffer_rsrc((void*)p.a.p, (short)0, (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff),
                                            0x00020000);
  }

  // GB: the lane's two column contexts (B half h: tile column (lc / 32) * 64 + h * 32 + lc % 32) — tap
  // offsets packed in 16 bits each and channel (-1: column past N) — and its first k-row
  // (no per-lane gather state is kept across the loop: the MN x MN tile has no registers to spare, so
  // each issue recomputes its column's tap and channel — two multiply-high divisions)
  pp_i32x4 gb_rs = sb.rs;
  if constexpr (GB) gb_rs = pp_rsrc_words(p.b.p, p.b.rows * 2);  // b.rows carries x's element count

  // one half image of K tile t (of this split): 2 DMAs per thread; tiles past the split read zero
  // (t & 1) == SLOT at every call site: the slot offsets fold into immediates
  auto issue = [&](auto hid_c, auto slot_c, int t) {
    constexpr int hid = decltype(hid_c)::value;
    constexpr int SLOT = decltype(slot_c)::value;
    constexpr bool isA = hid < 2;
    constexpr bool km = isA ? AK : BK;
    const PPSrc& s = isA ? sa : sb;
    char* dst = smem + SLOT * PP_SLOT + hid * PP_HALF + wid * 1024;
    if constexpr (GA && isA) {
      // tap of this K tile (uniform): k = (r, s, cb); rows whose shifted pixel leaves the image read zero
      const PPGather& g = p.ga;
      const uint32_t k = (uint32_t)(k0 + (int64_t)t * 64);
      const uint32_t rs = pp_fdiv(k, g.mC, g.sC), cb = k - rs * (uint32_t)g.C;
      const uint32_t r = pp_fdiv(rs, g.mS, g.sS), sx = rs - r * (uint32_t)g.S;
      const int dr = (int)r * g.tr, ds = (int)sx * g.ts;
      const int toff = (dr * g.W + ds) * g.C + (int)cb;
      char* dst = smem + SLOT * PP_SLOT + hid * PP_HALF + wid * 1024;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int j = (hid & 1) * 2 + i;
        const int ih = (int)(short)(g_hw[j] & 0xFFFF) + dr, iw = (g_hw[j] >> 16) + ds;
        const bool ok = t < nk && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const uint32_t off = ok ? (uint32_t)(g_pb[j] + toff) * 2u : PP_OOB;
        if constexpr (ASM_DMA) {
          const uint32_t l = __builtin_amdgcn_readfirstlane(
              (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(dst + i * 8192));
          pp_glds_asm(pp_rsrc_words(p.a.p, p.a.rows * 2), l, off);
        } else {
          pp_glds(g_r, dst + i * 8192, off);
        }
      }
      return;
    }
    if constexpr (GB && !isA) {
      // pixel k of each DMA's k-row (round i: +32), its tap-shifted source pixel; zero outside the image
      const PPWg& g = p.gb;
      const int lc = pp_mn_col((int)threadIdx.x);
      const uint32_t col = (uint32_t)n0 + (uint32_t)((lc >> 5) * 64 + (hid & 1) * 32 + (lc & 31));
      const uint32_t rs = pp_fdiv_nb(col, g.mC, g.sC);
      const uint32_t r = pp_fdiv_nb(rs, g.mS, g.sS);
      const uint32_t c = col - rs * (uint32_t)g.C;
      const int dr = (int)r * g.dil - g.pad, ds = (int)(rs - r * (uint32_t)g.S) * g.dil - g.pad;
      const bool cok = col < (uint32_t)p.N;
      const uint32_t kbase = (uint32_t)k0 + (uint32_t)t * 64u + ((uint32_t)threadIdx.x >> 4);
      const uint32_t kend = (uint32_t)p.K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t kk = kbase + (uint32_t)(i * 32);
        const uint32_t nq = pp_fdiv_nb(kk, g.mQ, g.sQ), q = kk - nq * (uint32_t)g.Q;
        const uint32_t n = pp_fdiv_nb(nq, g.mP, g.sP), pp = nq - n * (uint32_t)g.P;
        const int ih = (int)pp * g.st + dr, iw = (int)q * g.st + ds;
        const bool ok = t < nk && kk < kend && cok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const uint32_t off = ok ? (uint32_t)((((int)n * g.H + ih) * g.W + iw) * g.C + (int)c) * 2u : PP_OOB;
        const uint32_t l = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(dst + i * 8192));
        pp_glds_asm(gb_rs, l, off);
      }
      return;
    }
    uint32_t su;
    pp_i32x4 rs = s.rs;
    if constexpr (!km) {
      const uint32_t blk = (uint32_t)t >> p.rb_shift;  // uniform; 0 unless K spans past 2^31 bytes
      su = __builtin_amdgcn_readfirstlane((hid & 1) * s.dh + ((uint32_t)t - (blk << p.rb_shift)) * s.dk);
      const uint64_t adv = (uint64_t)blk * ((uint64_t)s.dk << p.rb_shift);
      const uint64_t b = ((uint64_t)(uint32_t)rs[1] << 32 | (uint32_t)rs[0]) + adv;
      rs[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
      rs[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
      const int64_t left = s.rem - (int64_t)adv;
      rs[2] = __builtin_amdgcn_readfirstlane(left <= 0 ? 0 : (int)(left < 0x7fffffff ? left : 0x7fffffff));
    } else {
      su = __builtin_amdgcn_readfirstlane((hid & 1) * s.dh + (uint32_t)t * s.dk);
    }
    bool ok0, ok1;
    if constexpr (km) {
      constexpr int hr = (hid & 1) * (isA ? 64 : 32);
      const bool kv = t < nk && t * 64 < s.lim;
      ok0 = kv && s.rows > hr;
      ok1 = kv && s.rows > hr + 128;
    } else {
      const bool cv = t < nk && s.lim > (hid & 1) * (isA ? 64 : 32);
      ok0 = cv && t * 64 < s.rows;
      ok1 = cv && t * 64 + 32 < s.rows;
    }
    if constexpr (ASM_DMA) {
      const uint32_t l = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)dst);
      pp_glds_asm(rs, l, ok0 ? s.v : PP_OOB, su);
      pp_glds_asm(rs, l + 8192, ok1 ? s.v : PP_OOB, su + s.di);
    } else {
      pp_glds(s.r, dst, ok0 ? s.v : PP_OOB, su);
      pp_glds(s.r, dst + 8192, ok1 ? s.v : PP_OOB, su + s.di);
    }
  };
  using HA0 = std::integral_constant<int, H_A0>;
  using HA1 = std::integral_constant<int, H_A1>;
  using HB0 = std::integral_constant<int, H_B0>;
  using HB1 = std::integral_constant<int, H_B1>;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;

  const int kl0 = pp_klane(lane, 0), kl1 = pp_klane(lane, 32);
  auto rd_a = [&](const char* half, ppbf16x8 (&f)[8]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (AK) f[kk * 4 + i] = pp_kfrag(half, wr * 64 + 16 * i, kk ? kl1 : kl0);
        else f[kk * 4 + i] = pp_mfrag(half, wr * 4 + i, kk * 32, lane);
      }
  };
  auto rd_b = [&](const char* half, ppbf16x8 (&f)[4]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (BK) f[kk * 2 + j] = pp_kfrag(half, wc * 32 + 16 * j, kk ? kl1 : kl0);
        else f[kk * 2 + j] = pp_mfrag(half, wc * 2 + j, kk * 32, lane);
      }
  };
  // end of a load section: own DMAs of the half read next are done, own fragment reads are done
  auto end_load = [&](auto vm_c) {
    constexpr int VM = decltype(vm_c)::value;
    if constexpr (VM == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (VM == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if constexpr (VM == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else static_assert(VM == -1, "vmcnt literal");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_sync();
  };
  using VM8 = std::integral_constant<int, 8>;
  using VM10 = std::integral_constant<int, 10>;
  using VM12 = std::integral_constant<int, 12>;
  using VMNONE = std::integral_constant<int, -1>;
  auto end_mma = [&]() {
    if constexpr (STAGGER) pp_sync();
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // RS: row sums of A (Epi::rowsum) by MFMA against a ones fragment — C = A * 1 puts every row's sum in
  // each of its columns.  The 4 waves that share A rows split the row tiles (wave wc takes row tile wc
  // of each 64-row quadrant): 2 MFMAs per A quadrant and K tile, +6 % matrix work, no VALU.
  float rsacc[2] = {0.f, 0.f};
  // only tile column 0 sums (every column tile sees the same A rows: the split-K atomics would count
  // them tiles_n times)
  const bool rs_on = RS && n0 == 0;
  auto rs_mma = [&](auto qa_c, const ppbf16x8 (&a)[8], auto wc_c) {
    if constexpr (RS) {
      if (!rs_on) return;
      constexpr int QA = decltype(qa_c)::value;
      rsacc[QA] += pp_rs_tile<decltype(wc_c)::value>(a);
    } else {
      (void)qa_c;
      (void)a;
      (void)wc_c;
    }
  };
  // the main loop, instantiated per wave column for RS (pp_rs_tile) and once otherwise
  auto per_wc = [&](auto body) {
    if constexpr (RS) {
      switch (__builtin_amdgcn_readfirstlane(wc)) {
        case 0: body(std::integral_constant<int, 0>{}); break;
        case 1: body(std::integral_constant<int, 1>{}); break;
        case 2: body(std::integral_constant<int, 2>{}); break;
        default: body(std::integral_constant<int, 3>{}); break;
      }
    } else {
      body(std::integral_constant<int, 0>{});
    }
  };
  auto rs_store = [&]() {
    if constexpr (RS) {
      if (rs_on && (lane >> 4) == 0) {
#pragma unroll
        for (int qa = 0; qa < 2; ++qa) {
          const int64_t m = m0 + wr * 128 + qa * 64 + 16 * wc + (lane & 15);
          if (m >= p.M) continue;
          const float v = rsacc[qa];
          if (p.epi.rowsum_mode == 4) ((float*)p.epi.rowsum)[(int64_t)blockIdx.y * p.M + m] = v;
          else if (p.epi.rowsum_mode == 3) unsafeAtomicAdd((float*)p.epi.rowsum + m, v);
          else if (p.epi.rowsum_mode == 2) ((bf16_t*)p.epi.rowsum)[m] = f2bf(v);
          else ((float*)p.epi.rowsum)[m] = v;
        }
      }
    }
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;

  constexpr bool TWO = (VAR & 8) != 0;
  if constexpr (TWO) {
    // Two phases of 32 MFMAs per K tile: (a0 x b) then (a1 x b).  Phase 0 reads a0 and all of b (16
    // fragments), phase 1 reads a1 (b stays in registers), so Ah0 / Bh0 / Bh1 are released after phase
    // 0 and refilled with K tile t+2 in phase 1; Ah1 is released after phase 1 and refilled with t+1
    // in the next tile's phase 0.  Issue order A0 B0 B1 (t+2) | A1 (t+1): every wait is vmcnt(8).
    // Half the barriers of the 4-phase schedule per MFMA, 192 live registers for the operands.
    ppbf16x8 ta[8], tb0[4], tb1[4];
    issue(HA0{}, S0{}, 0);
    issue(HB0{}, S0{}, 0);
    issue(HB1{}, S0{}, 0);
    issue(HA1{}, S0{}, 0);
    issue(HA0{}, S1{}, 1);
    issue(HB0{}, S1{}, 1);
    issue(HB1{}, S1{}, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0 B0 B1 of tile 0 landed
    pp_sync();
    if (lag) pp_sync();
    auto ktile2 = [&](auto slot_c, int t, auto wc_c) {
      constexpr int SLOT = decltype(slot_c)::value;
      const char* cs = smem + SLOT * PP_SLOT;
      rd_a(cs + H_A0 * PP_HALF, ta);
      rd_b(cs + H_B0 * PP_HALF, tb0);
      rd_b(cs + H_B1 * PP_HALF, tb1);
      if constexpr (SLOT == 0) issue(HA1{}, S1{}, t + 1);
      else issue(HA1{}, S0{}, t + 1);
      end_load(VM8{});
      pp_mma<0, 0, VAR>(acc, ta, tb0);
      pp_mma<0, 1, VAR>(acc, ta, tb1);
      rs_mma(Q0{}, ta, wc_c);
      end_mma();
      rd_a(cs + H_A1 * PP_HALF, ta);
      issue(HA0{}, slot_c, t + 2);
      issue(HB0{}, slot_c, t + 2);
      issue(HB1{}, slot_c, t + 2);
      end_load(VM8{});
      pp_mma<1, 0, VAR>(acc, ta, tb0);
      pp_mma<1, 1, VAR>(acc, ta, tb1);
      rs_mma(Q1{}, ta, wc_c);
      end_mma();
    };
    per_wc([&](auto wc_c) {
      int t2 = 0;
      for (; t2 + 1 < nk; t2 += 2) {
        ktile2(S0{}, t2, wc_c);
        ktile2(S1{}, t2 + 1, wc_c);
      }
      if (t2 < nk) ktile2(S0{}, t2, wc_c);
    });
    if (STAGGER && !lag) pp_sync();
    rs_store();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool reduced = false;
    if constexpr (!AK && !BK) {  // split-K weight gradients: the in-kernel fix-up when the caller gave tickets
      if (p.epi.tickets && p.epi.slab) {
        if (!splitk_fixup(acc, smem, p.epi, m0, n0, p.M, p.N)) return;
        reduced = true;
      }
    }
    wide_tile_epilogue(acc, smem, PP_STATS_OFF, p.epi, m0, n0, p.M, p.N, tm, blockIdx.y, reduced);
    return;
  }

  ppbf16x8 fa[8], fb1[4], fb0e[4], fb0o[4];
  // prologue: K tiles 0 and 1 in the steady-state issue order (Bh0, Ah0, Bh1, Ah1)
  issue(HB0{}, S0{}, 0);
  issue(HA0{}, S0{}, 0);
  issue(HB1{}, S0{}, 0);
  issue(HA1{}, S0{}, 0);
  issue(HB0{}, S1{}, 1);
  issue(HA0{}, S1{}, 1);
  issue(HB1{}, S1{}, 1);
  issue(HA1{}, S1{}, 1);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // Bh0(0), Ah0(0) landed
  pp_sync();
  if constexpr (!EARLY) {
    rd_b(smem + H_B0 * PP_HALF, fb0e);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_sync();
  }
  if (lag) pp_sync();

  // Default schedule: b0 of the next tile is read in phase 3 (a register copy per tile parity).
  // EARLY (MN-major A, whose transposing fragment reads need more registers): b0 is read in phase 0
  // beside a0 and Bh0 is refilled in phase 1 with Ah0 — one b0 register set, waits recounted:
  //   issue order per tile Bh0 Ah0 | Bh1 | Ah1 (phases 1, 2, 3); vmcnt(10) after phase 0 (Bh1 of this
  //   tile landed), 12 after phase 1 (Ah1), none after 2, 12 after 3 (Ah0 / Bh0 of the next tile).
  auto ktile = [&](auto slot_c, int t, ppbf16x8 (&b0c)[4], ppbf16x8 (&b0n)[4], auto wc_c) {
    constexpr int SLOT = decltype(slot_c)::value;
    const char* cs = smem + SLOT * PP_SLOT;
    const char* ns = smem + (SLOT ^ 1) * PP_SLOT;
    if constexpr (EARLY) {
      rd_a(cs + H_A0 * PP_HALF, fa);
      rd_b(cs + H_B0 * PP_HALF, b0c);
      end_load(VM10{});
      pp_mma<0, 0, VAR>(acc, fa, b0c);
      rs_mma(Q0{}, fa, wc_c);
      end_mma();
      rd_b(cs + H_B1 * PP_HALF, fb1);
      issue(HB0{}, slot_c, t + 2);
      issue(HA0{}, slot_c, t + 2);
      end_load(VM12{});
      pp_mma<0, 1, VAR>(acc, fa, fb1);
      end_mma();
      rd_a(cs + H_A1 * PP_HALF, fa);
      issue(HB1{}, slot_c, t + 2);
      end_load(VMNONE{});
      pp_mma<1, 1, VAR>(acc, fa, fb1);
      rs_mma(Q1{}, fa, wc_c);
      end_mma();
      issue(HA1{}, slot_c, t + 2);
      end_load(VM12{});
      pp_mma<1, 0, VAR>(acc, fa, b0c);
      end_mma();
      (void)ns;
      (void)b0n;
    } else {
      constexpr bool DMA_FIRST = (VAR & 4) != 0;
      // phase 0: a0 x b0 (refill Bh0 <- t+2)
      if constexpr (DMA_FIRST) issue(HB0{}, slot_c, t + 2);
      rd_a(cs + H_A0 * PP_HALF, fa);
      if constexpr (!DMA_FIRST) issue(HB0{}, slot_c, t + 2);
      end_load(VM12{});
      pp_mma<0, 0, VAR>(acc, fa, b0c);
      rs_mma(Q0{}, fa, wc_c);
      end_mma();
      // phase 1: a0 x b1 (refill Ah0)
      if constexpr (DMA_FIRST) issue(HA0{}, slot_c, t + 2);
      rd_b(cs + H_B1 * PP_HALF, fb1);
      if constexpr (!DMA_FIRST) issue(HA0{}, slot_c, t + 2);
      end_load(VM12{});
      pp_mma<0, 1, VAR>(acc, fa, fb1);
      end_mma();
      // phase 2: a1 x b1 (refill Bh1)
      if constexpr (DMA_FIRST) issue(HB1{}, slot_c, t + 2);
      rd_a(cs + H_A1 * PP_HALF, fa);
      if constexpr (!DMA_FIRST) issue(HB1{}, slot_c, t + 2);
      end_load(VM12{});
      pp_mma<1, 1, VAR>(acc, fa, fb1);
      rs_mma(Q1{}, fa, wc_c);
      end_mma();
      // phase 3: a1 x b0, next tile's b0 into registers (refill Ah1)
      if constexpr (DMA_FIRST) issue(HA1{}, slot_c, t + 2);
      rd_b(ns + H_B0 * PP_HALF, b0n);
      if constexpr (!DMA_FIRST) issue(HA1{}, slot_c, t + 2);
      end_load(VM12{});
      pp_mma<1, 0, VAR>(acc, fa, b0c);
      end_mma();
    }
  };
  per_wc([&](auto wc_c) {
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      ktile(S0{}, t, fb0e, fb0o, wc_c);
      ktile(S1{}, t + 1, fb0o, fb0e, wc_c);
    }
    if (t < nk) ktile(S0{}, t, fb0e, fb0o, wc_c);
  });
  if (STAGGER && !lag) pp_sync();
  rs_store();
  // drain the (zero-filling) DMAs of the tiles past the end before the LDS becomes the staging tile
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool reduced = false;
  if constexpr (!AK && !BK) {  // split-K weight gradients: the in-kernel fix-up when the caller gave tickets
    if (p.epi.tickets && p.epi.slab) {
      if (!splitk_fixup(acc, smem, p.epi, m0, n0, p.M, p.N)) return;
      reduced = true;
    }
  }
  wide_tile_epilogue(acc, smem, PP_STATS_OFF, p.epi, m0, n0, p.M, p.N, tm, blockIdx.y, reduced);
}

// ---------------------------------------------------------------- persistent variant
// One workgroup per CU walks tiles L = slot + i*G (G = grid size, slot = the XCD-aware rank of the
// block, so each round of G tiles is the same tile set as one wave of the non-persistent launch).  The
// K-tile stream does not stop at tile boundaries: the refills issued during a tile's last two K tiles
// already fetch the next tile's first two, and its epilogue (the banded, LDS-only-barrier form) runs
// while those are in flight — the prologue / epilogue gap that costs the non-persistent kernel ~15 %
// at K = 1024 (gemm_lab: 32768 x 3072 x 1024 vs x 4096) overlaps the next tile's loads.  Operand
// descriptors span whole matrices here (32-bit offsets: the host checks the operand sizes), so the
// per-tile source state is uniform (m0, n0) and any tile's DMA source costs a few scalar ops.
constexpr int PPP_LDS = PP_LDS_LOOP + 64 * 256 * 2;  // ring + one 64-row staging band
static_assert(PPP_LDS <= 160 * 1024, "LDS budget");

struct PPPArgs {
  PPOp a, b;
  int64_t M, N, K;
  int tiles_m, tiles_n, ntiles, nk;
  uint32_t nk_mul, nk_shr;  // u / nk
  Epi epi;
};

template <bool AK, bool BK, bool RS>
__global__ void __launch_bounds__(PP_NT, 1) gemm_pp_persist_kernel(PPPArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const bool lag = wr == 1;  // ping-pong stagger (variant 2 of the non-persistent kernel)
  constexpr bool EARLY = !AK;
  // inline-asm DMA for every layout: the unit's LDS slot is a runtime value here, so beside a visible
  // LDS-DMA hipcc drains vmcnt(0) before every fragment read it cannot prove disjoint from the DMA
  constexpr bool ASM_DMA = true;
  const int G = gridDim.x;
  const int slot_id = xcd_remap(blockIdx.x, G);
  const int my_tiles = slot_id < p.ntiles ? (p.ntiles - slot_id + G - 1) / G : 0;
  const int nk = p.nk;
  const int64_t K = p.K;

  // whole-matrix descriptors and the lane's fixed offsets
  const int64_t a_bytes = AK ? p.M * p.a.ld * 2 : ((K - 1) * p.a.ld + p.M) * 2;
  const int64_t b_bytes = BK ? p.N * p.b.ld * 2 : ((K - 1) * p.b.ld + p.N) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a.p, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.b.p, (short)0, (int)b_bytes, 0x00020000);
  const pp_i32x4 ras = pp_rsrc_words(p.a.p, a_bytes), rbs = pp_rsrc_words(p.b.p, b_bytes);
  // K-major: lane row rr (image row round*64 + wid*8 + lane/8) and logical chunk; MN-major: k-row and column
  const int kchunk = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
  const int a_rr = AK ? wid * 8 + (lane >> 3) : ((pp_mn_col(tid) >> 6) * 128 + (pp_mn_col(tid) & 63));
  const int b_rr = BK ? (wid >> 2) * 64 + (wid & 3) * 8 + (lane >> 3) : ((pp_mn_col(tid) >> 5) * 64 + (pp_mn_col(tid) & 31));
  const uint32_t a_lane = AK ? (uint32_t)((a_rr * p.a.ld + kchunk * 8) * 2) : (uint32_t)(((tid >> 4) * p.a.ld + a_rr) * 2);
  const uint32_t b_lane = BK ? (uint32_t)((b_rr * p.b.ld + kchunk * 8) * 2) : (uint32_t)(((tid >> 4) * p.b.ld + b_rr) * 2);
  const int klim = (int)K - kchunk * 8;

  auto tile_of = [&](int i, int& m0, int& n0) {
    const int L = slot_id + i * G;
    int tm, tn;
    grouped_tile(L, p.tiles_m, p.tiles_n, 8, tm, tn);
    m0 = tm * 256;
    n0 = tn * 256;
  };

  // the DMA stream's position (the unit being refilled, two ahead of the one computed): tile coordinates
  // of its tile, its K tile and whether the tile exists — uniform values advanced once per unit
  struct Pos {
    int m0, n0, kt, ti;
  };
  auto pos_at = [&](int ti, int kt) {
    Pos q;
    q.ti = ti;
    q.kt = kt;
    q.m0 = q.n0 = 0;
    if (ti < my_tiles) tile_of(ti, q.m0, q.n0);
    q.m0 = __builtin_amdgcn_readfirstlane(q.m0);
    q.n0 = __builtin_amdgcn_readfirstlane(q.n0);
    return q;
  };
  auto advance = [&](Pos& q) {
    if (++q.kt == nk) q = pos_at(q.ti + 1, 0);
  };
  // one half image of the unit at `q` into slot `slot`
  auto issue = [&](auto hid_c, int slot, const Pos& q) {
    constexpr int hid = decltype(hid_c)::value;
    constexpr bool isA = hid < 2;
    constexpr bool km = isA ? AK : BK;
    char* dst = smem + slot * PP_SLOT + hid * PP_HALF + wid * 1024;
    const bool live = q.ti < my_tiles;
    const int kt = q.kt;
    const int r0 = isA ? q.m0 : q.n0;
    const int64_t ld = isA ? p.a.ld : p.b.ld;
    const uint32_t lane_off = isA ? a_lane : b_lane;
    const int rows = (int)(isA ? p.M : p.N);
    const int rr = (isA ? a_rr : b_rr) + (hid & 1) * (isA ? 64 : 32);
    // the tile origin, half and K tile are uniform (soffset); validity explicit per lane as gemm_pp_kernel
    uint32_t su, s1;
    bool ok0, ok1;
    if constexpr (km) {
      su = (uint32_t)(((int64_t)(r0 + (hid & 1) * (isA ? 64 : 32)) * ld + (int64_t)kt * 64) * 2);
      s1 = su + (uint32_t)(128 * ld * 2);
      const bool kv = live && kt * 64 < klim;
      ok0 = kv && r0 + rr < rows;
      ok1 = kv && r0 + rr + 128 < rows;
    } else {
      su = (uint32_t)(((int64_t)kt * 64 * ld + r0 + (hid & 1) * (isA ? 64 : 32)) * 2);
      s1 = su + (uint32_t)(32 * ld * 2);
      const bool cv = live && r0 + rr < rows;
      ok0 = cv && kt * 64 + (tid >> 4) < (int)K;
      ok1 = cv && kt * 64 + (tid >> 4) + 32 < (int)K;
    }
    su = __builtin_amdgcn_readfirstlane(su);
    s1 = __builtin_amdgcn_readfirstlane(s1);
    if constexpr (ASM_DMA) {
      const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)dst);
      pp_glds_asm(isA ? ras : rbs, l, ok0 ? lane_off : PP_OOB, su);
      pp_glds_asm(isA ? ras : rbs, l + 8192, ok1 ? lane_off : PP_OOB, s1);
    } else {
      pp_glds(isA ? ra : rb, dst, ok0 ? lane_off : PP_OOB, su);
      pp_glds(isA ? ra : rb, dst + 8192, ok1 ? lane_off : PP_OOB, s1);
    }
  };
  using HA0 = std::integral_constant<int, H_A0>;
  using HA1 = std::integral_constant<int, H_A1>;
  using HB0 = std::integral_constant<int, H_B0>;
  using HB1 = std::integral_constant<int, H_B1>;

  const int kl0 = pp_klane(lane, 0), kl1 = pp_klane(lane, 32);
  auto rd_a = [&](const char* half, ppbf16x8 (&f)[8]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (AK) f[kk * 4 + i] = pp_kfrag(half, wr * 64 + 16 * i, kk ? kl1 : kl0);
        else f[kk * 4 + i] = pp_mfrag(half, wr * 4 + i, kk * 32, lane);
      }
  };
  auto rd_b = [&](const char* half, ppbf16x8 (&f)[4]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (BK) f[kk * 2 + j] = pp_kfrag(half, wc * 32 + 16 * j, kk ? kl1 : kl0);
        else f[kk * 2 + j] = pp_mfrag(half, wc * 2 + j, kk * 32, lane);
      }
  };
  auto end_load = [&](auto vm_c) {
    constexpr int VM = decltype(vm_c)::value;
    if constexpr (VM == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if constexpr (VM == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_sync();
  };
  using VM10 = std::integral_constant<int, 10>;
  using VM12 = std::integral_constant<int, 12>;
  using VMNONE = std::integral_constant<int, -1>;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rsacc[2] = {0.f, 0.f};
  auto rs_mma = [&](auto qa_c, const ppbf16x8 (&a)[8]) {
    if constexpr (RS) {
      constexpr int QA = decltype(qa_c)::value;
      rsacc[QA] += pp_rs_tile(a, wc);
    } else {
      (void)qa_c;
      (void)a;
    }
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;

  ppbf16x8 fa[8], fb0[4], fb1[4];
  // prologue: units 0 and 1 in the issue order of the loop below (Bh0 Ah0 | Bh1 | Ah1 per unit)
  Pos ip = pos_at(0, 0);
  issue(HB0{}, 0, ip);
  issue(HA0{}, 0, ip);
  issue(HB1{}, 0, ip);
  issue(HA1{}, 0, ip);
  advance(ip);
  issue(HB0{}, 1, ip);
  issue(HA0{}, 1, ip);
  issue(HB1{}, 1, ip);
  issue(HA1{}, 1, ip);
  advance(ip);  // ip: the unit two ahead of the first computed one
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // Bh0(0), Ah0(0) landed
  pp_sync();
  if (lag) pp_sync();

  // One K unit in the EARLY schedule of the per-tile kernel (b0 read beside a0 in phase 0, Bh0 and Ah0
  // refilled in phase 1): a single b0 register set, so the unit loop needs no parity unroll and the
  // tile epilogue has one call site (one copy of its code and register live ranges).
  auto kunit = [&](int slot) {
    const char* cs = smem + slot * PP_SLOT;
    rd_a(cs + H_A0 * PP_HALF, fa);
    rd_b(cs + H_B0 * PP_HALF, fb0);
    end_load(VM10{});
    pp_mma<0, 0, 2>(acc, fa, fb0);
    rs_mma(Q0{}, fa);
    pp_sync();
    rd_b(cs + H_B1 * PP_HALF, fb1);
    issue(HB0{}, slot, ip);
    issue(HA0{}, slot, ip);
    end_load(VM12{});
    pp_mma<0, 1, 2>(acc, fa, fb1);
    pp_sync();
    rd_a(cs + H_A1 * PP_HALF, fa);
    issue(HB1{}, slot, ip);
    end_load(VMNONE{});
    pp_mma<1, 1, 2>(acc, fa, fb1);
    rs_mma(Q1{}, fa);
    pp_sync();
    issue(HA1{}, slot, ip);
    end_load(VM12{});
    pp_mma<1, 0, 2>(acc, fa, fb0);
    pp_sync();
  };

  int u = 0;
  for (int ti = 0; ti < my_tiles; ++ti) {
    for (int kt = 0; kt < nk; ++kt, ++u) {
      kunit(u & 1);
      advance(ip);
    }
    // align the two wave groups, epilogue (the next tile's first two units are in flight), restagger
    int m0, n0;
    tile_of(ti, m0, n0);
    if (!lag) pp_sync();
    if constexpr (RS) {
      if (n0 == 0 && (lane >> 4) == 0) {  // tile column 0 only (see gemm_pp_kernel)
#pragma unroll
        for (int qa = 0; qa < 2; ++qa) {
          const int64_t m = m0 + wr * 128 + qa * 64 + 16 * wc + (lane & 15);
          if (m >= p.M) continue;
          const float v = rsacc[qa];
          if (p.epi.rowsum_mode == 3) unsafeAtomicAdd((float*)p.epi.rowsum + m, v);
          else if (p.epi.rowsum_mode == 2) ((bf16_t*)p.epi.rowsum)[m] = f2bf(v);
          else ((float*)p.epi.rowsum)[m] = v;
        }
      }
      rsacc[0] = rsacc[1] = 0.f;
    }
    wide_tile_epilogue_banded(acc, smem + PP_LDS_LOOP, p.epi, m0, n0, p.M, p.N, m0 / 256);
    // retire the tile's C stores where hipcc can see it (vmcnt(0), once per tile): otherwise its wait
    // for the store data registers merges into the unit loop's header and drains every unit's in-flight
    // DMAs (vmcnt(0) before a fragment read, per unit)
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (lag) pp_sync();
  }
  if (!lag) pp_sync();
  // the refills issued past the last unit (zero-filling) must land before the workgroup exits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool AK, bool BK, bool RS>
hipError_t launch_ppp(const PPPArgs& a, int grid, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp_persist_kernel<AK, BK, RS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, PPP_LDS);
    return true;
  }();
  (void)attr;
  gemm_pp_persist_kernel<AK, BK, RS><<<grid, PP_NT, PPP_LDS, st>>>(a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------
// 4-wave variant (one wave per SIMD): 256 threads, 2 x 2 waves of 128 x 128 (acc[8][8] = 256 registers,
// the accumulator file), so each fragment read feeds 8 MFMAs instead of 4 / 2 — 32 ds_read_b128 per 128
// MFMAs per K tile, 2/3 of the 8-wave tile's LDS traffic per MFMA.  With no partner wave on the SIMD
// the latency hiding is all software: the two 32-deep k halves of a K tile are double-buffered in
// registers (fragments of half kk+1 are read while half kk multiplies), the LDS holds two K-tile
// stages (tile t+2 is DMA'd into t's stage as soon as every wave has read it), and the DMA / fragment
// reads are interleaved with the MFMAs by sched_group_barrier so the matrix pipe never waits on an
// issue burst.  Two barriers per K tile: (B1) stage t fully read -> refill it; (B2) tile t+1 landed.
// Stage = four [128][64] K-major half images: A rows 0-127 / 128-255, B rows 0-127 / 128-255.
constexpr int P4_NT = 256;
constexpr int P4_STAGE = 4 * PP_HALF;
constexpr int P4_LOOP = 2 * P4_STAGE;
constexpr int P4_STATS_OFF = WT_STAGE_BYTES > P4_LOOP ? WT_STAGE_BYTES : P4_LOOP;
constexpr int P4_LDS = P4_STATS_OFF + 4 * 256 * 2 * 4;
static_assert(P4_LDS <= 160 * 1024, "LDS budget");

// DMA source of one operand for the 4-wave tile.  An operand stage is two [128]-row half images (rows
// 0-127 / 128-255 of the tile); each half is 4 DMA rounds of 1 KB per wave.
//   K-major ([128][64] image, gemm_pp's K-major half): round i, wave w, lane l fills image row
//     R = i*32 + w*8 + l/8, physical chunk l & 7 = logical chunk (l & 7) ^ ((R >> 1) & 7).
//   MN-major ([64 k][128] image, gemm_pp's MN-major half): round i fills k-rows i*16 + t/16 (t = thread),
//     the 8 columns pp_mn_col(t) (the swizzle key only sees k bits 0, 1, 3: rounds of 16 keep it).
// Every per-round / per-half / per-K-tile step is uniform (soffset); validity is explicit per lane.
struct P4Src {
  __amdgpu_buffer_rsrc_t r;
  pp_i32x4 rs;
  uint32_t v, ld2;  // per-lane byte offset; row (K-major) or k-row (MN-major) stride in bytes
  int lim, rows;    // K-major: K left from the lane's chunk, rows left from its round-0 row
                    // MN-major: columns left from the lane's first column, k-rows left from its first
};

template <bool KM>
__device__ __forceinline__ P4Src p4_src(const PPOp& op, int64_t r0, int64_t k0, int64_t K, int wid, int lane) {
  P4Src s;
  const int tid = wid * 64 + lane;
  const bf16_t* base;
  int64_t rem;
  if constexpr (KM) {
    const int chunk = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
    const int rr = wid * 8 + (lane >> 3);
    base = op.p + r0 * op.ld + k0;
    rem = (((op.rows - r0) - 1) * op.ld + (K - k0)) * 2;
    s.v = (uint32_t)((rr * op.ld + chunk * 8) * 2);
    s.lim = (int)(K - k0) - chunk * 8;
    const int64_t rl = op.rows - r0 - rr;
    s.rows = rl > 0x7fffffff ? 0x7fffffff : (int)rl;
  } else {
    const int col = pp_mn_col(tid), kr = tid >> 4;
    base = op.p + k0 * op.ld + r0;
    rem = (((K - k0) - 1) * op.ld + (op.rows - r0)) * 2;
    s.v = (uint32_t)((kr * op.ld + col) * 2);
    const int64_t cl = op.rows - r0 - col;
    s.lim = cl > 0x7fffffff ? 0x7fffffff : (int)cl;
    const int64_t kl = (K - k0) - kr;
    s.rows = kl > 0x7fffffff ? 0x7fffffff : (int)kl;
  }
  s.r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(rem < 0x7fffffff ? rem : 0x7fffffff),
                                          0x00020000);
  s.rs = pp_rsrc_words(base, rem);
  s.ld2 = (uint32_t)(op.ld * 2);
  return s;
}

// DMA x (0..7: half x >> 2, round x & 3) of K tile t: uniform soffset and the lane's voffset / validity
template <bool KM>
__device__ __forceinline__ void p4_dma_args(const P4Src& s, int x, int t, int nk, uint32_t& su, uint32_t& vo) {
  const int h = x >> 2, i = x & 3;
  bool ok;
  if constexpr (KM) {
    const int row = h * 128 + i * 32;
    su = (uint32_t)row * s.ld2 + (uint32_t)t * 128u;
    ok = t < nk && t * 64 < s.lim && s.rows > row;
  } else {
    su = (uint32_t)h * 256u + (uint32_t)(i * 16) * s.ld2 + (uint32_t)(t * 64) * s.ld2;
    ok = t < nk && s.lim > h * 128 && t * 64 + i * 16 < s.rows;
  }
  su = __builtin_amdgcn_readfirstlane(su);
  vo = ok ? s.v : PP_OOB;
}

template <bool AK, bool BK>
__global__ void __launch_bounds__(P4_NT) gemm_pp4_kernel(PPArgs p) {
  constexpr bool ASM_DMA = !(AK && BK);  // see pp_glds_asm
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  grouped_tile(tile, ntiles / p.tiles_n, p.tiles_n, 8, tm, tn);
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int ktiles = (int)((p.K + 63) >> 6);
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int nk = min(ktiles, kt0 + p.kt_per_split) - kt0;
  const int64_t k0 = (int64_t)kt0 * 64;

  const P4Src sa = p4_src<AK>(p.a, m0, k0, p.K, wid, lane);
  const P4Src sb = p4_src<BK>(p.b, n0, k0, p.K, wid, lane);

  // DMA x (0..15: A halves / rounds, then B) of K tile t into stage (t & 1); tiles past the split and
  // rows / columns / K past the operands read zero
  auto dma = [&](int x, int t, int stage) {
    const bool isA = x < 8;
    uint32_t su, vo;
    if (isA) p4_dma_args<AK>(sa, x & 7, t, nk, su, vo);
    else p4_dma_args<BK>(sb, x & 7, t, nk, su, vo);
    char* dst = smem + stage * P4_STAGE + ((isA ? 0 : 2) + ((x >> 2) & 1)) * PP_HALF + (x & 3) * 4096 + wid * 1024;
    if constexpr (ASM_DMA) {
      const uint32_t l = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)dst);
      pp_glds_asm(isA ? sa.rs : sb.rs, l, vo, su);
    } else {
      pp_glds(isA ? sa.r : sb.r, dst, vo, su);
    }
  };
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int x = 0; x < 16; ++x) dma(x, t, stage);
  };

  const int kl0 = pp_klane(lane, 0), kl1 = pp_klane(lane, 32);
  // fragment x of a k half in the order the MFMAs (row-major over acc) first use them: a0, b0..b7, a1..a7
  auto frag = [&](auto km_c, const char* half, int g, int kk) {
    if constexpr (decltype(km_c)::value) return pp_kfrag(half, 16 * g, kk ? kl1 : kl0);
    else return pp_mfrag(half, g, kk * 32, lane);
  };
  auto rd1 = [&](const char* stg, int kk, int x, ppbf16x8 (&fa)[8], ppbf16x8 (&fb)[8]) {
    const char* ha = stg + wr * PP_HALF;
    const char* hb = stg + (2 + wc) * PP_HALF;
    if (x == 0) fa[0] = frag(std::integral_constant<bool, AK>{}, ha, 0, kk);
    else if (x <= 8) fb[x - 1] = frag(std::integral_constant<bool, BK>{}, hb, x - 1, kk);
    else fa[x - 8] = frag(std::integral_constant<bool, AK>{}, ha, x - 8, kk);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // The MFMAs are inline asm with the accumulator pinned to the AGPR file ("+a"): with the builtin,
  // hipcc keeps the 256-register accumulator in the mixed class and shuffles it between the files
  // (~200 v_accvgpr moves per K tile) once the fragments and addresses need their VGPRs.  asm MFMAs
  // are invisible to sched_group_barrier, so the interleave is spelled out: each step is one extra
  // instruction (a fragment read or an LDS-DMA) then a group of MFMAs, fenced by sched_barrier.
  auto mfma = [&](int i, int j, const ppbf16x8 (&fa)[8], const ppbf16x8 (&fb)[8]) {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fb[j]), "v"(fa[i]));
  };
  ppbf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  issue(0, 0);
  issue(1, 1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  pp_sync();
#pragma unroll
  for (int x = 0; x < 16; ++x) rd1(smem, 0, x, fa0, fb0);
  auto ktile = [&](auto st_c, int t) {
    constexpr int ST = decltype(st_c)::value;
    const char* cur = smem + ST * P4_STAGE;
    const char* nxt = smem + (ST ^ 1) * P4_STAGE;
    // (1) k half 0 multiplies (64 MFMAs); k half 1's 16 fragments are read one per 4 MFMAs
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      rd1(cur, 1, x, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int y = 0; y < 4; ++y) mfma(x >> 1, (x & 1) * 4 + y, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_sync();  // B1: every wave has read stage t
    // (2) stage t <- tile t+2 (16 DMAs, one per 2 MFMAs) under rows 0-3 of k half 1
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      dma(x, t + 2, ST);
      __builtin_amdgcn_sched_barrier(0);
      mfma(x >> 2, (x & 3) * 2, fa1, fb1);
      mfma(x >> 2, (x & 3) * 2 + 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    pp_sync();  // B2: tile t+1 landed for every wave
    // (3) k half 0 of tile t+1 read (one fragment per 2 MFMAs) under rows 4-7 of k half 1
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      rd1(nxt, 0, x, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      mfma(4 + (x >> 2), (x & 3) * 2, fa1, fb1);
      mfma(4 + (x >> 2), (x & 3) * 2 + 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(std::integral_constant<int, 0>{}, t);
    ktile(std::integral_constant<int, 1>{}, t + 1);
  }
  if (t < nk) ktile(std::integral_constant<int, 0>{}, t);
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA's result -> the epilogue's accumulator reads
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  wide_tile_epilogue<2, false>(acc, smem, P4_STATS_OFF, p.epi, m0, n0, p.M, p.N, tm, blockIdx.y);  // (lab: no BN-bwd sums)
}

template <bool AK, bool BK>
hipError_t launch_pp4(const PPArgs& a, int splits, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp4_kernel<AK, BK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, P4_LDS);
    return true;
  }();
  (void)attr;
  const int tiles = (int)((a.M + 255) / 256) * a.tiles_n;
  gemm_pp4_kernel<AK, BK><<<dim3(tiles, splits), P4_NT, P4_LDS, st>>>(a);
  return hipGetLastError();
}

template <bool AK, bool BK, int VAR, bool RS = false, int GM = 0>
hipError_t launch_pp_v(const PPArgs& a, int splits, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp_kernel<AK, BK, VAR, RS, GM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS);
    return true;
  }();
  (void)attr;
  const int tiles = (int)((a.M + 255) / 256) * a.tiles_n;
  gemm_pp_kernel<AK, BK, VAR, RS, GM><<<dim3(tiles, splits), PP_NT, PP_LDS, st>>>(a);
  return hipGetLastError();
}

template <int VAR>
hipError_t launch_pp_var(bool ak, bool bk, const PPArgs& a, int splits, hipStream_t st) {
  if (a.epi.rowsum) {  // row sums of A: weight-gradient layout only (A = dY^T, MN-major)
    if (ak || bk) return hipErrorInvalidValue;
    return launch_pp_v<false, false, VAR, true>(a, splits, st);
  }
  if (ak && bk) return launch_pp_v<true, true, VAR>(a, splits, st);
  if (ak) return launch_pp_v<true, false, VAR>(a, splits, st);
  if (bk) return launch_pp_v<false, true, VAR>(a, splits, st);
  return launch_pp_v<false, false, VAR>(a, splits, st);
}

}  // namespace

// PDA_PP_PERSIST=0: one workgroup per tile (A/B knob for the persistent walk)
bool pp_persist_mode() {
  static const bool on = [] {
    const char* e = getenv("PDA_PP_PERSIST");  // opt-in: measured slower than the per-tile grid so far
    return e && e[0] == '1';
  }();
  return on;
}

static void pp_magic(uint32_t d, uint32_t& mul, uint32_t& shr);

// Persistent pipelined GEMM (no split-K): hipErrorInvalidValue when the operands do not fit its
// whole-matrix 32-bit offsets (the caller launches the per-tile kernel instead).
hipError_t gemm_pp_persistent(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor,
                              int64_t ldb, int64_t M, int64_t N, int64_t K, const Epi& epi, hipStream_t st) {
  const int64_t lim = ((int64_t)1 << 31) - 4096;
  const int64_t a_bytes = a_kmajor ? (M + 256) * lda * 2 : (K + 64) * lda * 2;
  const int64_t b_bytes = b_kmajor ? (N + 256) * ldb * 2 : (K + 64) * ldb * 2;
  if (a_bytes >= lim || b_bytes >= lim) return hipErrorInvalidValue;
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  PPPArgs a{};
  a.a = {A, lda, M};
  a.b = {B, ldb, N};
  a.M = M;
  a.N = N;
  a.K = K;
  a.tiles_m = (int)((M + 255) / 256);
  a.tiles_n = (int)((N + 255) / 256);
  a.ntiles = a.tiles_m * a.tiles_n;
  a.nk = (int)((K + 63) / 64);
  pp_magic((uint32_t)a.nk, a.nk_mul, a.nk_shr);
  a.epi = epi;
  a.epi.slab = nullptr;
  const int grid = a.ntiles < cus ? a.ntiles : cus;
  if (epi.rowsum) {
    if (a_kmajor || b_kmajor) return hipErrorInvalidValue;
    return launch_ppp<false, false, true>(a, grid, st);
  }
  if (a_kmajor && b_kmajor) return launch_ppp<true, true, false>(a, grid, st);
  if (a_kmajor) return launch_ppp<true, false, false>(a, grid, st);
  if (b_kmajor) return launch_ppp<false, true, false>(a, grid, st);
  return launch_ppp<false, false, false>(a, grid, st);
}

// PDA_PP_RB_SHIFT (tests): cap on the descriptor-rebase period of MN-major operands (2^s K tiles), so
// small GEMMs exercise the rebase that only K spans past 2 GB need
int pp_rb_shift_cap() {
  static const int v = [] {
    const char* e = getenv("PDA_PP_RB_SHIFT");
    const int x = e ? atoi(e) : 30;
    return x < 0 ? 0 : (x > 30 ? 30 : x);
  }();
  return v;
}

// PDA_EPI_NT=1: the pipelined tile writes bf16 C with nontemporal stores (A/B knob)
int pp_epi_nt() {
  static const int v = [] {
    const char* e = getenv("PDA_EPI_NT");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return v;
}

int pp_group_m() {
  static const int v = [] {
    const char* e = getenv("PDA_PP_GROUP");
    const int x = e ? atoi(e) : 8;
    return x < 1 ? 1 : x;
  }();
  return v;
}

// PDA_PP_VAR: the main-loop schedule.  10 (two MFMA phases per K tile + staggered wave groups) over 2 (staggered
// four-phase): +1-3 % on the transformer GEMM shapes, Llama-3-8B FSDP +2.6 %, ResNet-50 +0.3-0.6 %, GPT-2 even
// (profiles/r6_gemm_lab_transformer_fwd.jsonl, r6_pp_var10_ab.jsonl)
int pp_default_variant() {
  static const int v = [] {
    const char* e = getenv("PDA_PP_VAR");
    return e ? atoi(e) : 10;
  }();
  return v;
}

// C = A * B through the pipelined tile (see the header).  Operand conventions as gemm_bf16:
// a_kmajor: A(m,k) = A[m*lda+k] else A[k*lda+m]; b_kmajor: B(k,n) = B[n*ldb+k] else B[k*ldb+n].
// splits > 1: `epi.slab` receives [splits][M][N] fp32 partials (the caller reduces them); the split
// count actually used (K tiles per split rounded) is returned through `*used_splits`.
hipError_t gemm_pp(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                   int64_t M, int64_t N, int64_t K, const Epi& epi, int splits, int variant, hipStream_t st,
                   int* used_splits) {
  if (M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  if ((a_kmajor || b_kmajor) && K % 8) return hipErrorInvalidValue;
  if ((!a_kmajor && M % 8) || N % 8) return hipErrorInvalidValue;
  const int ktiles = (int)((K + 63) / 64);
  if (splits < 1) splits = 1;
  int kps = (ktiles + splits - 1) / splits;
  // an MN-major operand addresses 2^rb_shift K tiles from each descriptor base with 32-bit offsets
  const int64_t ld_mn = std::max(a_kmajor ? (int64_t)0 : lda, b_kmajor ? (int64_t)0 : ldb);
  int rb_shift = pp_rb_shift_cap();
  if (ld_mn > 0) {
    while (rb_shift > 0 && (((int64_t)64 << rb_shift) + 128) * ld_mn * 2 >= ((int64_t)1 << 31)) --rb_shift;
    if ((64 + 128) * ld_mn * 2 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  }
  splits = (ktiles + kps - 1) / kps;  // <= the requested count (the caller sized the slab for that)
  if (splits > 1 && !epi.slab) return hipErrorInvalidValue;
  // a K-major operand's 256-row panel must stay within 32-bit offsets
  if ((a_kmajor && 257 * lda * 2 >= ((int64_t)1 << 31)) || (b_kmajor && 257 * ldb * 2 >= ((int64_t)1 << 31)))
    return hipErrorInvalidValue;
  if (used_splits) *used_splits = splits;
  // (the persistent walk's banded epilogue has no BN-backward statistics path)
  if (splits == 1 && variant < 0 && pp_persist_mode() && !epi.bst_z) {
    const hipError_t r = gemm_pp_persistent(A, a_kmajor, lda, B, b_kmajor, ldb, M, N, K, epi, st);
    if (r != hipErrorInvalidValue) return r;
  }
  PPArgs a{{A, lda, M}, {B, ldb, N}, M, N, K, (int)((N + 255) / 256), kps, epi, {}};
  a.rb_shift = rb_shift;
  a.group_m = pp_group_m();
  a.epi.nt_store = pp_epi_nt();
  if (splits <= 1) a.epi.slab = nullptr;
  const int var = variant < 0 ? pp_default_variant() : variant;
  if (var == 200 && !epi.rowsum && !epi.bst_z && !(epi.tickets && splits > 1)) {  // (no fix-up in pp4)
    if (a_kmajor && b_kmajor) return launch_pp4<true, true>(a, splits, st);
    if (a_kmajor) return launch_pp4<true, false>(a, splits, st);
    if (b_kmajor) return launch_pp4<false, true>(a, splits, st);
    return launch_pp4<false, false>(a, splits, st);
  }
  switch (var) {
    case 0: return launch_pp_var<0>(a_kmajor, b_kmajor, a, splits, st);
    case 1: return launch_pp_var<1>(a_kmajor, b_kmajor, a, splits, st);
    case 3: return launch_pp_var<3>(a_kmajor, b_kmajor, a, splits, st);
    case 6: return launch_pp_var<6>(a_kmajor, b_kmajor, a, splits, st);
    case 10: return launch_pp_var<10>(a_kmajor, b_kmajor, a, splits, st);
    default: return launch_pp_var<2>(a_kmajor, b_kmajor, a, splits, st);
  }
}

static void pp_magic(uint32_t d, uint32_t& mul, uint32_t& shr) {
  if (d <= 1) {
    mul = 0;
    shr = 0;
    return;
  }
  uint32_t l = 0;
  while ((1u << l) < d) ++l;
  const uint32_t pw = 31 + l;
  mul = (uint32_t)(((1ull << pw) + d - 1) / d);
  shr = pw - 32;
}

// Implicit GEMM through the pipelined tile: C[N*P*Q, Cout] = gather(src) W^T (PPGather above) with
// W [Cout][K] K-major.  Returns hipErrorInvalidValue when the shape does not fit the kernel's 32-bit
// offsets (the caller keeps its other paths).
hipError_t gemm_pp_gather(const bf16_t* src, int Nimg, int H, int W, int C, int P, int Q, int S, int K, int st,
                          int o_r, int o_c, int tr, int ts, const bf16_t* w, int Cout, const Epi& epi, hipStream_t stream) {
  const int64_t M = (int64_t)Nimg * P * Q, xn = (int64_t)Nimg * H * W * C;
  if (C % 64 || Cout % 8 || K % 64 || K <= 0 || xn * 2 >= ((int64_t)1 << 31) || M >= ((int64_t)1 << 31) ||
      257 * (int64_t)K * 2 >= ((int64_t)1 << 31) || H >= 16384 || W >= 16384)
    return hipErrorInvalidValue;
  PPArgs a{{src, 0, xn}, {w, K, Cout}, M, Cout, K, (int)((Cout + 255) / 256), (int)((K + 63) / 64), epi, {}};
  a.epi.slab = nullptr;
  a.epi.nt_store = pp_epi_nt();
  PPGather& g = a.ga;
  g.H = H; g.W = W; g.C = C; g.P = P; g.Q = Q; g.S = S; g.st = st; g.o_r = o_r; g.o_c = o_c; g.tr = tr; g.ts = ts;
  pp_magic((uint32_t)C, g.mC, g.sC);
  pp_magic((uint32_t)S, g.mS, g.sS);
  return launch_pp_v<true, true, 2, false, 1>(a, 1, stream);
}

// Convolution weight gradient through the pipelined tile: dw[Cout, R*S*C] = dy[N*P*Q, Cout]^T gather(x)
// (PPWg), both operands MN-major, split-K into `slab` ([splits][Cout][R*S*C] fp32, reduced by the
// caller).  hipErrorInvalidValue when the shape does not fit (the caller keeps its other paths).
hipError_t gemm_pp_wgrad(const bf16_t* dy, const bf16_t* x, int Nimg, int H, int W, int C, int Cout, int R, int S,
                         int P, int Q, int stride, int pad, int dil, const Epi& epi, int splits, hipStream_t stream,
                         int* used_splits) {
  const int64_t K = (int64_t)Nimg * P * Q, Nn = (int64_t)R * S * C, xn = (int64_t)Nimg * H * W * C;
  if (C % 8 || Cout % 8 || xn * 2 >= ((int64_t)1 << 31) || K >= ((int64_t)1 << 31) - 256) return hipErrorInvalidValue;
  const int ktiles = (int)((K + 63) / 64);
  if (splits < 1) splits = 1;
  const int kps = (ktiles + splits - 1) / splits;
  splits = (ktiles + kps - 1) / kps;
  if (splits > 1 && !epi.slab) return hipErrorInvalidValue;
  int rb_shift = 30;
  while (rb_shift > 0 && (((int64_t)64 << rb_shift) + 128) * Cout * 2 >= ((int64_t)1 << 31)) --rb_shift;
  PPArgs a{{dy, Cout, Cout}, {x, 0, xn}, Cout, Nn, K, (int)((Nn + 255) / 256), kps, epi, {}};
  a.rb_shift = rb_shift;
  if (splits <= 1) a.epi.slab = nullptr;
  PPWg& g = a.gb;
  g.H = H; g.W = W; g.C = C; g.P = P; g.Q = Q; g.st = stride; g.pad = pad; g.dil = dil; g.S = S;
  pp_magic((uint32_t)Q, g.mQ, g.sQ);
  pp_magic((uint32_t)P, g.mP, g.sP);
  pp_magic((uint32_t)C, g.mC, g.sC);
  pp_magic((uint32_t)S, g.mS, g.sS);
  if (used_splits) *used_splits = splits;
  return launch_pp_v<false, false, 2, false, 2>(a, splits, stream);
}

// Lab entry (tools/gemm_lab.py): C[M,N] = A B (+ bf16 bias), bf16 output, the given operand majorness.
hipError_t gemm_pp_lab(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                       bf16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, const bf16_t* bias, int variant,
                       hipStream_t st) {
  Epi epi{};
  epi.C = C;
  epi.ldc = ldc;
  epi.bias = bias;
  if (variant == 100 && epi.bst_z) return hipErrorInvalidValue;
  if (variant == 100) return gemm_pp_persistent(A, a_kmajor, lda, B, b_kmajor, ldb, M, N, K, epi, st);
  return gemm_pp(A, a_kmajor, lda, B, b_kmajor, ldb, M, N, K, epi, 1, variant, st, nullptr);
}

}  // namespace pda
