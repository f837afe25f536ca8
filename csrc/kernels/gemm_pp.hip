// Pipelined 256 x 256 bf16 GEMM main loop for gfx950 (VERDICT r3 "what's next" #1).
//
// Why a new loop (profiles/r3_conv_roofline_bs640.md): the 2-stage wide kernel of gemm_conv.hip ends
// every 64-deep K step with `vmcnt(0)` + a workgroup barrier and issues each K step's 64 KB of
// LDS-DMA in one burst in lockstep on all 8 waves, so the matrix pipe idles while both waves of a
// SIMD issue DMAs and while they wait: 53 % MFMA busy at 4096^3.
//
// Structure here (cdna_hip_programming.md §5 "256^2 8-phase template", T2/T3/T4/T5):
//   * 512 threads = 8 waves, 2 (M) x 4 (N); each wave owns a 128 x 64 output (acc[8][4], 16x16x32 MFMA).
//   * The LDS holds two K-tile slots of four 16 KB "half" images each: Ah0 / Ah1 are the rows
//     {0-63, 128-191} / {64-127, 192-255} of the A tile (every wave's first / second 64-row quadrant
//     row), Bh0 / Bh1 the columns {32-wide first / second half of every wave's 64 columns}.
//   * A K tile is 4 phases of 16 MFMAs, quadrants (a0,b0) (a0,b1) (a1,b1) (a1,b0).  Each phase reads
//     one operand quadrant into registers (8 or 4 ds_read_b128), so each half image is released after
//     ONE phase: Bh0 after phase 3 of the previous tile (b0 is kept in registers), Ah0 after phase 0,
//     Bh1 after 1, Ah1 after 2.  The very next phase refills it with K tile t+2 (2 LDS-DMA per thread),
//     so 7 half images (~1.75 K tiles) stay in flight and every wait is the same counted `vmcnt(12)`
//     — never 0 inside the loop.
//   * Ping-pong: waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave issues its
//     fragment reads + DMAs (load section) while its partner runs 16 MFMAs (compute section).
//   * Operands come through buffer descriptors (`buffer_load_dwordx4 ... lds`): one 32-bit offset per
//     lane and operand, rows past M / N and K past the end read as zero (hardware range check).
#include "pda_common.h"
#include "pda_kernels.h"

#include <type_traits>

namespace pda {
namespace {

typedef __bf16 ppbf16x8 __attribute__((ext_vector_type(8)));

constexpr int PP_NT = 512;
constexpr int PP_HALF = 128 * 64 * 2;  // one half image: 128 rows x 64 k, bf16
constexpr int PP_SLOT = 4 * PP_HALF;   // Ah0 Ah1 Bh0 Bh1
constexpr int PP_LDS_LOOP = 2 * PP_SLOT;
constexpr int PP_SROW = 256 + 8;  // epilogue staging row (bf16 elements)
constexpr int PP_LDS = PP_LDS_LOOP > 256 * PP_SROW * 2 ? PP_LDS_LOOP : 256 * PP_SROW * 2;
constexpr uint32_t PP_OOB = 0x80000000u;  // an offset past every descriptor's range: reads zero

enum { H_A0 = 0, H_A1 = 1, H_B0 = 2, H_B1 = 3 };

// K-major [128][64] half image: 128-B rows, 16-B chunk XOR ((row >> 1) & 7) (conflict-free for the
// 16-row x 4-chunk pattern of a 16x16x32 fragment read, see gemm_conv.hip kmaj_off)
__device__ __forceinline__ int pp_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// Fragment of the 16 rows starting at row0 (a multiple of 16) for k-substep kk: lane l holds
// (row0 + (l & 15), kk + 8 (l >> 4) + j).  For such rows the XOR key ((row >> 1) & 7) = (l >> 1) & 7
// does not depend on row0, so the lane part of the address is one of two per-lane offsets (kk = 0 / 32)
// and row0 / the half base fold into the instruction's immediate offset.
__device__ __forceinline__ int pp_lane_off(int lane, int kk) {
  const int key = (lane >> 1) & 7, chunk = (kk >> 3) + (lane >> 4);
  return (lane & 15) * 128 + ((chunk ^ key) << 4);
}
__device__ __forceinline__ ppbf16x8 pp_frag(const char* half, int row0, int loff) {
  return *reinterpret_cast<const ppbf16x8*>(half + row0 * 128 + loff);
}

__device__ __forceinline__ void pp_glds(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
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

struct PPArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  const bf16_t* bias;
  int64_t lda, ldb, ldc;
  int M, N, K, tiles_n;
};

// VAR bits: 1 = s_setprio(1) around each MFMA section, 2 = ping-pong stagger of the two wave groups
template <int VAR>
__global__ void __launch_bounds__(PP_NT, 1) gemm_pp_kernel(PPArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  constexpr bool STAGGER = (VAR & 2) != 0;
  const bool lag = STAGGER && wr == 1;

  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  grouped_tile(tile, ntiles / p.tiles_n, p.tiles_n, 8, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int K = p.K;
  const int nk = (K + 63) >> 6;

  // descriptors over this tile's row panels; num_records = bytes from the panel start to the end of
  // the operand, so rows >= M (N) fall outside the range and read as zero
  const int64_t a_rem = ((int64_t)(p.M - m0) - 1) * p.lda * 2 + (int64_t)K * 2;
  const int64_t b_rem = ((int64_t)(p.N - n0) - 1) * p.ldb * 2 + (int64_t)K * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.A + (int64_t)m0 * p.lda), (short)0, (int)(a_rem < 0x7fffffff ? a_rem : 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.B + (int64_t)n0 * p.ldb), (short)0, (int)(b_rem < 0x7fffffff ? b_rem : 0x7fffffff), 0x00020000);

  // this lane's source (row, chunk) for LDS-DMA round 0 of half 0: image row R = i*64 + wid*8 + lane/8
  // holds logical chunk (lane & 7) ^ ((R >> 1) & 7) at slot lane & 7
  const int chunk = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
  const int kc = chunk * 8;
  const int klim = K - kc;  // K tile t is in range for this lane's chunk iff t * 64 < klim
  // A image row R of half h -> tile row (R >> 6) * 128 + h * 64 + (R & 63)
  const uint32_t a_v = (uint32_t)(((int64_t)(wid * 8 + (lane >> 3)) * p.lda + kc) * 2);
  const uint32_t a_h = (uint32_t)(64 * p.lda * 2), a_i = (uint32_t)(128 * p.lda * 2);
  // B image row R of half h -> tile column (R >> 5) * 64 + h * 32 + (R & 31)
  const uint32_t b_v = (uint32_t)(((int64_t)((wid >> 2) * 64 + (wid & 3) * 8 + (lane >> 3)) * p.ldb + kc) * 2);
  const uint32_t b_h = (uint32_t)(32 * p.ldb * 2), b_i = (uint32_t)(128 * p.ldb * 2);

  auto issue = [&](auto hid_c, int t) {
    constexpr int hid = decltype(hid_c)::value;
    char* dst = smem + (t & 1) * PP_SLOT + hid * PP_HALF + wid * 1024;
    const bool kv = t * 64 < klim;
    const uint32_t kb = (uint32_t)t * 128u;
    if constexpr (hid < 2) {
      const uint32_t o = a_v + (hid & 1) * a_h + kb;
      pp_glds(ra, dst, kv ? o : PP_OOB);
      pp_glds(ra, dst + 8192, kv ? o + a_i : PP_OOB);
    } else {
      const uint32_t o = b_v + (hid & 1) * b_h + kb;
      pp_glds(rb, dst, kv ? o : PP_OOB);
      pp_glds(rb, dst + 8192, kv ? o + b_i : PP_OOB);
    }
  };
  using HA0 = std::integral_constant<int, H_A0>;
  using HA1 = std::integral_constant<int, H_A1>;
  using HB0 = std::integral_constant<int, H_B0>;
  using HB1 = std::integral_constant<int, H_B1>;

  const int loff0 = pp_lane_off(lane, 0), loff1 = pp_lane_off(lane, 32);
  auto rd_a = [&](const char* half, ppbf16x8 (&f)[8]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) f[kk * 4 + i] = pp_frag(half, wr * 64 + 16 * i, kk ? loff1 : loff0);
  };
  auto rd_b = [&](const char* half, ppbf16x8 (&f)[4]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) f[kk * 2 + j] = pp_frag(half, wc * 32 + 16 * j, kk ? loff1 : loff0);
  };
  // end of a load section: own DMAs of the half read next are done, own fragment reads are done
  auto end_load = [&]() {
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_sync();
  };
  auto end_mma = [&]() {
    if constexpr (STAGGER) pp_sync();
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  ppbf16x8 fa[8], fb1[4], fb0e[4], fb0o[4];
  // prologue: K tiles 0 and 1 in the steady-state issue order (Bh0, Ah0, Bh1, Ah1)
  issue(HB0{}, 0);
  issue(HA0{}, 0);
  issue(HB1{}, 0);
  issue(HA1{}, 0);
  issue(HB0{}, 1);
  issue(HA0{}, 1);
  issue(HB1{}, 1);
  issue(HA1{}, 1);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // Bh0(0), Ah0(0) landed
  pp_sync();
  rd_b(smem + H_B0 * PP_HALF, fb0e);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pp_sync();
  if (lag) pp_sync();

  auto ktile = [&](int t, ppbf16x8 (&b0c)[4], ppbf16x8 (&b0n)[4]) {
    const char* cs = smem + (t & 1) * PP_SLOT;
    const char* ns = smem + ((t + 1) & 1) * PP_SLOT;
    // phase 0: a0 x b0
    rd_a(cs + H_A0 * PP_HALF, fa);
    issue(HB0{}, t + 2);
    end_load();
    pp_mma<0, 0, VAR>(acc, fa, b0c);
    end_mma();
    // phase 1: a0 x b1
    rd_b(cs + H_B1 * PP_HALF, fb1);
    issue(HA0{}, t + 2);
    end_load();
    pp_mma<0, 1, VAR>(acc, fa, fb1);
    end_mma();
    // phase 2: a1 x b1
    rd_a(cs + H_A1 * PP_HALF, fa);
    issue(HB1{}, t + 2);
    end_load();
    pp_mma<1, 1, VAR>(acc, fa, fb1);
    end_mma();
    // phase 3: a1 x b0, next tile's b0 read
    rd_b(ns + H_B0 * PP_HALF, b0n);
    issue(HA1{}, t + 2);
    end_load();
    pp_mma<1, 0, VAR>(acc, fa, b0c);
    end_mma();
  };
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, fb0e, fb0o);
    ktile(t + 1, fb0o, fb0e);
  }
  if (t < nk) ktile(t, fb0e, fb0o);
  if (STAGGER && !lag) pp_sync();
  // drain the (zero-filling) DMAs of the tiles past the end before the LDS becomes the staging tile
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: bias in registers, bf16 rows staged through LDS, 16-B coalesced row stores
  bf16_t* stg = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = wr * 128 + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cc = wc * 64 + 16 * j + 4 * (lane >> 4);
      f32x4 v = acc[i][j];
      if (p.bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (n0 + cc + q < p.N) v[q] += bf2f(p.bias[n0 + cc + q]);
      }
      u16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
      *reinterpret_cast<u16x4*>(stg + r * PP_SROW + cc) = o;
    }
  }
  __syncthreads();
  for (int c = tid; c < 256 * 32; c += PP_NT) {
    const int r = c >> 5, ch = c & 31;
    const int m = m0 + r, n = n0 + ch * 8;
    if (m >= p.M || n >= p.N) continue;
    *reinterpret_cast<u16x8*>(p.C + (int64_t)m * p.ldc + n) = *reinterpret_cast<const u16x8*>(stg + r * PP_SROW + ch * 8);
  }
}

template <int VAR>
hipError_t launch_pp(const PPArgs& a, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp_kernel<VAR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS);
    return true;
  }();
  (void)attr;
  const int tiles = ((a.M + 255) / 256) * a.tiles_n;
  gemm_pp_kernel<VAR><<<tiles, PP_NT, PP_LDS, st>>>(a);
  return hipGetLastError();
}

}  // namespace

// Lab entry (tools/gemm_lab.py): C[M,N] = A[M,K] B[N,K]^T (+ bias), bf16, both operands K-major.
hipError_t gemm_pp_lab(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int64_t M,
                       int64_t N, int64_t K, const bf16_t* bias, int variant, hipStream_t st) {
  if (K % 8 || N % 8 || M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  PPArgs a{A, B, C, bias, lda, ldb, ldc, (int)M, (int)N, (int)K, (int)((N + 255) / 256)};
  switch (variant) {
    case 0: return launch_pp<0>(a, st);
    case 1: return launch_pp<1>(a, st);
    case 2: return launch_pp<2>(a, st);
    case 3: return launch_pp<3>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pda
