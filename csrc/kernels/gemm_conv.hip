// MFMA GEMM + implicit-GEMM convolution for gfx950.
//
// One tiled kernel template serves every matmul-shaped op of the framework:
//   Linear fwd / dgrad / wgrad            (plain operands, any of the 4 major-ness combinations)
//   Conv2d fwd    C[npq, co]   = im2col(x)[npq, rsc]   * W[co, rsc]^T          (NHWC, weights OHWI)
//   Conv2d dgrad  C[nhw, ci]   = col(dy)[nhw, rs co]   * Wt[ci, rs co]^T       (stride folded into the gather)
//   Conv2d wgrad  C[co, rsc]   = dy[npq, co]^T         * im2col(x)[npq, rsc]   (split-K over N*P*Q)
// The reference reaches these through cuBLAS / cuDNN (`nn.Linear` `PY1:77`, torchvision ResNet-50
// convs `NB03:314,325-349`); here they are one CDNA4 kernel family.
//
// Design (cdna_hip_programming.md §3, §5, §5.5):
//   * v_mfma_f32_16x16x32_bf16, 256 threads = 4 waves in a 2x2 grid, block tile BM x BN x 64.
//   * Operands are staged global -> VGPR -> LDS (register staging: conv gathers need per-lane
//     predication / zero fill), double-buffered, loads for tile k+1 issued before the MFMAs of
//     tile k and written to LDS after them (T14), one barrier per K tile.
//   * K-major tiles ([rows][64], 128-B rows) are read with ds_read_b128 and XOR-swizzled on the
//     16-B chunk index by (row & 7) -> conflict-free for the MFMA fragment pattern (T2).
//   * MN-major tiles ([64][rows]) are read with ds_read_b64_tr_b16 (T10), so transposed operands
//     (dgrad / wgrad of Linear, dy and im2col(x) in conv wgrad) need no transpose pass; their
//     32-B slots are XOR-swizzled by k so the 8 rows a half-wave touches hit distinct banks.
//   * MFMA roles are swapped (A-operand = N tile) so each lane ends with 4 consecutive output
//     columns (channels): 8-B bf16 / 16-B fp32 stores and per-channel epilogues.
//   * Workgroup ids are remapped XCD-aware so tiles that share an A panel share an L2 (T1).
//   * Index math uses precomputed multiply-shift division (no integer divides in the K loop).
#include "pda_common.h"
#include "pda_kernels.h"
#include "gemm_epi.h"

#include <cmath>

#include <cstdlib>
#include <mutex>
#include <type_traits>

namespace pda {
namespace {

constexpr int NT = 256;
constexpr int BK = 64;

typedef __bf16 mfma_bf16x8 __attribute__((ext_vector_type(8)));

// ------------------------------------------------------------------ fast division (n < 2^31)
struct FastDiv {
  uint32_t d, mul, shr;
};
FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d <= 1) {
    f.mul = 0;
    f.shr = 0;
  } else {
    uint32_t l = 0;
    while ((1u << l) < d) ++l;  // ceil(log2 d)
    const uint32_t p = 31 + l;
    f.mul = (uint32_t)(((1ull << p) + d - 1) / d);
    f.shr = p - 32;
  }
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.mul) >> f.shr);
}

// ------------------------------------------------------------------ operand loaders
// Operands go global -> LDS directly with `global_load_lds_dwordx4` (no VGPR staging, no ds_write):
// the LDS destination of one wave instruction is a wave-uniform base + lane x 16 B, so the swizzled
// LDS images below are produced by choosing, per lane, WHICH global 16-B chunk it fetches.  Round i
// of thread t always lands at tile byte i*4096 + t*16.  Invalid (padding / out-of-range) lanes fetch
// from a zero page, which makes the gathers of the implicit-GEMM convolutions branch-free.
//   K-major tile [R][64]:  thread t fills row (t >> 3) + 32 i, logical k-chunk (t & 7) ^ ((t >> 4) & 7)
//   MN-major tile [64][R]: thread t fills k-row t / (R/8) + KSTEP i, column mn_col<R>(t)
// Loaders return R/32 source pointers per thread per K tile.

__device__ __attribute__((aligned(64))) bf16_t g_zero_page[32];

__device__ __forceinline__ int kmaj_chunk(int tid) { return (tid & 7) ^ ((tid >> 4) & 7); }

template <int R>
__device__ __forceinline__ int mn_swz(int k) {
  if constexpr (R == 128) return (k & 3) | (((k >> 3) & 1) << 2);
  else return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
}
template <int R>
__device__ __forceinline__ int mn_col(int tid) {
  const int p = tid % (R / 8), k = tid / (R / 8);
  return ((((p >> 1) ^ mn_swz<R>(k)) & (R / 16 - 1)) << 4) + (p & 1) * 8;
}

template <int R>
struct PlainK {  // element (row, k) = p[row * ld + k]
  static constexpr bool kMajor = true;
  static constexpr int NCH = R / 32;
  const bf16_t* p;
  int64_t rows, K, ld;
  struct State {
    const bf16_t* ptr[NCH];
    bool ok[NCH];
    int kc;
  };
  __device__ void init(State& s, int64_t row0, int tid) const {
    s.kc = kmaj_chunk(tid) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t row = row0 + (tid >> 3) + 32 * i;
      s.ok[i] = row < rows;
      s.ptr[i] = p + (s.ok[i] ? row : 0) * ld + s.kc;
    }
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
    const bool kok = k0 + s.kc < K;
#pragma unroll
    for (int i = 0; i < NCH; ++i) q[i] = (s.ok[i] && kok) ? s.ptr[i] + k0 : g_zero_page;
  }
};

template <int R>
struct PlainMN {  // element (k, col) = p[k * ld + col]
  static constexpr bool kMajor = false;
  static constexpr int NCH = R / 32;
  static constexpr int KSTEP = NT / (R / 8);
  const bf16_t* p;
  int64_t K, cols, ld;
  struct State {
    const bf16_t* base;
    bool ok;
    int krow;
  };
  __device__ void init(State& s, int64_t col0, int tid) const {
    const int64_t col = col0 + mn_col<R>(tid);
    s.ok = col < cols;
    s.base = p + (s.ok ? col : 0);
    s.krow = tid / (R / 8);
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t k = k0 + s.krow + KSTEP * i;
      q[i] = (s.ok && k < K) ? s.base + k * ld : g_zero_page;
    }
  }
};

struct ConvGeom {
  int H, W, C;     // input (fwd/wgrad) or dx (dgrad) spatial dims and its channel count
  int P, Q;        // output spatial dims
  int R, S, st, pad, dil;
  int Cg;          // channel count of the gathered tensor (C for fwd/wgrad, Cout for dgrad)
  FastDiv fC, fS, fQ, fP, fW, fH;
};

// Conv fwd A operand: element (m = (n,p,q), k = (r,s,ci)) = x[n, p*st-pad+r*dil, q*st-pad+s*dil, ci]
template <int R>
struct ConvFwdK {
  static constexpr bool kMajor = true;
  static constexpr int NCH = R / 32;
  const bf16_t* x;
  ConvGeom g;
  int64_t M, K;
  struct State {
    int nH[NCH], ih0[NCH], iw0[NCH];
    bool ok[NCH];
    int kc;
  };
  __device__ void init(State& s, int64_t row0, int tid) const {
    s.kc = kmaj_chunk(tid) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t m = row0 + (tid >> 3) + 32 * i;
      s.ok[i] = m < M;
      const uint32_t mm = s.ok[i] ? (uint32_t)m : 0u;
      const uint32_t t = fdiv(mm, g.fQ);
      const int q = (int)(mm - t * g.Q);
      const uint32_t n = fdiv(t, g.fP);
      const int p = (int)(t - n * g.P);
      s.nH[i] = (int)n * g.H;
      s.ih0[i] = p * g.st - g.pad;
      s.iw0[i] = q * g.st - g.pad;
    }
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
    const int64_t k = k0 + s.kc;
    const bool kok = k < K;
    const uint32_t kk = kok ? (uint32_t)k : 0u;
    const uint32_t rs = fdiv(kk, g.fC);
    const int ci = (int)(kk - rs * g.C);
    const uint32_t r = fdiv(rs, g.fS);
    const int sidx = (int)(rs - r * g.S);
    const int dr = (int)r * g.dil, ds = sidx * g.dil;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ih = s.ih0[i] + dr, iw = s.iw0[i] + ds;
      const bool ok = kok && s.ok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const int64_t off = ((int64_t)(s.nH[i] + ih) * g.W + iw) * g.C + ci;
      q[i] = ok ? x + off : g_zero_page;
    }
  }
};

// Conv fwd A operand when C % 64 == 0: a 64-deep K tile then lies inside ONE tap (r, s), so the tap
// and the channel base are wave-uniform (scalar ALU) and each row keeps a pointer to its tap-(0, 0)
// pixel: per K tile a row costs one 64-bit add of a uniform offset and two bounds compares, instead of
// ConvFwdK's two fast divisions per 16-B chunk and a 64-bit multiply-add per row.
template <int R>
struct ConvFwdKU {
  static constexpr bool kMajor = true;
  static constexpr int NCH = R / 32;
  const bf16_t* x;
  ConvGeom g;
  int64_t M, K;
  struct State {
    const bf16_t* base[NCH];  // x + pixel (n, p*st - pad, q*st - pad) * C + this thread's chunk
    int ih0[NCH], iw0[NCH];   // (row invalid: ih0 = -2^20, never in range)
    int kc;
  };
  __device__ void init(State& s, int64_t row0, int tid) const {
    s.kc = kmaj_chunk(tid) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t m = row0 + (tid >> 3) + 32 * i;
      const bool ok = m < M;
      const uint32_t mm = ok ? (uint32_t)m : 0u;
      const uint32_t t = fdiv(mm, g.fQ);
      const int q = (int)(mm - t * g.Q);
      const uint32_t n = fdiv(t, g.fP);
      const int p = (int)(t - n * g.P);
      s.ih0[i] = ok ? p * g.st - g.pad : -(1 << 20);
      s.iw0[i] = q * g.st - g.pad;
      s.base[i] = x + (((int64_t)n * g.H + s.ih0[i]) * g.W + s.iw0[i]) * g.C + s.kc;
    }
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
    const bool kok = k0 < K;  // K is a multiple of 64 here
    const uint32_t kk = kok ? (uint32_t)k0 : 0u;
    const uint32_t rs = fdiv(kk, g.fC);
    const int cb = (int)(kk - rs * g.C);
    const uint32_t r = fdiv(rs, g.fS);
    const int sx = (int)(rs - r * g.S);
    const int dr = (int)r * g.dil, ds = sx * g.dil;
    const int64_t toff = ((int64_t)dr * g.W + ds) * g.C + cb;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ih = s.ih0[i] + dr, iw = s.iw0[i] + ds;
      const bool ok = kok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const bf16_t* a = s.base[i] + toff;  // formed unconditionally, then selected
      q[i] = ok ? a : g_zero_page;
    }
  }
};

// Conv dgrad A operand, folded form (stride > 1 with dilation > 1 only): element (m = (n,h,w),
// k = (r,s,co)) = dy[n, p, q, co] where p*st - pad + r*dil = h (zero when not integral / out of range).
template <int R>
struct ConvDgradK {
  static constexpr bool kMajor = true;
  static constexpr int NCH = R / 32;
  const bf16_t* dy;
  ConvGeom g;
  int64_t M, K;
  struct State {
    int nP[NCH], h[NCH], w[NCH];
    bool ok[NCH];
    int kc;
  };
  __device__ void init(State& s, int64_t row0, int tid) const {
    s.kc = kmaj_chunk(tid) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t m = row0 + (tid >> 3) + 32 * i;
      s.ok[i] = m < M;
      const uint32_t mm = s.ok[i] ? (uint32_t)m : 0u;
      const uint32_t t = fdiv(mm, g.fW);
      s.w[i] = (int)(mm - t * g.W);
      const uint32_t n = fdiv(t, g.fH);
      s.h[i] = (int)(t - n * g.H);
      s.nP[i] = (int)n * g.P;
    }
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
    const int64_t k = k0 + s.kc;
    const bool kok = k < K;
    const uint32_t kk = kok ? (uint32_t)k : 0u;
    const uint32_t rs = fdiv(kk, g.fC);  // fC divides by Cg here
    const int co = (int)(kk - rs * g.Cg);
    const uint32_t r = fdiv(rs, g.fS);
    const int sidx = (int)(rs - r * g.S);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ph = s.h[i] + g.pad - (int)r * g.dil;
      const int pw = s.w[i] + g.pad - sidx * g.dil;
      const int p = ph / g.st, qq = pw / g.st;
      const bool ok = kok && s.ok[i] && ph >= 0 && pw >= 0 && p * g.st == ph && qq * g.st == pw && p < g.P &&
                      qq < g.Q;
      const int64_t off = ((int64_t)(s.nP[i] + p) * g.Q + qq) * g.Cg + co;
      q[i] = ok ? dy + off : g_zero_page;
    }
  }
};

// Conv dgrad A operand, stride-decomposed (dil == 1 or stride == 1): the rows of one launch are the
// dx pixels of ONE output phase (h = hh*st + ph, w = ww*st + pw), and K runs over only the taps that
// reach that phase (r = r0 + ri*st) — no zero taps are gathered, unlike the folded form above (a
// stride-2 3x3 dgrad wastes 3/4 of its MFMA work there).  p = hh + base_r - ri*step_r (step_r = dil
// for stride 1, 1 otherwise); likewise q.  dy has dims [N,P,Q,Cg]; k = (ri, si, co).
struct PhaseGeom {
  int Hh, Wh, Sv;
  int base_r, step_r, base_s, step_s;
  FastDiv fWh, fHh, fSv;
};

template <int R>
struct ConvDgradPhaseK {
  static constexpr bool kMajor = true;
  static constexpr int NCH = R / 32;
  const bf16_t* dy;
  ConvGeom g;
  PhaseGeom ph;
  int64_t M, K;
  struct State {
    int nP[NCH], hh[NCH], ww[NCH];
    bool ok[NCH];
    int kc;
  };
  __device__ void init(State& s, int64_t row0, int tid) const {
    s.kc = kmaj_chunk(tid) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t m = row0 + (tid >> 3) + 32 * i;
      s.ok[i] = m < M;
      const uint32_t mm = s.ok[i] ? (uint32_t)m : 0u;
      const uint32_t t = fdiv(mm, ph.fWh);
      s.ww[i] = (int)(mm - t * ph.Wh);
      const uint32_t n = fdiv(t, ph.fHh);
      s.hh[i] = (int)(t - n * ph.Hh);
      s.nP[i] = (int)n * g.P;
    }
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
    const int64_t k = k0 + s.kc;
    const bool kok = k < K;
    const uint32_t kk = kok ? (uint32_t)k : 0u;
    const uint32_t t = fdiv(kk, g.fC);  // fC divides by Cg (= Cout) here
    const int co = (int)(kk - t * g.Cg);
    const uint32_t ri = fdiv(t, ph.fSv);
    const int si = (int)(t - ri * ph.Sv);
    const int dr = ph.base_r - (int)ri * ph.step_r, ds = ph.base_s - si * ph.step_s;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int p = s.hh[i] + dr, qq = s.ww[i] + ds;
      const bool ok = kok && s.ok[i] && (unsigned)p < (unsigned)g.P && (unsigned)qq < (unsigned)g.Q;
      const int64_t off = ((int64_t)(s.nP[i] + p) * g.Q + qq) * g.Cg + co;
      q[i] = ok ? dy + off : g_zero_page;
    }
  }
};

// ConvDgradPhaseK when Cg % 64 == 0: tap-uniform K tiles as in ConvFwdKU (the tap (ri, si) and the
// channel base are wave-uniform; each row keeps a pointer to its tap-(0, 0) source pixel).
template <int R>
struct ConvDgradPhaseKU {
  static constexpr bool kMajor = true;
  static constexpr int NCH = R / 32;
  const bf16_t* dy;
  ConvGeom g;
  PhaseGeom ph;
  int64_t M, K;
  struct State {
    const bf16_t* base[NCH];  // dy + pixel (n, hh, ww) * Cg + this thread's chunk
    int hh[NCH], ww[NCH];     // (row invalid: hh = -2^20)
    int kc;
  };
  __device__ void init(State& s, int64_t row0, int tid) const {
    s.kc = kmaj_chunk(tid) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t m = row0 + (tid >> 3) + 32 * i;
      const bool ok = m < M;
      const uint32_t mm = ok ? (uint32_t)m : 0u;
      const uint32_t t = fdiv(mm, ph.fWh);
      const int ww = (int)(mm - t * ph.Wh);
      const uint32_t n = fdiv(t, ph.fHh);
      const int hh = (int)(t - n * ph.Hh);
      s.hh[i] = ok ? hh : -(1 << 20);
      s.ww[i] = ww;
      s.base[i] = dy + (((int64_t)n * g.P + s.hh[i]) * g.Q + ww) * g.Cg + s.kc;
    }
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
    const bool kok = k0 < K;  // K is a multiple of 64 here
    const uint32_t kk = kok ? (uint32_t)k0 : 0u;
    const uint32_t t = fdiv(kk, g.fC);  // fC divides by Cg (= Cout) here
    const int cb = (int)(kk - t * g.Cg);
    const uint32_t ri = fdiv(t, ph.fSv);
    const int si = (int)(t - ri * ph.Sv);
    const int dr = ph.base_r - (int)ri * ph.step_r, ds = ph.base_s - si * ph.step_s;
    const int64_t toff = ((int64_t)dr * g.Q + ds) * g.Cg + cb;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int p = s.hh[i] + dr, qq = s.ww[i] + ds;
      const bool ok = kok && (unsigned)p < (unsigned)g.P && (unsigned)qq < (unsigned)g.Q;
      const bf16_t* a = s.base[i] + toff;  // formed unconditionally, then selected
      q[i] = ok ? a : g_zero_page;
    }
  }
};

// Conv wgrad B operand (MN-major): element (k = (n,p,q), col = (r,s,ci)) = x[n, p*st-pad+r*dil, ...]
template <int R>
struct ConvWgradMN {
  static constexpr bool kMajor = false;
  static constexpr int NCH = R / 32;
  static constexpr int KSTEP = NT / (R / 8);
  const bf16_t* x;
  ConvGeom g;
  int64_t K, cols;
  struct State {
    int roff, soff, ci;
    bool ok;
    int krow;
  };
  __device__ void init(State& s, int64_t col0, int tid) const {
    const int64_t col = col0 + mn_col<R>(tid);
    s.ok = col < cols;
    const uint32_t cc = s.ok ? (uint32_t)col : 0u;
    const uint32_t rs = fdiv(cc, g.fC);
    s.ci = (int)(cc - rs * g.C);
    const uint32_t r = fdiv(rs, g.fS);
    s.roff = (int)r * g.dil - g.pad;
    s.soff = (int)(rs - r * g.S) * g.dil - g.pad;
    s.krow = tid / (R / 8);
  }
  __device__ void src(const State& s, int64_t k0, const bf16_t* (&q)[NCH]) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int64_t k = k0 + s.krow + KSTEP * i;
      bool ok = s.ok && k < K;
      const uint32_t kk = ok ? (uint32_t)k : 0u;
      const uint32_t t = fdiv(kk, g.fQ);
      const int qq = (int)(kk - t * g.Q);
      const uint32_t n = fdiv(t, g.fP);
      const int p = (int)(t - n * g.P);
      const int ih = p * g.st + s.roff, iw = qq * g.st + s.soff;
      ok = ok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const int64_t off = ((int64_t)((int)n * g.H + ih) * g.W + iw) * g.C + s.ci;
      q[i] = ok ? x + off : g_zero_page;
    }
  }
};

// ------------------------------------------------------------------ LDS images
// K-major [R][64] bf16: 128-B rows, 16-B chunk index XOR ((row >> 1) & 7).  A ds_read_b128 lane group
// reads one chunk of 16 consecutive rows; rows r and r+2 share a bank base (128-B rows = half a bank
// row), so the XOR key must differ across the 8 row PAIRS — (row & 7) repeats after 8 rows and made
// rows r, r+8 collide (measured 16 % bank-conflict cycles, SQ_LDS_BANK_CONFLICT).
__device__ __forceinline__ int kmaj_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// MN-major [64][R] bf16: 32-B slots XOR-swizzled by k (see header).
template <int R>
__device__ __forceinline__ int mn_off(int k, int m) {
  if constexpr (R == 128) {
    const int h = (k & 3) | (((k >> 3) & 1) << 2);
    return k * 256 + ((((m >> 4) ^ h) & 7) << 5) + ((m & 15) << 1);
  } else {
    const int h = ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
    return k * 128 + ((((m >> 4) ^ h) & 3) << 5) + ((m & 15) << 1);
  }
}

// One K tile of an operand: NCH global_load_lds_dwordx4 per thread (see "operand loaders").
template <class L>
__device__ __forceinline__ void glds_tile(const L& ld, const typename L::State& st, int64_t k0, char* tile, int wid) {
  const bf16_t* q[L::NCH];
  ld.src(st, k0, q);
#pragma unroll
  for (int i = 0; i < L::NCH; ++i)
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)q[i],
                                     (void __attribute__((address_space(3)))*)(tile + i * 4096 + wid * 1024), 16, 0,
                                     0);
}

// Fragment for one 16-row group starting at `row0`, k-substep kk (0 or 32):
// lane l holds (row0 + (l & 15), kk + 8 (l >> 4) + j), j = 0..7.
template <bool KMAJ, int R>
__device__ __forceinline__ mfma_bf16x8 read_frag(const char* tile, int row0, int kk, int lane) {
  if constexpr (KMAJ) {
    const int row = row0 + (lane & 15);
    const int chunk = (kk >> 3) + (lane >> 4);
    return *reinterpret_cast<const mfma_bf16x8*>(tile + kmaj_off(row, chunk));
  } else {
    const int i = lane & 15, g = lane >> 4;
    const int k1 = kk + 8 * g + (i >> 2);
    const int m = row0 + 4 * (i & 3);
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + mn_off<R>(k1, m)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + mn_off<R>(k1 + 4, m)));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return __builtin_bit_cast(mfma_bf16x8, f);
  }
}


// Counted vmcnt waits and a barrier that does not drain outstanding LDS-DMA (multi-stage pipelines:
// `__syncthreads()` would wait for every global_load_lds with vmcnt(0)).  A three-stage variant of
// the 128-tile kernel (two K tiles in flight) measured slower on every ResNet-50 shape it could
// serve at two workgroups per CU (64-row / 64-column tiles): latency is not what bounds them.
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0 || N == 2 || N == 4 || N == 6 || N == 8 || N == 16, "add the literal");
}

// LDS-DMA of one 16-B chunk per lane (wave-uniform LDS base + lane x 16 B) as inline asm, as gemm_pp.hip
// pp_glds_asm: beside a compiler-visible global_load_lds, hipcc (ROCm 7.2) waits vmcnt(0) in front of
// every ds_read_b64_tr_b16 (it cannot tell the read from the DMA's LDS range), which drained the next
// group's DMA before this group's first read.  Hidden in asm, the DMA is ordered by the kernel's own
// s_waitcnt only (no other vector-memory op is in flight in its K loop).
__device__ __forceinline__ void glds_asm(const bf16_t* src, char* lds_wave_base) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(l) : "memory", "m0");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// bf16 epilogue of a 4-wave (2x2) BM x BN tile whose accumulators are acc[i][j][r] =
// C[m0 + wm*WM + 16 i + (lane & 15)][n0 + wn*WN + 16 j + 4 (lane >> 4) + r]; `smem` is the operand LDS
// (>= BM * (BN + 8) * 2 bytes + the statistics scratch), free once every wave has left the K loop.
// RAW: the staging barrier is an LDS-only one (lgkmcnt + s_barrier), so LDS-DMA loads of a later tile
// that are in flight survive the epilogue (a __syncthreads() would wait for them with vmcnt(0)).
// DEFER: the BN sums of this tile are ADDED into the caller's st1 / st2 (this thread's fixed column
// chunk) instead of being flushed — a workgroup walking several tiles flushes once (epi_stats_flush).
// BST: compile the BN-backward sums path (epi.bst_z).  Off, the epilogue's register peak stays below the
// K loop's: the 128x64 tile keeps 114 VGPRs and 3 workgroups per CU (173 and 2 with the path compiled
// in: the 56^2 64-channel convs ran 20-25 % slower, profiles/r5_conv_table_bs640.jsonl).
template <int BM, int BN, bool RAW = false, bool DEFER = false, bool BST = true, int GM = 0, bool LEAN = false>
__device__ __forceinline__ void tile_epilogue_bf16_impl(const f32x4 (&acc)[BM / 32][BN / 32], char* smem,
                                                        const Epi& epi, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                                        int tm, float (&st1)[8], float (&st2)[8]) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  // bf16 output: stage the tile through LDS (row stride BN + 8 elements keeps both the 8-B fragment
  // writes and the 16-B row reads bank-conflict free), then write whole 16-B chunks of rows —
  // coalesced stores (and addend loads) instead of 16 rows x 32 B per wave instruction.  The K loop
  // ended with a barrier, so every wave is done reading the operand tiles.
  constexpr int SROW = BN + 8;
  bf16_t* stg = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * WM + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cc = wn * WN + 16 * j + 4 * (lane >> 4);
      f32x4 v = acc[i][j];
      if (epi.bias) {
        const int64_t n = n0 + cc;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (n + q < N)
            v[q] += epi.bias_f32 ? ((const float*)epi.bias)[n + q] : bf2f(((const bf16_t*)epi.bias)[n + q]);
      }
      if (epi.relu) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
      }
      u16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
      *reinterpret_cast<u16x4*>(stg + r * SROW + cc) = o;
    }
  }
  if constexpr (RAW) raw_barrier();
  else __syncthreads();
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "a thread keeps one column chunk");
  // column chunk of this thread is fixed (NT % CPR == 0): BN statistics accumulate in registers
  const bool want_stats = epi.stats != nullptr;
  EpiStatCols scol;
  epi_stat_cols(epi, want_stats, n0 + (tid % CPR) * 8, N, scol);
  float st3[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) st3[q] = 0.f;
  if (BST && epi.bst_z) {
    auto rd = [&](int r, int ch) { return *reinterpret_cast<const u16x8*>(stg + r * SROW + ch * 8); };
    epi_bst_chunks<BM, CPR, NT, decltype(rd), GM ? GM : (BN == 64 ? 2 : 4), LEAN>(epi, scol, rd, m0, n0, M, N, st1,
                                                                                 st2, st3);
  } else
#pragma unroll
  for (int c = tid; c < BM * CPR; c += NT) {
    const int r = c / CPR, ch = c % CPR;
    const int64_t m = m0 + r, n = n0 + ch * 8;
    if (m >= M || n >= N) continue;
    const int64_t crow = epi_row(epi, m);
    u16x8 v = *reinterpret_cast<const u16x8*>(stg + r * SROW + ch * 8);
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
  if (!DEFER && want_stats) {
    epi_stats_flush_all(epi, st1, st2, st3, reinterpret_cast<float*>(smem + BM * SROW * 2), CPR, NT, tm, n0, N);
  }
}

template <int BM, int BN, bool RAW = false, bool BST = true, int GM = 0, bool LEAN = false>
__device__ __forceinline__ void tile_epilogue_bf16(const f32x4 (&acc)[BM / 32][BN / 32], char* smem, const Epi& epi,
                                                   int64_t m0, int64_t n0, int64_t M, int64_t N, int tm) {
  float st1[8], st2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = 0.f;
  tile_epilogue_bf16_impl<BM, BN, RAW, false, BST, GM, LEAN>(acc, smem, epi, m0, n0, M, N, tm, st1, st2);
}

// ------------------------------------------------------------------ the kernel
template <int BM, int BN, class LA, class LB, bool BST = false>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(LA la, LB lb, int64_t M, int64_t N, int64_t K, int tiles_n,
                                                     int ktiles_per_split, Epi epi) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  grouped_tile(tile, ntiles / tiles_n, tiles_n, 8, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const int ktiles = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.y * ktiles_per_split;
  const int kt1 = min(ktiles, kt0 + ktiles_per_split);

  typename LA::State sa;
  typename LB::State sb;
  la.init(sa, m0, tid);
  lb.init(sb, n0, tid);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma_tile = [&](const char* As, const char* Bs) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      mfma_bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag<LA::kMajor, BM>(As, wm * WM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<LB::kMajor, BN>(Bs, wn * WN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  // Two LDS buffers: the DMA of tile t+1 runs while tile t is multiplied; one vmcnt(0) + barrier per
  // K tile retires it (cdna_hip_programming.md §5 "glds vs register staging").
  if (kt0 < kt1) {
    glds_tile(la, sa, (int64_t)kt0 * BK, smem, wid);
    glds_tile(lb, sb, (int64_t)kt0 * BK, smem + A_BYTES, wid);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
    if (kt + 1 < kt1) {
      char* An = smem + (buf ^ 1) * (A_BYTES + B_BYTES);
      glds_tile(la, sa, (int64_t)(kt + 1) * BK, An, wid);
      glds_tile(lb, sb, (int64_t)(kt + 1) * BK, An + A_BYTES, wid);
    }
    mma_tile(As, Bs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: acc[i][j][r] = C[m0 + wm*WM + 16 i + (lane & 15)][n0 + wn*WN + 16 j + 4 (lane >> 4) + r]
  if (!epi.slab && !epi.c_f32) {
    static_assert(BM * (BN + 8) * 2 + (NT / 64) * BN * 2 * 4 <= 2 * (A_BYTES + B_BYTES),
                  "staging tile + stats scratch must fit the operand LDS");
    tile_epilogue_bf16<BM, BN, false, BST>(acc, smem, epi, m0, n0, M, N, tm);
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int64_t m = m0 + wm * WM + 16 * i + (lane & 15);
    if (m >= M) continue;
    const int64_t crow = epi_row(epi, m);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t n = n0 + wn * WN + 16 * j + 4 * (lane >> 4);
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if (epi.slab) {
        float* dst = epi.slab + (int64_t)blockIdx.y * M * N + m * N + n;
        *reinterpret_cast<f32x4*>(dst) = v;
        continue;
      }
      if (epi.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] += epi.bias_f32 ? ((const float*)epi.bias)[n + r] : bf2f(((const bf16_t*)epi.bias)[n + r]);
      }
      if (epi.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (epi.addend) {
        float a[4];
        epi_addend4(epi, crow, n, a);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += a[r];
      }
      *reinterpret_cast<f32x4*>((float*)epi.C + crow * epi.ldc + n) = v;
    }
  }
}

// ------------------------------------------------------------------ 3x3 / stride-1 halo kernel
// Conv fwd (and stride-1 dgrad, which is the same conv over dy with the 180-degree-rotated transposed
// weights) of a 3x3 / pad-1 / stride-1 conv without the implicit-GEMM im2col gather.  The gather
// fetches every input pixel 9 times through L2 (once per tap); with the 256x256 and 128-row tiles
// already at the L2's per-CU share of bandwidth, that traffic, not the MFMAs, bounds the 3x3 convs
// (~0.5-0.6 PF/s).  Here a workgroup owns 128 consecutive output pixels (flattened n,p,q) x BN
// output channels; per 64-channel chunk of the source it DMAs the BAND of source rows those pixels
// touch — their rows plus one halo row each side, full width, once — into LDS, then runs the 9 taps
// as 9 K-steps whose A fragments are read from the band at the tap's pixel offset (zero outside the
// image), while only the weight tiles stream (double-buffered) per tap.  L2 operand traffic per
// K-step drops from (128 + BN) rows to ~BN rows + band/9.
//   band: source rows v0 .. v1 (flattened n*H + h) of W pixels x 64 channels, 128-B rows, chunk XOR
//   swizzle as kmaj_off (pixel = (v - v0) * W + w); sized by the host: band_px >= rows * W.
// B operand: K-major weights, row = output channel, k = tap * Cg + channel (OHWI for fwd; for dgrad
// the plain transposed wt[ci][r][s][co], read at tap 8 - t: `flip`).
// weight-stage ring depth: 4 x 8 KB for 64-channel tiles, 3 x 16 KB for 128
constexpr __host__ __device__ int halo_stages(int bn) { return bn == 64 ? 4 : 3; }

struct HaloGeom {
  int H, W, Cg;      // source spatial dims (= output dims) and channels
  FastDiv fW, fH;
  int band_px;       // LDS band capacity in pixels (host bound)
  int flip;
};

template <int BN>
__global__ void __launch_bounds__(NT, 2) conv3x3_halo_kernel(const bf16_t* __restrict__ src, HaloGeom hg,
                                                            PlainK<BN> lb, int64_t M, int64_t N, int tiles_n,
                                                            Epi epi) {
  constexpr int BM = 128, WM = 64, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int D = halo_stages(BN);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* band = smem;
  char* bst = smem + hg.band_px * 128;  // D weight stages

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  grouped_tile(tile, ntiles / tiles_n, tiles_n, 8, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int H = hg.H, W = hg.W, Cg = hg.Cg;

  // band rows: from the first pixel's row - 1 to the last pixel's row + 1, clipped to their images
  int v0, v1;
  {
    const uint32_t t0 = fdiv((uint32_t)m0, hg.fW);  // n*H + p of the first pixel
    const uint32_t n0i = fdiv(t0, hg.fH);
    const int p0 = (int)(t0 - n0i * H);
    v0 = (int)t0 - (p0 > 0 ? 1 : 0);
    const int64_t ml = (m0 + BM - 1 < M ? m0 + BM - 1 : M - 1);
    const uint32_t t1 = fdiv((uint32_t)ml, hg.fW);
    const uint32_t n1i = fdiv(t1, hg.fH);
    const int p1 = (int)(t1 - n1i * H);
    v1 = (int)t1 + (p1 < H - 1 ? 1 : 0);
  }
  const int band_n = (v1 - v0 + 1) * W;  // < hg.band_px (host bound): pixel band_px - 1 stays zero
  const int zpx = hg.band_px - 1;

  // per-lane output pixels of the TM fragment rows: band pixel of the centre tap, p, q
  int cpix[TM], pp[TM], qq[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int64_t m = m0 + wm * WM + 16 * i + (lane & 15);
    const bool ok = m < M;
    const uint32_t mm = ok ? (uint32_t)m : 0u;
    const uint32_t t = fdiv(mm, hg.fW);
    qq[i] = (int)(mm - t * W);
    const uint32_t n = fdiv(t, hg.fH);
    pp[i] = ok ? (int)(t - n * H) : -4;  // -4: every tap invalid
    cpix[i] = ((int)t - v0) * W + qq[i];
  }

  typename PlainK<BN>::State sb;
  lb.init(sb, n0, tid);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = Cg / 64;
  const int64_t src_px0 = (int64_t)v0 * W;
  auto load_band = [&](int c) {
    // thread t fills pixel (t >> 3) + 32 k, LDS slot t & 7 with logical chunk slot ^ swizzle(pixel)
    const int slot = tid & 7;
    for (int k = 0; k * 32 < hg.band_px; ++k) {
      const int px = k * 32 + (tid >> 3);
      const int lc = slot ^ ((px >> 1) & 7);
      const bf16_t* q = px < band_n ? src + (src_px0 + px) * Cg + c * 64 + lc * 8 : g_zero_page;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)q,
                                       (void __attribute__((address_space(3)))*)(band + k * 4096 + wid * 1024), 16,
                                       0, 0);
    }
  };
  auto load_b = [&](int c, int t, int stage) {
    const int tb = hg.flip ? 8 - t : t;
    glds_tile(lb, sb, (int64_t)tb * Cg + c * 64, bst + stage * B_BYTES, wid);
  };

  // weights stream through a ring of D stages, D - 1 K-steps ahead (a K-step is short — 128 x BN x 64
  // — so one step of prefetch cannot cover the L2 latency); at the top of step s the loads of steps
  // s .. s + D - 2 are in flight, vmcnt counts them in issue order
  const int S = 9 * nchunks;
  load_band(0);
#pragma unroll
  for (int d = 0; d < D - 1; ++d)
    if (d < S) load_b(d / 9, d % 9, d);
#pragma unroll 1
  for (int st = 0; st < S; ++st) {
    const int c = st / 9, t = st - 9 * c;
    if (t == 0 && c > 0) {
      raw_barrier();  // every wave is done with the previous chunk's band
      load_band(c);
      wait_vm<0>();
    } else if (st + D - 2 < S) {
      wait_vm<(D - 2) * PlainK<BN>::NCH>();
    } else {
      wait_vm<0>();
    }
    raw_barrier();  // everyone's loads for step st landed; everyone is done with step st - 1's stage
    if (st + D - 1 < S) load_b((st + D - 1) / 9, (st + D - 1) % 9, (st + D - 1) % D);
    const int dr = t / 3 - 1, ds = t % 3 - 1;
    const int off = dr * W + ds;
    const char* Bs = bst + (st % D) * B_BYTES;
    // every fragment of the step is read up front (unconditional reads: a tap outside the image reads
    // the band's zero pixel), then the 2 x TM x TN MFMAs
    mfma_bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int chunk = 4 * h + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool ok = (unsigned)(pp[i] + dr) < (unsigned)H && (unsigned)(qq[i] + ds) < (unsigned)W;
        const int px = ok ? cpix[i] + off : zpx;
        af[h][i] = *reinterpret_cast<const mfma_bf16x8*>(band + kmaj_off(px, chunk));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[h][j] = read_frag<true, BN>(Bs, wn * WN + 16 * j, 32 * h, lane);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[h][j], af[h][i], acc[i][j], 0, 0, 0);
  }
  __syncthreads();
  // (every wave has left the K loop: the band and weight stages are free for the staging tile)
  tile_epilogue_bf16<BM, BN>(acc, smem, epi, m0, n0, M, N, tm);
}

// ------------------------------------------------------------------ 3x3 / stride-1, 64 -> 64 channels
// The 56^2 layer of ResNet-50 (forward, and the stride-1 dgrad as the conv of dy with the rotated
// weights).  The implicit GEMM is bound by its 9x im2col re-reads through L2 (0.28 ms vs a 0.09 ms HBM
// roof at bs 640), and the halo kernel's one-tile-per-workgroup at 64 output channels is ~1 us of MFMAs
// behind a ~2 us band load.  This kernel:
//  * tiles = 4 whole image rows (224 pixels, W = 56): a band is the 4 rows + 1 halo row each side;
//  * the band is stored with a 64-pixel row pitch, column -1 and columns >= 56 and out-of-image rows
//    zero-filled by the DMA, so every tap reads a real band pixel (no validity selects) and a tap's row
//    step is +-64 pixels, which keeps the (pixel >> 1) & 7 chunk swizzle unchanged: a lane's 42 fragment
//    addresses (7 pixel groups x 3 column offsets x 2 channel halves) are computed ONCE per kernel (tile
//    rows are aligned, so they are the same for every tile) and every tap is ds_read_b128 at an
//    immediate row offset — the per-tap address math had made the first version VALU-bound (5.9 VALU per
//    MFMA, rocprofv3 pmc);
//  * the 9 x 2 x 2 weight fragments of a wave's 32 output channels live in VGPRs (one wave per SIMD:
//    512 VGPRs), loaded once; the LDS holds only two band stages (2 x 48 KB);
//  * workgroups are persistent over a contiguous run of tiles; the next tile's band is DMA'd (inline
//    asm: hipcc adds no vmcnt(0) before the band reads) while this tile multiplies; the finished stage is
//    the epilogue's staging tile (LDS-only barriers, so the other stage's DMA stays in flight).
constexpr int R64_QW = 56;                        // image width this kernel is built for
constexpr int R64_PITCH = 64;                     // band pixels per row
constexpr int R64_ROWS = 6;                       // 4 tile rows + 2 halo rows
constexpr int R64_BAND = R64_ROWS * R64_PITCH * 128;  // 49,152 B per band stage
constexpr int R64_LDS = 2 * R64_BAND;             // 98,304 B

// BSTM: 0 no BN-backward sums, 1 the generic sums epilogue, 2 lean (z only: no addend / bits / second BN)
template <int BSTM>
__global__ void __launch_bounds__(NT, 1) conv3x3_res64_kernel(const bf16_t* __restrict__ src,
                                                               const bf16_t* __restrict__ wts, int H, int flip,
                                                               int64_t M, int ntiles, Epi epi) {
  constexpr int TMW = 7, BM = 32 * TMW, BN = 64, WM = 16 * TMW, WN = 32;
  constexpr int TM = TMW, TN = WN / 16;
  static_assert(BM == 4 * R64_QW, "a tile is 4 image rows");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1, g = lane >> 4;
  const int per = (ntiles + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t_begin = (int)blockIdx.x * per;
  const int t_end = min(ntiles, t_begin + per);
  if (t_begin >= t_end) return;
  // BN sums (forward statistics, or the lean backward sums) accumulate in registers over the whole run
  // of tiles and are flushed once (table row = workgroup): no per-tile LDS reduction + atomics
  constexpr bool DEFER = BSTM != 1;
  float st1[8], st2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = 0.f;

  // weight fragments: B(k = ci, n = co) of tap t (flip: the rotated tap 8 - t), half h, column group j:
  // lane holds w[co = wn*32 + 16 j + (lane & 15)][tap][ci = 32 h + 8 g .. + 7]
  mfma_bf16x8 wf[9][2][TN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = wn * WN + 16 * j + (lane & 15);
        const int tb = flip ? 8 - t : t;
        wf[t][h][j] = *reinterpret_cast<const mfma_bf16x8*>(wts + (int64_t)co * 576 + tb * 64 + 32 * h + 8 * g);
      }
  // band byte offsets (row 0 of the band, column offset ds = -1, 0, +1) of this lane's 7 pixel groups
  int aoff[TM][3][2];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int loc = wm * WM + 16 * i + (lane & 15);  // pixel within the 4-row tile
    const int lr = loc / R64_QW, q = loc - lr * R64_QW;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int b = lr * R64_PITCH + q + d;  // band column = image column + 1; ds = d - 1
#pragma unroll
      for (int h = 0; h < 2; ++h) aoff[i][d][h] = b * 128 + ((((4 * h + g) ^ ((b >> 1) & 7))) << 4);  // NOLINT
    }
  }
  // band of tile tm: rows p0 - 1 .. p0 + 4 of image n, 64 pixel slots each (slot s = column s - 1)
  auto load_band = [&](int tm, char* band) {
    const int r0 = tm * 4;           // flattened (n * H + p) row of the tile's first row
    const int n = r0 / H, p0 = r0 - n * H;
    const bf16_t* img = src + (int64_t)n * H * R64_QW * 64;
    const int slot = tid & 7;
#pragma unroll
    for (int k = 0; k < R64_ROWS * R64_PITCH / 32; ++k) {
      const int b = k * 32 + (tid >> 3);
      const int r = b >> 6, sc = b & 63;
      const int ph = p0 - 1 + r, qc = sc - 1;
      const int lc = slot ^ ((b >> 1) & 7);
      const bool ok = (unsigned)ph < (unsigned)H && (unsigned)qc < (unsigned)R64_QW;
      const bf16_t* a = img + ((int64_t)ph * R64_QW + qc) * 64 + lc * 8;  // formed unconditionally, selected
      glds_asm(ok ? a : g_zero_page, band + k * 4096 + wid * 1024);
    }
  };

  auto tile = [&](int tm, char* band, char* nband) {
    if (tm + 1 < t_end) load_band(tm + 1, nband);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dr = t / 3, d = t % 3;  // band row offset (dr - 1 + 1) and column variant
      mfma_bf16x8 af[2][TM];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[h][i] = *reinterpret_cast<const mfma_bf16x8*>(band + aoff[i][d][h] + dr * R64_PITCH * 128);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][h][j], af[h][i], acc[i][j], 0, 0, 0);
    }
    raw_barrier();  // every wave is done with this band: it becomes the staging tile
    if constexpr (DEFER) {
      tile_epilogue_bf16_impl<BM, BN, true, true, BSTM != 0, 7, BSTM == 2>(acc, band, epi, (int64_t)tm * BM, 0, M, BN,
                                                                           tm, st1, st2);
    } else {
      tile_epilogue_bf16<BM, BN, true, BSTM != 0, 7, BSTM == 2>(acc, band, epi, (int64_t)tm * BM, 0, M, BN, tm);
    }
    // the next band has landed (and this tile's stores).  The builtin, not asm: hipcc's waitcnt pass sees
    // the counters drained here, so it adds no vmcnt(0) of its own at the top of the next tile — after
    // that tile's band DMA has been issued
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
    raw_barrier();
  };

  char* const b0 = smem;
  char* const b1 = smem + R64_BAND;
  load_band(t_begin, b0);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
#pragma unroll 1
  for (int tm = t_begin, it = 0; tm < t_end; ++tm, ++it) tile(tm, (it & 1) ? b1 : b0, (it & 1) ? b0 : b1);
  if (DEFER && epi.stats) epi_stats_flush(epi, st1, st2, reinterpret_cast<float*>(smem), BN / 8, NT, blockIdx.x, 0, BN);
}

// ------------------------------------------------------------------ 3x3 / stride-1 weight gradient, all taps
// dw[co][r][s][ci] = sum over output pixels of dy[px][co] * x[px + (r-1, s-1)][ci].  The implicit GEMM
// (M = Cout, N = 9 C, K = pixels) gathers im2col(x) per N tile: every x pixel is fetched from L2 once
// per tap and per 128-column tile (~43 FLOP per L2 byte at 64 output channels: L2-bound, 0.3 PF/s
// on the 56^2 layer).  Here one workgroup owns a 64 x 576 output block — 64 output channels x all
// 9 taps of 64 input channels — and walks K in row groups: R_k whole output rows of one image
// (R_k * W <= 64 pixels) per K-step.  Per step it DMAs the dy rows (an MN-major [64 px][64 co] tile)
// and the x BAND they touch (R_k + 2 rows of W + 2 pixels, zero-padded at the image border) into LDS
// once, and the 9 taps are 9 shifted views of the band (~150 FLOP per L2 byte).  Wave w owns input
// channels 16w .. 16w+15 of every tap: acc[co block][tap] (36 tiles).  Split-K over row groups writes
// fp32 slabs that splitk_reduce_kernel sums into dw.
//   band pixel b = row_slot * (W + 2) + col + 1 (row_slot 0 = image row p0 - 1); [b][64 ci] MN-major
//   image with the 32-B slot XOR swizzle of mn_off<64> keyed by b.
struct Wg3Geom {
  int N, H, W, C, Cout;
  int rk;         // output rows per K-step (rk * W <= 64)
  int gpi;        // row groups per image = ceil(H / rk)
  int groups;     // N * gpi
  int gps;        // row groups per split
  int band_px;    // band pixels (multiple of 32) >= (rk + 2) * (W + 2)
  int tiles_ci;   // C / 64
  FastDiv fW2;    // W + 2
};

__device__ __forceinline__ int band_mn_off(int b, int m) {
  const int h = ((b >> 1) & 1) | (((b >> 3) & 1) << 1);
  return b * 128 + ((((m >> 4) ^ h) & 3) << 5) + ((m & 15) << 1);
}

constexpr int WG3_STAGE = 40 * 1024;  // [64 px][64 co] dy tile + a band of <= 256 pixels x 128 B

__global__ void __launch_bounds__(NT, 2) conv3x3_wgrad_kernel(const bf16_t* __restrict__ dy,
                                                              const bf16_t* __restrict__ x, Wg3Geom g,
                                                              float* __restrict__ slab) {
  constexpr int A_BYTES = 64 * BK * 2;  // [64 px][64 co]
  // two stages as separate __shared__ objects, loop unrolled by two (see conv_stem_fwd_kernel: with
  // one dynamic array the compiler drained the next group's DMA before this group's reads)
  __shared__ __attribute__((aligned(16))) char s_st0[WG3_STAGE];
  __shared__ __attribute__((aligned(16))) char s_st1[WG3_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tco = blockIdx.x / g.tiles_ci, tci = blockIdx.x - tco * g.tiles_ci;
  const int co0 = tco * 64, ci0 = tci * 64;
  const int W = g.W, H = g.H, W2 = W + 2;
  const int gb = blockIdx.y * g.gps;
  const int ge = min(g.groups, gb + g.gps);

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane band pixels of the k-rows this lane addresses in the transposed B reads:
  // j = kk + 8 (lane >> 4) + ((lane & 15) >> 2) (+ 4), kk in {0, 32}
  int pixj[2][2];
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
    for (int lh = 0; lh < 2; ++lh) {
      const int j = 32 * h2 + 8 * (lane >> 4) + ((lane & 15) >> 2) + 4 * lh;
      const int rj = j / W, cj = j - rj * W;
      pixj[h2][lh] = j < g.rk * W ? rj * W2 + cj : 0;  // past the group: any finite band pixel (dy = 0)
    }

  auto issue = [&](int grp, char* base) {
    const int n = grp / g.gpi, p0 = (grp - n * g.gpi) * g.rk;
    const int rows = min(g.rk, H - p0);
    // dy rows p0 .. p0 + rows - 1: rows * W consecutive pixels, an MN-major [k = px][m = co] tile
    PlainMN<64> la;
    la.p = dy + ((int64_t)n * H + p0) * W * g.Cout + co0;
    la.K = rows * W;
    la.cols = 64;
    la.ld = g.Cout;
    typename PlainMN<64>::State sa;
    la.init(sa, 0, tid);
    glds_tile(la, sa, 0, base, w);
    // x band: image rows p0 - 1 .. p0 + rk, cols -1 .. W (zero outside the image).  Always 8 DMA rounds
    // (256 pixels, the stage's capacity; pixels past the band are zeros nobody reads) with the
    // addresses selected, not branched around: a runtime-length loop / branch join made the compiler
    // drain the DMA before the next reads
    char* band = base + A_BYTES;
    const int s16 = tid & 7;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int b = k * 32 + (tid >> 3);
      const int rs = (int)fdiv((uint32_t)b, g.fW2), cs = b - rs * W2;
      const int hb = ((b >> 1) & 1) | (((b >> 3) & 1) << 1);
      const int ci = ci0 + 16 * ((s16 >> 1) ^ hb) + 8 * (s16 & 1);
      const int ih = p0 - 1 + rs, iw = cs - 1;
      const bool ok = rs < g.rk + 2 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const bf16_t* a = x + (((int64_t)n * H + ih) * W + iw) * g.C + ci;  // formed unconditionally
      const bf16_t* q = ok ? a : g_zero_page;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)q,
                                       (void __attribute__((address_space(3)))*)(band + k * 4096 + w * 1024), 16,
                                       0, 0);
    }
  };

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const int mcol = 16 * w + 4 * ((lane & 15) & 3);
  auto step = [&](int grp, const char* As, char* next) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // this group landed for every wave; every wave is done with `next`
    issue(min(grp + 1, ge - 1), next);  // unconditional: see conv_stem_fwd_kernel
    const char* band = As + A_BYTES;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      mfma_bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<false, 64>(As, 16 * i, 32 * h2, lane);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int toff = (t / 3) * W2 + (t % 3);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(band + band_mn_off(pixj[h2][0] + toff, mcol)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(band + band_mn_off(pixj[h2][1] + toff, mcol)));
        s16x8 f;
        f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
        f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
        const mfma_bf16x8 bf = __builtin_bit_cast(mfma_bf16x8, f);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af[i], acc[i][t], 0, 0, 0);
      }
    }
  };
  if (gb < ge) {  // (every split has groups: wg3_splits; an empty one would still write its zero slab)
    issue(gb, s_st0);
    for (int grp = gb; grp < ge; grp += 2) {
      step(grp, s_st0, s_st1);
      if (grp + 1 < ge) step(grp + 1, s_st1, s_st0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // fp32 partials: acc[i][t][q] = dw[co0 + 16 i + (lane & 15)][t][ci0 + 16 w + 4 (lane >> 4) + q]
  const int64_t Nn = 9LL * g.C;
  float* out = slab + (int64_t)blockIdx.y * g.Cout * Nn;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + 16 * i + (lane & 15);
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *reinterpret_cast<f32x4*>(out + (int64_t)co * Nn + (int64_t)t * g.C + ci0 + 16 * w + 4 * (lane >> 4)) =
          acc[i][t];
  }
}

// ------------------------------------------------------------------ 3x3 weight gradient v2 (all layers)
// dw[co][r][s][ci] = sum over output pixels of dy[px][co] * x[st*px + (r-1, s-1)][ci], stride 1 or 2, for
// every 3x3 layer of ResNet-50 (56^2 .. 7^2, the three strided ones included).  The round-4 kernels left
// these at 0.22-0.34 of their roofline: the 64 x 576 all-taps kernel above moves one 64-pixel row group
// per barrier with a single DMA stage of cover at two 4-wave workgroups per CU (latency-bound, and
// each x row is fetched 3 times), and the 14^2 / 7^2 / strided layers took the implicit GEMM whose
// im2col gather re-reads every x pixel per tap through L2.
// Here one 8-wave workgroup (one per CU, 144 KB of LDS in two 72 KB stages) owns CO_T output channels x
// 64 input channels x 9 taps and walks K in row groups of ONE image: rk output rows (<= 128 pixels,
// in 32-pixel halves) per step.  A step DMAs the dy rows (MN-major [px][CO_T] images) and the x BAND
// those rows touch — (rk - 1) st + 3 input rows of W + 2 pixels (zero outside the image) — and the 9
// taps are 9 views of the band at pixel offsets r (W + 2) + s from the output pixel's (st rj, st cj):
// x crosses the L2 once per row group instead of once per tap.  Waves: ci block w & 3 (16 channels)
// x (CO_T = 128) the co half w >> 2, or (CO_T = 64, KSPLIT) the pixel-half parity w >> 2 with its own
// slab (two slabs per split): every wave multiplies 4 co blocks x 9 taps against one ci block, so an
// A fragment serves 9 MFMAs and a B (band) fragment 4.  Split-K over row groups; fp32 slabs summed by
// splitk_reduce_kernel.
struct Wg3v2Geom {
  int N, H, W, P, Q, C, Cout, st;
  int rk;        // output rows per K-step (rk * Q <= 128)
  int gpi;       // row groups per image = ceil(P / rk)
  int groups;    // N * gpi
  int gps;       // row groups per split
  int band_rows; // (rk - 1) * st + 3
  int w2l;       // log2 of the band row pitch in pixels (>= W + 2, >= 16)
  int tiles_ci;  // C / 64
  int tiles_co;  // Cout / CO_T
  FastDiv fQ;
};

constexpr int WG3V2_NT = 512;
constexpr int WG3V2_DY = 32 * 1024;    // dy: two [64 px][<= 128 co] MN-major images
constexpr int WG3V2_BAND = 40 * 1024;  // band: <= 320 pixels x 64 channels (128-B rows)
constexpr int WG3V2_STAGE = WG3V2_DY + WG3V2_BAND;

template <int CO_T, int W2L>
__global__ void __launch_bounds__(WG3V2_NT, 1) conv3x3_wg_kernel(const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ x, Wg3v2Geom g,
                                                                 float* __restrict__ slab) {
  constexpr bool KSPLIT = CO_T == 64;   // 8 waves = 4 ci blocks x 2 pixel-half parities
  constexpr int NCB = 4;                // co blocks per wave
  constexpr int IMG = 64 * CO_T * 2;    // one [64 px][CO_T] dy image
  // two stages as separate __shared__ objects, loop unrolled by two (conv_stem_fwd_kernel: with one
  // dynamic array hipcc drains the next group's DMA before this group's reads)
  __shared__ __attribute__((aligned(16))) char s_st0[WG3V2_STAGE];
  __shared__ __attribute__((aligned(16))) char s_st1[WG3V2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = w & 3, wh = w >> 2;
  const int tco = blockIdx.x / g.tiles_ci, tci = blockIdx.x - tco * g.tiles_ci;
  const int co0 = tco * CO_T, ci0 = tci * 64;
  const int cow = KSPLIT ? 0 : wh * 64;  // this wave's first co within the tile
  // band rows are W2P = 2^W2L >= W + 2 pixels (>= 16): the swizzle key (pixel bits 1 and 3) then depends on
  // the column only, so a tap's row step r W2P is a constant LDS offset and only the 3 column shifts need
  // their swizzled addresses computed (the per-tap address arithmetic had made the loop VALU-bound)
  constexpr int W2P = 1 << W2L;
  const int W = g.W, H = g.H, Q = g.Q, st = g.st;
  const int gb = blockIdx.y * g.gps;
  const int ge = min(g.groups, gb + g.gps);

  f32x4 acc[NCB][9];
#pragma unroll
  for (int i = 0; i < NCB; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane band pixel (tap (0,0)) of k row j of the transposed B reads, j = 32 h + 8 (lane >> 4) +
  // ((lane & 15) >> 2) (+ 4): output pixel (rj, cj) -> (st rj) W2 + st cj (computed per half: a table of
  // all 8 stays live across the MFMAs)
  const int jl = 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int jmax = g.rk * Q;
  auto band_px = [&](int j) {
    const int rj = (int)fdiv((uint32_t)j, g.fQ), cj = j - rj * Q;
    return j < jmax ? ((rj * st) << W2L) + cj * st : 0;  // past the group: dy = 0 there
  };

  // dy DMA mapping of [64 px][CO_T co] images: round i of thread t writes byte i*8192 + t*16 = mn_off<CO_T>(k, m)
  // with k = i * PXR + t / TPR; the swizzle key of k (k & 63's low bits) does not depend on i, so the
  // thread's column m is the same in every round
  constexpr int RB = CO_T * 2;               // image row bytes
  constexpr int TPR = RB / 16;               // threads per pixel row
  constexpr int PXR = WG3V2_NT / TPR;        // pixels per DMA round: 32 (CO_T = 128) or 64 (CO_T = 64)
  constexpr int DY_ROUNDS = 128 / PXR;
  const int dy_k0 = tid / TPR;
  int dy_m;
  {
    const int kl = dy_k0 & 63, rb = (tid % TPR) * 16;
    int hsw;
    if constexpr (CO_T == 128) hsw = (kl & 3) | (((kl >> 3) & 1) << 2);
    else hsw = ((kl >> 1) & 1) | (((kl >> 3) & 1) << 1);
    dy_m = ((((rb >> 5) ^ hsw) & (CO_T / 16 - 1)) << 4) + ((rb >> 4) & 1) * 8;
  }
  const int s16 = tid & 7;

  auto issue = [&](int grp, char* base) {
    const int n = grp / g.gpi, p0 = (grp - n * g.gpi) * g.rk;
    const int rows = min(g.rk, g.P - p0);
    const int npx = rows * Q;
    // dy rows p0 .. p0 + rows - 1 of image n: npx consecutive pixels (zero past them)
    const bf16_t* dyb = dy + ((int64_t)n * g.P + p0) * Q * g.Cout + co0 + dy_m;
#pragma unroll
    for (int i = 0; i < DY_ROUNDS; ++i) {
      const int k = dy_k0 + i * PXR;
      const bf16_t* a = dyb + (int64_t)k * g.Cout;  // formed unconditionally, then selected
      glds_asm(k < npx ? a : g_zero_page, base + i * 8192 + w * 1024);
    }
    // x band: input rows st*p0 - 1 .. + band_rows - 1, cols -1 .. W (zero outside the image); always 5 DMA
    // rounds of 64 pixels (the band capacity; pixels past the band are zeros nobody reads), addresses
    // selected, not branched around
    char* band = base + WG3V2_DY;
    const int ih0 = st * p0 - 1;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int b = k * 64 + (tid >> 3);
      const int rs = b >> W2L, cs = b & (W2P - 1);
      const int hb = ((b >> 1) & 1) | (((b >> 3) & 1) << 1);
      const int ci = ci0 + 16 * ((s16 >> 1) ^ hb) + 8 * (s16 & 1);
      const int ih = ih0 + rs, iw = cs - 1;
      const bool ok = rs < g.band_rows && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W && cs < W + 2;
      const bf16_t* a = x + (((int64_t)n * H + ih) * W + iw) * g.C + ci;
      glds_asm(ok ? a : g_zero_page, band + k * 8192 + w * 1024);
    }
  };

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const int mcol = 16 * cb + 4 * ((lane & 15) & 3);
  auto half = [&](const char* As, const char* band, int h) {
    const int pj0 = band_px(32 * h + jl), pj1 = band_px(32 * h + jl + 4);
    int alo[3], ahi[3];  // swizzled addresses of the three column shifts (tap row r adds r W2P 128 B)
#pragma unroll
    for (int sx = 0; sx < 3; ++sx) {
      alo[sx] = band_mn_off(pj0 + sx, mcol);
      ahi[sx] = band_mn_off(pj1 + sx, mcol);
    }
    mfma_bf16x8 af[NCB];
#pragma unroll
    for (int i = 0; i < NCB; ++i) af[i] = read_frag<false, CO_T>(As + (h >> 1) * IMG, cow + 16 * i, 32 * (h & 1), lane);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      constexpr int RB = W2P * 128;
      const int roff = (t / 3) * RB;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(band + alo[t % 3] + roff));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(band + ahi[t % 3] + roff));
      s16x8 f;
      f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
      f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
      const mfma_bf16x8 bf = __builtin_bit_cast(mfma_bf16x8, f);
#pragma unroll
      for (int i = 0; i < NCB; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af[i], acc[i][t], 0, 0, 0);
    }
  };
  // the halves with data of this group (a runtime count; one loop body, so its fragments do not pile up
  // in registers across halves); the asm DMA keeps hipcc from draining the next group's loads here
  auto step = [&](int grp, const char* As, char* next) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // this group landed for every wave; every wave is done with `next`
    issue(min(grp + 1, ge - 1), next);
    const int n = grp / g.gpi, p0 = (grp - n * g.gpi) * g.rk;
    const int nh = (min(g.rk, g.P - p0) * Q + 31) >> 5;
    const char* band = As + WG3V2_DY;
    const int h0 = KSPLIT ? wh : 0, hs = KSPLIT ? 2 : 1;
#pragma unroll 1
    for (int h = h0; h < nh; h += hs) half(As, band, h);
  };
  if (gb < ge) {
    issue(gb, s_st0);
    for (int grp = gb; grp < ge; grp += 2) {
      step(grp, s_st0, s_st1);
      if (grp + 1 < ge) step(grp + 1, s_st1, s_st0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // fp32 partials: acc[i][t][q] = dw[co0 + cow + 16 i + (lane & 15)][t][ci0 + 16 cb + 4 (lane >> 4) + q]
  const int64_t Nn = 9LL * g.C;
  const int sl = KSPLIT ? 2 * blockIdx.y + wh : blockIdx.y;
  float* out = slab + (int64_t)sl * g.Cout * Nn;
#pragma unroll
  for (int i = 0; i < NCB; ++i) {
    const int co = co0 + cow + 16 * i + (lane & 15);
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *reinterpret_cast<f32x4*>(out + (int64_t)co * Nn + (int64_t)t * g.C + ci0 + 16 * cb + 4 * (lane >> 4)) =
          acc[i][t];
  }
}

// ------------------------------------------------------------------ stem forward (4x4 valid conv, 16 channels)
// y[n,p,q,co] = sum_(r,s,ci) x[n,p+r,q+s,ci] w[co][r][s][ci] over the 2x2 space-to-depth image: K = 256,
// N = 64, M = 8 M output pixels at batch 640.  The implicit GEMM re-gathers every input byte 16 times
// through L2 and re-streams the 32 KB weight per 128-pixel tile (720 us at bs 640, 3x its HBM roofline,
// on the critical path at the start of every step).  Here a workgroup keeps the weight resident in LDS
// (four [64 co][64 k] K-major images) and walks output rows: a row's 4-input-row band (4 x W pixels x
// 32 B, linear: the ds_read_b128 lane groups then read 16 distinct 16-B slots) is DMA'd once and the
// A fragments (pixel q, k = (s, ci-half) chunks of tap row r) are read at band pixel r*W + q + s.  Two
// band stages: row t+1 is in flight while row t is multiplied; after the MFMAs row t's stage becomes
// the epilogue's staging tile (bf16 row stores + the BN column sums of the conv epilogue).
struct StemGeom {
  int N, H, W, P, Q, Cout;
  int rows;        // N * P output rows (K-steps)
  int rps;         // rows per split
  int band_px;     // 512: four 128-pixel DMA rounds (4 W and every tap read fit)
};

__device__ __forceinline__ int stem_band_row(int b) { return b ^ (((b >> 3) & 1) << 2); }

constexpr int STEMF_W_BYTES = 4 * 64 * BK * 2;  // resident weight: 4 x [64 co][64 k]
constexpr int STEMF_STAGE = 20 * 1024;          // >= 512 band pixels, >= the 128 x 64 staging tile + sums

// The weight and the two stages are separate __shared__ objects and the row loop is unrolled by two,
// so every LDS access names one object: with one dynamic array, the compiler cannot prove that the
// current stage's reads do not alias the next row's in-flight DMA and drains it (vmcnt(0)) before them.
__global__ void __launch_bounds__(NT, 2) conv_stem_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                              StemGeom g, Epi epi) {
  __shared__ __attribute__((aligned(16))) char s_w[STEMF_W_BYTES];
  __shared__ __attribute__((aligned(16))) char s_b0[STEMF_STAGE];
  __shared__ __attribute__((aligned(16))) char s_b1[STEMF_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int rb = blockIdx.x * g.rps, re = min(g.rows, rb + g.rps);
  if (rb >= re) return;

  {  // resident weight [Cout = 64][256] (OHWI flattened), K-major images per 64-deep k block
    PlainK<64> lw;
    lw.p = w;
    lw.rows = 64;
    lw.K = 256;
    lw.ld = 256;
    typename PlainK<64>::State sw;
    lw.init(sw, 0, tid);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) glds_tile(lw, sw, 64 * kb, s_w + kb * (64 * BK * 2), wid);
  }
  auto issue = [&](int row, char* band) {
    const int n = row / g.P, p = row - n * g.P;
    const int64_t xrow0 = ((int64_t)n * g.H + p) * g.W;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = k * 128 + (tid >> 1);
      const bool ok = b < 4 * g.W;
      const bf16_t* q = ok ? x + (xrow0 + b) * 16 + 8 * (tid & 1) : g_zero_page;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)q,
                                       (void __attribute__((address_space(3)))*)(band + k * 4096 + wid * 1024), 16,
                                       0, 0);
    }
  };
  float st1[8], st2[8];  // this thread's BN column sums over all of the workgroup's rows
#pragma unroll
  for (int q = 0; q < 8; ++q) st1[q] = st2[q] = 0.f;
  auto step = [&](int row, char* band, char* next) {
    // row's band (and, first time round, the weight) landed for every wave; every wave is done with
    // the previous row's epilogue, whose staging tile is `next`
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    // unconditional (the last row re-fetches itself into the idle stage): a branch around the DMA
    // makes the compiler's LDS-DMA tracking merge paths and drain it before the reads below
    issue(min(row + 1, re - 1), next);
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        const int ch = (kk >> 3) + (lane >> 4);  // this lane's 8-wide k chunk: (s, ci half)
        const int boff = (r * g.W + (ch >> 1)) * 32 + (ch & 1) * 16;
        mfma_bf16x8 af[4], bw[2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *reinterpret_cast<const mfma_bf16x8*>(band + boff + (wm * 64 + 16 * i + (lane & 15)) * 32);
#pragma unroll
        for (int j = 0; j < 2; ++j) bw[j] = read_frag<true, 64>(s_w + r * (64 * BK * 2), wn * 32 + 16 * j, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
      }
    raw_barrier();  // every wave is done reading the band: it becomes the staging tile
    const int64_t m0 = (int64_t)row * g.Q;
    tile_epilogue_bf16_impl<128, 64, true, true, false>(acc, band, epi, m0, 0, m0 + g.Q, 64, row, st1, st2);
  };
  issue(rb, s_b0);
  for (int row = rb; row < re; row += 2) {
    step(row, s_b0, s_b1);
    if (row + 1 < re) step(row + 1, s_b1, s_b0);
  }
  // one BN-sum flush per workgroup into table row blockIdx.x % R: with at most R workgroups (the host
  // sizes small problems so) every row receives one atomic add and the sums are reproducible
  if (epi.stats) epi_stats_flush(epi, st1, st2, reinterpret_cast<float*>(s_b0 + 128 * 72 * 2), 8, NT, blockIdx.x, 0, 64);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (redundant) band DMA lands before LDS is released
}

// ------------------------------------------------------------------ stem weight gradient (4x4 valid conv, 16 channels)
// The ResNet-50 stem runs as a 4x4 / stride-1 / pad-0 conv over the 2x2 space-to-depth image (16
// channels).  Its weight gradient dw[co][r][s][ci] = sum_(n,p,q) dy[n,p,q,co] x[n,p+r,q+s,ci] is a
// 64 x 256 output with K = N*P*Q (8 M pixels at batch 640): the implicit GEMM gathers im2col(x), i.e.
// every input byte 16 times through L2 (920 us at bs 640, the last — fully exposed — kernel of the
// backward).  Here a K-step is ONE output row (n, p): its dy row ([Q px][64 co], MN-major, padded to
// 128 px) and the 4 input rows it touches (a band of 4 x W pixels x 32 B) are DMA'd into LDS once, and
// the 16 taps read the band at pixel offsets r*W + s — L2 traffic is dy once plus x ~4x (each input row
// feeds 4 output rows, mostly from L2).  Wave w owns tap row r = w: acc[co group][s] over 64 co x 4 s
// x 16 ci.  Band pixels are 32 B; pixel row b is stored at b ^ (((b >> 3) & 1) << 2) so the 8 pixels a
// half-wave's ds_read_b64_tr_b16 touches (b0..b0+3, b0+8..b0+11) fill all 32 8-B slots of a bank row.

constexpr int STEM_STAGE = 128 * 64 * 2 + 512 * 32;  // dy row [128 px][64 co] + the 512-pixel band

// Two row stages as separate __shared__ objects with the row loop unrolled by two (every LDS access
// names one object: see conv_stem_fwd_kernel), two workgroups per CU.  A 4-stage ring at one
// workgroup per CU measured slower (586 vs 457 us, both with the next row's DMA drained by the
// compiler before the reads): occupancy matters more than DMA depth here.
__global__ void __launch_bounds__(NT, 2) conv_stem_wgrad_kernel(const bf16_t* __restrict__ dy,
                                                                const bf16_t* __restrict__ x, StemGeom g,
                                                                float* __restrict__ slab) {
  constexpr int DY_BYTES = 128 * 64 * 2;  // [128 px][64 co]: two [64][64] MN-major images
  __shared__ __attribute__((aligned(16))) char s_st0[STEM_STAGE];
  __shared__ __attribute__((aligned(16))) char s_st1[STEM_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int co0 = blockIdx.x * 64;
  const int rb = blockIdx.y * g.rps, re = min(g.rows, rb + g.rps);  // (stem_splits: never empty)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int row, char* base) {
    const int n = row / g.P, p = row - n * g.P;
    PlainMN<64> la;  // dy row: Q consecutive pixels x 64 output channels
    la.p = dy + (int64_t)row * g.Q * g.Cout + co0;
    la.K = g.Q;
    la.cols = 64;
    la.ld = g.Cout;
    typename PlainMN<64>::State sa;
    la.init(sa, 0, tid);
    glds_tile(la, sa, 0, base, w);
    glds_tile(la, sa, 64, base + DY_BYTES / 2, w);
    // band: input rows p .. p+3, all W pixels, 16 channels (two 16-B chunks per pixel)
    char* band = base + DY_BYTES;
    const bf16_t* row0 = x + ((int64_t)n * g.H + p) * g.W * 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = stem_band_row(k * 128 + (tid >> 1));
      const bf16_t* a = row0 + (int64_t)b * 16 + 8 * (tid & 1);  // formed unconditionally, then selected
      const bf16_t* q = b < 4 * g.W ? a : g_zero_page;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)q,
                                       (void __attribute__((address_space(3)))*)(band + k * 4096 + w * 1024), 16,
                                       0, 0);
    }
  };

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const int mcol = 4 * (lane & 3);  // ci of this lane's transposed reads
  const int jl = 8 * (lane >> 4) + ((lane & 15) >> 2);
  auto step = [&](int row, char* As, char* next) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // row landed for every wave; every wave is done with `next`
    issue(min(row + 1, re - 1), next);  // unconditional: see conv_stem_fwd_kernel
    const char* band = As + DY_BYTES;
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // 32-pixel k-chunks of the (padded) output row
      mfma_bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<false, 64>(As + (c >> 1) * (DY_BYTES / 2), 16 * i, 32 * (c & 1), lane);
      // pixels past Q read finite band data (their dy rows are zero)
      const int j = 32 * c + jl + w * g.W;
#pragma unroll
      for (int sx = 0; sx < 4; ++sx) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(band + stem_band_row(j + sx) * 32 + mcol * 2));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(band + stem_band_row(j + sx + 4) * 32 + mcol * 2));
        s16x8 f;
        f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
        f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
        const mfma_bf16x8 bf = __builtin_bit_cast(mfma_bf16x8, f);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][sx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af[i], acc[i][sx], 0, 0, 0);
      }
    }
  };
  if (rb < re) {  // an empty split would still write its zero slab
    issue(rb, s_st0);
    for (int row = rb; row < re; row += 2) {
      step(row, s_st0, s_st1);
      if (row + 1 < re) step(row + 1, s_st1, s_st0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // fp32 partials: acc[i][s][q] = dw[co0 + 16 i + (lane & 15)][r = w][s][ci = 4 (lane >> 4) + q]
  float* out = slab + (int64_t)blockIdx.y * g.Cout * 256;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + 16 * i + (lane & 15);
#pragma unroll
    for (int sx = 0; sx < 4; ++sx)
      *reinterpret_cast<f32x4*>(out + (int64_t)co * 256 + (w * 4 + sx) * 16 + 4 * (lane >> 4)) = acc[i][sx];
  }
}

// ------------------------------------------------------------------ big-tile kernel (K-major x K-major)
// 256 x 128 output tile, 8 waves (4 along M x 2 along N, 64 x 64 each — the same per-wave work as the
// 128-tile kernel), THREE LDS stages of 48 KB (144 KB of the CU's 160 KB): the DMA of tile t+2 is in
// flight while tile t is multiplied, retired by a counted `s_waitcnt vmcnt(N)` (never 0 inside the
// loop) and a raw `s_barrier` — `__syncthreads()` would drain every outstanding LDS-DMA with
// vmcnt(0) (cdna_hip_programming.md, "Pipelining across barriers").  The two 256-thread halves of the
// workgroup each stage one 128-row half of A and one 64-row half of B with the ordinary 256-thread
// loaders, so every loader / LDS image of the 128-tile kernel is reused unchanged.
// Used for the large-M, N >= 128 GEMMs of conv fwd / dgrad / Linear when they yield >= 256 tiles.
constexpr int BIG_NT = 512;
constexpr int BIG_A_HALF = 128 * BK * 2, BIG_B_HALF = 64 * BK * 2;
constexpr int BIG_STAGE = 2 * BIG_A_HALF + 2 * BIG_B_HALF;
constexpr int BIG_LDS = 3 * BIG_STAGE;

template <class LA, class LB>
__global__ void __launch_bounds__(BIG_NT, 1) gemm_big_kernel(LA la, LB lb, int64_t M, int64_t N, int64_t K,
                                                            int tiles_n, Epi epi) {
  static_assert(LA::kMajor && LB::kMajor && LA::NCH == 4 && LB::NCH == 2, "K-major 128-row A / 64-row B loaders");
  constexpr int BM = 256, BN = 128, TM = 4, TN = 4;
  constexpr int LPT = LA::NCH + LB::NCH;  // glds per thread per K tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = tid >> 8, gtid = tid & 255, gwid = wid & 3;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int nk = (int)((K + BK - 1) / BK);

  typename LA::State sa;
  typename LB::State sb;
  la.init(sa, m0 + 128 * grp, gtid);
  lb.init(sb, n0 + 64 * grp, gtid);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* base = smem + (t % 3) * BIG_STAGE;
    glds_tile(la, sa, (int64_t)t * BK, base + grp * BIG_A_HALF, gwid);
    glds_tile(lb, sb, (int64_t)t * BK, base + 2 * BIG_A_HALF + grp * BIG_B_HALF, gwid);
  };
  if (nk > 0) issue(0);
  if (nk > 1) {
    issue(1);
    wait_vm<LPT>();
  } else {
    wait_vm<0>();
  }
  raw_barrier();
  for (int t = 0; t < nk; ++t) {
    if (t + 2 < nk) issue(t + 2);
    const char* base = smem + (t % 3) * BIG_STAGE;
    const char* As = base + (wm >> 1) * BIG_A_HALF;
    const char* Bs = base + 2 * BIG_A_HALF + wn * BIG_B_HALF;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      mfma_bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag<true, 128>(As, (wm & 1) * 64 + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<true, 64>(Bs, 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (t + 2 < nk) wait_vm<LPT>();  // tile t+1 landed, tile t+2 still in flight
    else wait_vm<0>();
    raw_barrier();
  }

  // epilogue (bf16 output only — the launcher routes fp32 / split-K work to the 128-tile kernel):
  // stage the tile through LDS, then coalesced 16-B row stores (+ addend)
  constexpr int SROW = BN + 8;
  static_assert(BM * SROW * 2 <= BIG_LDS, "staging tile must fit");
  bf16_t* stg = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * 64 + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cc = wn * 64 + 16 * j + 4 * (lane >> 4);
      f32x4 v = acc[i][j];
      if (epi.bias) {
        const int64_t n = n0 + cc;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (n + q < N)
            v[q] += epi.bias_f32 ? ((const float*)epi.bias)[n + q] : bf2f(((const bf16_t*)epi.bias)[n + q]);
      }
      if (epi.relu) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
      }
      u16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
      *reinterpret_cast<u16x4*>(stg + r * SROW + cc) = o;
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int c = tid; c < BM * CPR; c += BIG_NT) {
    const int r = c / CPR, ch = c % CPR;
    const int64_t m = m0 + r, n = n0 + ch * 8;
    if (m >= M || n >= N) continue;
    const int64_t crow = epi_row(epi, m);
    u16x8 v = *reinterpret_cast<const u16x8*>(stg + r * SROW + ch * 8);
    if (epi.addend) {
      float a[8];
      epi_addend8(epi, crow, n, a);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = f2bf(bf2f(v[q]) + a[q]);
    }
    if (epi.act) epi_act8(epi, crow, n, v);
    *reinterpret_cast<u16x8*>((bf16_t*)epi.C + crow * epi.ldc + n) = v;
  }
}

// ------------------------------------------------------------------ wide-tile kernel (K-major x K-major)
// 256 x 256 output tile, 8 waves (2 along M x 4 along N), 128 x 64 per wave (acc[8][4]).  Why: the
// 128-tile kernel needs ~62 B/clk/CU of operand fetch at full MFMA rate (64 KB per 1024 SIMD-cycles
// with 2 workgroups per CU) — about the L2's per-CU share — so it stalls at ~0.9 PF/s on large
// shapes; a 256^2 tile halves the bytes per FLOP and a 128x64 wave tile halves the LDS reads per MFMA.
// Per 64-deep K step a wave runs 8 phases of 8 MFMAs (quadrant x k-half) and reads the fragments of
// the NEXT phase while the current one multiplies; quadrants are ordered so one operand is reused:
//   k 0..31 : (A0,B0) (A0,B1) (A1,B1) (A1,B0)    k 32..63 : (A1,B1) (A1,B0) (A0,B0) (A0,B1)
// which needs only two A and two B fragment sets (fa0/fa1, fb0/fb1; 24 ds_read_b128 per step, the
// minimum).  The next K step's operands are DMA'd (global_load_lds) into the other of two 64 KB LDS
// stages during phases 0-1 and retired by one vmcnt(0) + barrier after phase 6; phase 7's MFMAs run
// behind the first fragment reads of the next step.  Each 256-thread half of the workgroup stages one
// 64-row group of every 128-row operand half with the ordinary 64-row loaders (NCH = 2), so the LDS
// images and fragment reads are those of the 128-tile kernel.
constexpr int W_NT = 512;
constexpr int W_HALF = 128 * BK * 2;  // one 128-row half of an operand tile (16 KB)
constexpr int W_STAGE = 4 * W_HALF;   // A0 A1 B0 B1
constexpr int W_SROW = 256 + 8;       // epilogue staging row (bf16 elements)
constexpr int W_STATS_OFF = 2 * W_STAGE > 256 * W_SROW * 2 ? 2 * W_STAGE : 256 * W_SROW * 2;
constexpr int W_LDS = W_STATS_OFF + (W_NT / 64) * 256 * 2 * 4;  // + epilogue BN-statistics scratch (16 KB)

// VAR (schedule bits; production = 3): bit 0 = s_setprio(1) around each MFMA cluster,
// bit 1 = interleave each MFMA with one of the next phase's ds_reads (sched_group_barrier).
template <int QA, int QB, int VAR>
__device__ __forceinline__ void wide_mma(f32x4 (&acc)[8][4], const mfma_bf16x8 (&fa)[4], const mfma_bf16x8 (&fb)[2]) {
  if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc[4 * QA + i][2 * QB + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[4 * QA + i][2 * QB + j],
                                                                            0, 0, 0);
      if constexpr (VAR & 2) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);    // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // then one DS read
      }
    }
  if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(0);
}

// Fragment of a 128-row operand half.  K-major halves are one [128][64] image; an MN-major half is
// two [64 k][64] images (one per 256-thread group, 8 KB apart), read with ds_read_b64_tr_b16.
template <class L>
__device__ __forceinline__ mfma_bf16x8 wide_frag(const char* half, int row, int kk, int lane) {
  if constexpr (L::kMajor) return read_frag<true, 128>(half, row, kk, lane);
  else return read_frag<false, 64>(half + (row >> 6) * (W_HALF / 2), row & 63, kk, lane);
}

// blockIdx.y = K split (ktiles_per_split K tiles each); split launches write fp32 slabs.
// the wide kernel compiles the BN-backward statistics epilogue only for plain-operand launches (a dgrad
// with statistics never takes a gathered wide tile: dispatch_bn routes it to the 128 tile)
template <class L> struct WideBst : std::false_type {};
template <int R> struct WideBst<PlainK<R>> : std::true_type {};
template <int R> struct WideBst<PlainMN<R>> : std::true_type {};

template <class LA, class LB, int VAR>
__global__ void __launch_bounds__(W_NT, 1) gemm_wide_kernel(LA la, LB lb, int64_t M, int64_t N, int64_t K,
                                                           int tiles_n, int ktiles_per_split, Epi epi) {
  static_assert(LA::NCH == 2 && LB::NCH == 2, "64-row / 64-column loaders");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = tid >> 8, gtid = tid & 255, gwid = wid & 3;
  const int wr = wid >> 2, wc = wid & 3;
  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  grouped_tile(tile, ntiles / tiles_n, tiles_n, 8, tm, tn);
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int ktiles = (int)((K + BK - 1) / BK);
  const int kt0 = blockIdx.y * ktiles_per_split;
  const int nk = min(ktiles, kt0 + ktiles_per_split);  // K-tile loop bound (exclusive)

  typename LA::State sa0, sa1;
  typename LB::State sb0, sb1;
  la.init(sa0, m0 + 64 * grp, gtid);
  la.init(sa1, m0 + 128 + 64 * grp, gtid);
  lb.init(sb0, n0 + 64 * grp, gtid);
  lb.init(sb1, n0 + 128 + 64 * grp, gtid);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue_a = [&](int t) {
    char* b = smem + (t & 1) * W_STAGE + grp * (W_HALF / 2);
    glds_tile(la, sa0, (int64_t)t * BK, b, gwid);
    glds_tile(la, sa1, (int64_t)t * BK, b + W_HALF, gwid);
  };
  auto issue_b = [&](int t) {
    char* b = smem + (t & 1) * W_STAGE + 2 * W_HALF + grp * (W_HALF / 2);
    glds_tile(lb, sb0, (int64_t)t * BK, b, gwid);
    glds_tile(lb, sb1, (int64_t)t * BK, b + W_HALF, gwid);
  };
  // fragments: A rows of this wave's half (wr), B rows (= output columns) of its 64-column slice
  const int a_off = wr * W_HALF, b_off = 2 * W_HALF + (wc >> 1) * W_HALF, b_row = (wc & 1) * 64;
  auto rd_a = [&](const char* st, int qa, int kk, mfma_bf16x8 (&f)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = wide_frag<LA>(st + a_off, 64 * qa + 16 * i, kk, lane);
  };
  auto rd_b = [&](const char* st, int qb, int kk, mfma_bf16x8 (&f)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) f[j] = wide_frag<LB>(st + b_off, b_row + 32 * qb + 16 * j, kk, lane);
  };

  {
  mfma_bf16x8 fa0[4], fa1[4], fb0[2], fb1[2];
  if (kt0 < nk) {
    issue_a(kt0);
    issue_b(kt0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    rd_a(smem + (kt0 & 1) * W_STAGE, 0, 0, fa0);
    rd_b(smem + (kt0 & 1) * W_STAGE, 0, 0, fb0);
  }
  for (int t = kt0; t < nk; ++t) {
    const char* cs = smem + (t & 1) * W_STAGE;
    const bool more = t + 1 < nk;
    // k 0..31
    if (more) issue_a(t + 1);
    rd_b(cs, 1, 0, fb1);
    wide_mma<0, 0, VAR>(acc, fa0, fb0);
    if (more) issue_b(t + 1);
    rd_a(cs, 1, 0, fa1);
    wide_mma<0, 1, VAR>(acc, fa0, fb1);
    wide_mma<1, 1, VAR>(acc, fa1, fb1);
    rd_a(cs, 1, 32, fa0);
    rd_b(cs, 1, 32, fb1);
    wide_mma<1, 0, VAR>(acc, fa1, fb0);
    // k 32..63
    rd_b(cs, 0, 32, fb0);
    wide_mma<1, 1, VAR>(acc, fa0, fb1);
    rd_a(cs, 0, 32, fa1);
    wide_mma<1, 0, VAR>(acc, fa0, fb0);
    wide_mma<0, 0, VAR>(acc, fa1, fb0);
    if (more) {
      // next step's operands landed (own DMAs, then everyone's); this stage is no longer read
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const char* ns = smem + ((t + 1) & 1) * W_STAGE;
      rd_a(ns, 0, 0, fa0);
      rd_b(ns, 0, 0, fb0);
    }
    wide_mma<0, 1, VAR>(acc, fa1, fb1);
  }
  }
  __syncthreads();  // every wave is done with the operand stages before they become the staging tile
  wide_tile_epilogue<4, WideBst<LA>::value && WideBst<LB>::value>(acc, smem, W_STATS_OFF, epi, m0, n0, M, N, tm, blockIdx.y);
}

// Split-K reduction: out[m, n] = act(sum_s slab[s, m, n] + bias[n]).  A workgroup is (256 / L) output
// float4s x L split lanes; each lane keeps 8 slab loads in flight and the L partials meet in LDS, so
// a small output with a deep split (conv wgrad of 64 x 64 with ~1000 slabs) still spreads over
// many CUs instead of serialising 1000 dependent loads per thread.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, int splits, int64_t M,
                                                            int64_t N, int lanes_log2, Epi epi) {
  __shared__ f32x4 red[256];
  if (epi.rowsum_out && epi.rowsum_mode == 4) {  // trailing workgroups: the bias gradient's split sums
    const int rb = (int)((M + 255) / 256);
    const int b = (int)blockIdx.x - ((int)gridDim.x - rb);
    if (b >= 0) {
      const int64_t i = (int64_t)b * 256 + threadIdx.x;
      if (i < M) {
        const float* rs = (const float*)epi.rowsum;
        float v = 0.f;
        for (int s = 0; s < splits; ++s) v += rs[(int64_t)s * M + i];
        if (epi.rowsum_out_bf16) ((bf16_t*)epi.rowsum_out)[i] = f2bf(v);
        else ((float*)epi.rowsum_out)[i] = v;
      }
      return;
    }
  }
  const int L = 1 << lanes_log2;
  const int lane = threadIdx.x & (L - 1), o = threadIdx.x >> lanes_log2;
  const int64_t total4 = M * N / 4;
  const int64_t t = (int64_t)blockIdx.x * (256 >> lanes_log2) + o;
  const int64_t sstride = M * N;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (t < total4) {
    const float* p = slab + t * 4;
    f32x4 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    int s = lane;
    for (; s + 7 * L < splits; s += 8 * L) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += *reinterpret_cast<const f32x4*>(p + (int64_t)(s + u * L) * sstride);
    }
    for (; s < splits; s += L) a[0] += *reinterpret_cast<const f32x4*>(p + (int64_t)s * sstride);
    acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  if (L > 1) {
    red[threadIdx.x] = acc;
    __syncthreads();
    if (lane != 0) return;
    for (int l = 1; l < L; ++l) acc += red[threadIdx.x + l];
  }
  if (t >= total4) return;
  f32x4 v = acc;
  const int64_t m = (t * 4) / N, n = (t * 4) % N;
  if (epi.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] += epi.bias_f32 ? ((const float*)epi.bias)[n + r] : bf2f(((const bf16_t*)epi.bias)[n + r]);
    }
    if (epi.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    }
    if (epi.c_f32) {
      *reinterpret_cast<f32x4*>((float*)epi.C + m * epi.ldc + n) = v;
    } else {
      u16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(v[r]);
      *reinterpret_cast<u16x4*>((bf16_t*)epi.C + m * epi.ldc + n) = o;
    }
}

// Stride phases of a dgrad with dilation 1 (or stride 1): phase ph of the rows takes the taps
// r = r0 + ri*st, ri < Rv, with r0 = (ph + pad) mod st.
struct TapPhase {
  int r0, n;     // first tap, tap count
  int cum;       // taps of all earlier phases
  int base;      // p = hh + base - ri*step
};
__host__ __device__ inline TapPhase tap_phase(int ph, int R, int st, int pad, int dil) {
  TapPhase t;
  if (st == 1) {
    t.r0 = 0; t.n = R; t.cum = 0; t.base = pad;  // p = h + pad - r*dil
    return t;
  }
  t.cum = 0;
  for (int q = 0; q <= ph; ++q) {
    const int r0 = (q + pad) % st;
    const int n = r0 < R ? (R - r0 + st - 1) / st : 0;
    if (q < ph) t.cum += n;
    else { t.r0 = r0; t.n = n; t.base = (q + pad - r0) / st; }
  }
  return t;
}

// Weight transpose for conv dgrad, phase-packed: for every (ph, pw) phase block (row-major) the taps
// it uses are stored as wt[ci][ri][si][co] (for stride 1 this is simply wt[ci][r][s][co]).
// blockIdx.z = source tap (r, s).  `packed` = 0 keeps the plain [ci][r][s][co] layout (folded path).
__global__ void __launch_bounds__(256) conv_wt_transpose_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                                                int Cout, int R, int S, int Cin, int st, int pad,
                                                                int packed) {
  __shared__ bf16_t tile[32][33];
  const int rs = blockIdx.z, r = rs / S, sx = rs % S;
  int64_t base = 0;
  int T = R * S, t = rs;
  if (packed && st > 1) {
    const int ph = ((r - pad) % st + st) % st, pw = ((sx - pad) % st + st) % st;
    const TapPhase a = tap_phase(ph, R, st, pad, 1), b = tap_phase(pw, S, st, pad, 1);
    base = ((int64_t)a.cum * S + (int64_t)a.n * b.cum) * Cin * Cout;
    T = a.n * b.n;
    t = ((r - a.r0) / st) * b.n + (sx - b.r0) / st;
  }
  const int co0 = blockIdx.y * 32, ci0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int yy = ty; yy < 32; yy += 8) {
    const int co = co0 + yy, ci = ci0 + tx;
    tile[yy][tx] = (co < Cout && ci < Cin) ? w[((int64_t)co * R * S + rs) * Cin + ci] : (bf16_t)0;
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    const int ci = ci0 + yy, co = co0 + tx;
    if (co < Cout && ci < Cin) wt[base + ((int64_t)ci * T + t) * Cout + co] = tile[tx][yy];
  }
}

// ------------------------------------------------------------------ dgrad phases no tap reaches
// A strided conv's dgrad runs one launch per stride phase (dx pixels (hh*st + ph, ww*st + pw)); a phase
// that no tap reaches (3 of 4 for a stride-2 1x1 conv) is dx = addend (ReLU-bit masked) or 0.  One
// streaming pass, 8 channels per thread, instead of a K = 0 GEMM launch whose 128-tile staged
// epilogue wrote them at ~2.6 TB/s (56^2 256 -> 512 / 2: 3 x ~95 us).
__global__ void __launch_bounds__(256) dgrad_fill_phase_kernel(void* __restrict__ dx, int dx_f32,
                                                               const bf16_t* __restrict__ addend,
                                                               const uint8_t* __restrict__ bits, int64_t total,
                                                               FastDiv fC8, FastDiv fWh, FastDiv fHh, int H, int W,
                                                               int C, int st, int ph, int pw) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t tt = (uint32_t)t;  // total < 2^31 (host-checked)
    const uint32_t pix = fdiv(tt, fC8);
    const int c8 = (int)(tt - pix * fC8.d);
    const uint32_t r1 = fdiv(pix, fWh);
    const int ww = (int)(pix - r1 * fWh.d);
    const uint32_t n = fdiv(r1, fHh);
    const int hh = (int)(r1 - n * fHh.d);
    const int64_t row = ((int64_t)n * H + hh * st + ph) * W + ww * st + pw;
    const int64_t off = row * C + c8 * 8;
    float v[8];
    if (addend) {
      const u16x8 a = *reinterpret_cast<const u16x8*>(addend + off);
      const uint32_t mb = bits ? bits[off >> 3] : 0xFFu;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = (mb >> q) & 1u ? bf2f(a[q]) : 0.f;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = 0.f;
    }
    if (dx_f32) {
      float* d = (float*)dx + off;
      *reinterpret_cast<f32x4*>(d) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(d + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
      u16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = f2bf(v[q]);
      *reinterpret_cast<u16x8*>((bf16_t*)dx + off) = o;
    }
  }
}

// ------------------------------------------------------------------ host-side dispatch
struct Plan {
  int bm, bn;       // 64 or 128 each
  int tiles_m, tiles_n, splits, ktiles_per_split;
};

// target_blocks: workgroups wanted in flight (>= 2 per CU); split-K is only used when the output
// tiles alone cannot fill the chip, with >= 4 K tiles per split and at most max_splits slabs.
Plan plan_gemm(int64_t M, int64_t N, int64_t K, bool allow_split, int target_blocks, int max_splits = 64) {
  Plan p;
  p.bm = M <= 64 ? 64 : 128;
  p.bn = N <= 64 ? 64 : 128;
  p.tiles_m = (int)((M + p.bm - 1) / p.bm);
  p.tiles_n = (int)((N + p.bn - 1) / p.bn);
  const int ktiles = (int)((K + BK - 1) / BK);
  p.splits = 1;
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  if (allow_split && tiles < target_blocks) {
    int s = (int)(target_blocks / tiles);
    const int max_s = ktiles / 4 > 1 ? ktiles / 4 : 1;  // keep >= 4 K-tiles per split
    if (s > max_s) s = max_s;
    if (s > max_splits) s = max_splits;
    p.splits = s < 1 ? 1 : s;
  }
  p.ktiles_per_split = ktiles > 0 ? (ktiles + p.splits - 1) / p.splits : 0;
  p.splits = p.ktiles_per_split > 0 ? (ktiles + p.ktiles_per_split - 1) / p.ktiles_per_split : 1;
  if (p.splits < 1) p.splits = 1;
  return p;
}

// conv wgrad: M = Cout, N = R*S*C are small, K = N*P*Q is huge -> deep split-K.  Aim for 2 workgroups
// per CU (one workgroup per CU leaves every SIMD with a single wave: SQ_WAIT_ANY doubled on the
// 14x14 3x3 256 layer at 252 workgroups), with the fp32 partial slabs (written + re-read once)
// capped at 48 MB but always allowing 4 splits.
// PDA_WGRAD_CUS=n sizes every split-K (weight-gradient) grid for n CUs instead of all 256: the
// wgrad kernels hold a whole CU per workgroup pair (230-256 VGPRs x 2 waves per SIMD) for their
// entire one-round lifetime, so a side-stream wgrad sized for the chip locks the main stream's
// BN / dgrad kernels out of every CU until it drains; fewer, longer-lived split-K workgroups leave
// 256 - n CUs to the critical path.  ResNet-50 bs 640 (profiles/r2_wgrad_cus_sweep_v26.jsonl, two
// interleaved passes): 256 -> 11.34k img/s, 128 -> 11.29k, 160 -> 11.43k, 176 -> 11.45k, 184-224 ->
// 11.47-11.56k (plateau); default 192.
int wgrad_cus() {
  static const int n = [] {
    const char* e = getenv("PDA_WGRAD_CUS");
    int v = e ? atoi(e) : 192;
    return v < 16 ? 16 : (v > 256 ? 256 : v);
  }();
  return n;
}

int env_cus(const char* name) {  // per-kernel-family override of wgrad_cus() (A/B knobs)
  const char* e = getenv(name);
  if (!e) return wgrad_cus();
  int v = atoi(e);
  return v < 16 ? 16 : (v > 256 ? 256 : v);
}
int wide_wgrad_cus() {
  static const int n = env_cus("PDA_WGRAD_CUS_WIDE");
  return n;
}
int wg3_wgrad_cus() {
  static const int n = env_cus("PDA_WGRAD_CUS_WG3");
  return n;
}

Plan plan_wgrad(int64_t M, int64_t N, int64_t K, bool allow_split) {
  int64_t cap = ((int64_t)48 << 20) / (M * N * 4);
  if (cap > 1024) cap = 1024;
  if (cap < 4) cap = 4;
  return plan_gemm(M, N, K, allow_split, 2 * wgrad_cus(), (int)cap);
}

// loaders whose GEMM can be a conv data gradient (the only producers of BN-backward sums; a stride-1
// 3x3 dgrad is a forward conv over flipped weights)
template <class L> struct BstLoader : std::false_type {};
template <int R> struct BstLoader<ConvFwdK<R>> : std::true_type {};
template <int R> struct BstLoader<ConvFwdKU<R>> : std::true_type {};
template <int R> struct BstLoader<PlainK<R>> : std::true_type {};
template <int R> struct BstLoader<PlainMN<R>> : std::true_type {};
template <int R> struct BstLoader<ConvDgradK<R>> : std::true_type {};
template <int R> struct BstLoader<ConvDgradPhaseK<R>> : std::true_type {};
template <int R> struct BstLoader<ConvDgradPhaseKU<R>> : std::true_type {};

template <int BM, int BN, class LA, class LB>
hipError_t launch(const LA& la, const LB& lb, int64_t M, int64_t N, int64_t K, const Plan& p, Epi epi,
                  float* slab, hipStream_t st) {
  const int ntiles = p.tiles_m * p.tiles_n;
  Epi e = epi;
  if (p.splits > 1) e.slab = slab;
  static const bool lean = [] {  // PDA_EPI_BST_LEAN=0: every launch takes the BN-backward-sums build (A/B)
    const char* v = getenv("PDA_EPI_BST_LEAN");
    return !(v && v[0] == '0');
  }();
  if (e.bst_z || (!lean && BstLoader<LA>::value)) {  // BN-backward sums: only the data-gradient loaders produce a BN input's gradient
    if constexpr (BstLoader<LA>::value)
      gemm_kernel<BM, BN, LA, LB, true><<<dim3(ntiles, p.splits), NT, 0, st>>>(la, lb, M, N, K, p.tiles_n,
                                                                               p.ktiles_per_split, e);
    else
      return hipErrorNotSupported;
  } else {
    gemm_kernel<BM, BN, LA, LB><<<dim3(ntiles, p.splits), NT, 0, st>>>(la, lb, M, N, K, p.tiles_n,
                                                                       p.ktiles_per_split, e);
  }
  PDA_CHECK_HIP(hipGetLastError());
  if (p.splits > 1) {
    int ll = 0;  // split lanes per output: ~16 slabs per lane, at most 16 lanes
    while (ll < 4 && (p.splits >> ll) > 16) ++ll;
    const int64_t per_block = 256 >> ll;
    const int64_t g = (M * N / 4 + per_block - 1) / per_block;
    splitk_reduce_kernel<<<(unsigned)g, 256, 0, st>>>(slab, p.splits, M, N, ll, epi);
    PDA_CHECK_HIP(hipGetLastError());
  }
  return hipSuccess;
}

// The 256 x 128 three-stage kernel only pays off on long-K GEMMs with many tiles (8192^3: 0.96 vs
// 0.88 PF/s); on every ResNet-50 conv shape and at 4096^3 the 128-tile kernel (2 workgroups/CU, more
// tiles in flight) measured equal or faster (profiles/r1_conv_gemm_microbench_v6*.jsonl), so it is
// selected for K >= 2048 with >= 512 tiles.  PDA_GEMM_BIG=0 disables it, =1 forces it where legal.
bool use_big(int64_t M, int64_t N, int64_t K, const Plan& p, const Epi& epi) {
  static const int mode = [] {
    const char* e = getenv("PDA_GEMM_BIG");
    return e ? (e[0] == '0' ? 0 : 2) : 1;
  }();
  if (mode == 0 || p.splits > 1 || epi.c_f32 || epi.slab || epi.stats || N < 128) return false;
  const int64_t tiles = ((M + 255) / 256) * ((N + 127) / 128);
  if (mode == 2) return tiles >= 1;
  return K >= 2048 && tiles >= 512;
}

template <class LA, class LB>
hipError_t launch_big(const LA& la, const LB& lb, int64_t M, int64_t N, int64_t K, Epi epi, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big_kernel<LA, LB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, BIG_LDS);
    return true;
  }();
  (void)attr;
  const int tiles_n = (int)((N + 127) / 128);
  const int ntiles = (int)((M + 255) / 256) * tiles_n;
  gemm_big_kernel<LA, LB><<<ntiles, BIG_NT, BIG_LDS, st>>>(la, lb, M, N, K, tiles_n, epi);
  return hipGetLastError();
}

// 256 x 256 wide-tile kernel: bf16 output, no split-K / statistics, N >= 256.  PDA_GEMM_WIDE=0
// disables it, =1 forces it wherever legal; by default it is chosen when its tile count keeps the
// chip's 256 CUs about as busy as the 128-tile kernel's (see wide_pays).
int g_wide_override = -1;  // set_gemm_paths(): tests / benchmarks force a path at run time

int wide_mode() {
  static const int mode = [] {
    const char* e = getenv("PDA_GEMM_WIDE");
    return e ? (e[0] == '0' ? 0 : 2) : 1;
  }();
  return g_wide_override >= 0 ? g_wide_override : mode;
}

bool wide_pays(int64_t M, int64_t N) {
  // A wide tile does 4x a 128-tile's work ~1.35x more efficiently per CU (measured on the ResNet-50
  // conv shapes and 4096^3, profiles/r1_conv_gemm_microbench_v7_wide.jsonl); compare the two
  // configurations' wave-quantised times over 256 CUs (1 wide / 2 narrow workgroups per CU).
  const double wt = (double)((M + 255) / 256) * ((N + 255) / 256);
  const double nt = (double)((M + 127) / 128) * ((N + 127) / 128);
  const double w_time = std::ceil(wt / 256.0) * 4.0 / 1.35, n_time = std::ceil(nt / 512.0) * 2.0;
  return w_time < n_time;
}

// PDA_WIDE_MIN_K: shortest reduction that takes the (one workgroup per CU) wide tile; below it the
// 128-tile kernel's two workgroups per CU overlap one tile's epilogue stores with the other's loads
int wide_min_k() {
  static const int k = [] {
    const char* e = getenv("PDA_WIDE_MIN_K");
    return e ? atoi(e) : 64;
  }();
  return k;
}

bool use_wide(int64_t M, int64_t N, int64_t K, const Plan& p, const Epi& epi) {
  const int mode = wide_mode();
  if (mode == 0 || p.splits > 1 || epi.c_f32 || epi.slab || N < 256 || K < 64) return false;
  if (mode == 1 && K < wide_min_k()) return false;
  if (mode == 2) return true;
  return wide_pays(M, N);
}

// Split-K GEMMs (conv wgrad: small M x N, huge K).  The wide tile pays when it wastes little of
// M x N: compare useful-work fractions, the wide kernel's at its measured ~1.35x per-CU advantage
// (more for wgrad, whose MN-major operands need two ds_read_b64_tr per fragment — the wide tile's
// 128 x 64 wave tile halves those reads per MFMA).  One 512-thread workgroup per CU means ~2x the
// narrow plan's splits; the fp32 slabs are capped at 96 MB (the 128-tile plan's 48 MB cap starved
// the wide launches of workgroups: 108 of 256 CUs on the 7x7 512->512 3x3 wgrad).
int wide_split_count(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int ktiles = (int)((K + BK - 1) / BK);
  int s = (int)(wide_wgrad_cus() / tiles);  // floor: a 257th workgroup would start a second round on one CU
  const int max_s = ktiles / 4 > 1 ? ktiles / 4 : 1;
  int64_t cap = ((int64_t)96 << 20) / (M * N * 4);
  if (cap < 4) cap = 4;
  if (s > max_s) s = max_s;
  if (s > cap) s = (int)cap;
  return s < 1 ? 1 : s;
}

// Returns the wide split count (0: keep the 128-tile plan).
int wgrad_wide_mode() {  // PDA_WGRAD_WIDE=0: split-K GEMMs stay on the 128-tile kernel (A/B knob)
  static const int m = [] {
    const char* e = getenv("PDA_WGRAD_WIDE");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return m;
}

int wide_splits(int64_t M, int64_t N, int64_t K, const Plan& p, const Epi& epi) {
  const int mode = wide_mode();
  if (mode == 0 || !wgrad_wide_mode() || p.splits <= 1 || epi.stats || K < 64) return 0;
  if (mode == 1) {
    if (M < 256 || N < 256) return 0;
    const double useful = (double)M * N;
    const double w = 1.35 * useful / ((double)((M + 255) / 256 * 256) * (double)((N + 255) / 256 * 256));
    const double n = useful / ((double)((M + p.bm - 1) / p.bm * p.bm) * (double)((N + p.bn - 1) / p.bn * p.bn));
    if (w < 1.05 * n) return 0;
  }
  return wide_split_count(M, N, K);
}



template <class LA, class LB, int VAR>
hipError_t launch_wide_v(const LA& la, const LB& lb, int64_t M, int64_t N, int64_t K, Epi epi, int splits,
                         hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_wide_kernel<LA, LB, VAR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, W_LDS);
    return true;
  }();
  (void)attr;
  const int tiles_n = (int)((N + 255) / 256);
  const int ntiles = (int)((M + 255) / 256) * tiles_n;
  const int ktiles = (int)((K + BK - 1) / BK);
  const int kps = splits > 1 ? (ktiles + splits - 1) / splits : (ktiles > 0 ? ktiles : 1);
  gemm_wide_kernel<LA, LB, VAR><<<dim3(ntiles, splits), W_NT, W_LDS, st>>>(la, lb, M, N, K, tiles_n, kps, epi);
  return hipGetLastError();
}

// splits > 1: epi.slab receives [splits][M][N] fp32 partials, reduced (with the caller's epilogue)
// by splitk_reduce_kernel; the effective split count is recomputed from the per-split K tiles.
template <class LA, class LB>
hipError_t launch_wide(const LA& la, const LB& lb, int64_t M, int64_t N, int64_t K, Epi epi, hipStream_t st,
                       int splits = 1, float* slab = nullptr) {
  Epi e = epi;
  if (splits > 1) {
    const int ktiles = (int)((K + BK - 1) / BK);
    const int kps = (ktiles + splits - 1) / splits;
    splits = (ktiles + kps - 1) / kps;
  }
  if (splits > 1) e.slab = slab;
  const hipError_t r = launch_wide_v<LA, LB, 3>(la, lb, M, N, K, e, splits, st);
  if (r != hipSuccess || splits <= 1) return r;
  int ll = 0;
  while (ll < 4 && (splits >> ll) > 16) ++ll;
  const int64_t per_block = 256 >> ll;
  const int64_t g = (M * N / 4 + per_block - 1) / per_block;
  splitk_reduce_kernel<<<(unsigned)g, 256, 0, st>>>(slab, splits, M, N, ll, epi);
  return hipGetLastError();
}

// Plain-operand GEMMs that take the 256 x 256 tile run on the pipelined kernel of gemm_pp.hip
// (PDA_GEMM_PP=0: the 2-stage wide kernel above, for A/B).  Conv gathers stay on the wide kernel.
template <class L> struct IsPlain : std::false_type {};
template <int R> struct IsPlain<PlainK<R>> : std::true_type {};
template <int R> struct IsPlain<PlainMN<R>> : std::true_type {};

int g_pp_override = -1;  // set_gemm_pp(): tests force the pipelined kernel on / off at run time

bool pp_mode() {
  static const bool on = [] {
    const char* e = getenv("PDA_GEMM_PP");
    return !(e && e[0] == '0');
  }();
  return g_pp_override >= 0 ? g_pp_override != 0 : on;
}

// PDA_GEMM_PP_CONV=0: implicit-GEMM convolutions stay on the 2-stage wide kernel (A/B knob)
bool pp_conv_mode() {
  static const bool on = [] {
    const char* e = getenv("PDA_GEMM_PP_CONV");
    return !(e && e[0] == '0');
  }();
  return on;
}

// PDA_SPLITK_FIXUP=1: split-K weight gradients on the pipelined tile reduce in the kernel (splitk_fixup in
// gemm_epi.h: the last split of each tile sums the slabs) instead of the separate reduce launch.  Opt-in:
// measured 7 % slower on GPT-2-medium and 13 % on ResNet-50 (profiles/r6_splitk_fixup_DROPPED.jsonl) —
// every split's release fence writes its XCD's whole L2 back while the compute stream's kernels fill it,
// and a deep split (12-48 slabs) serialises the sum on one CU per tile.
int g_fixup_override = -1;  // set_splitk_fixup(): tests compare both paths in one process

bool splitk_fixup_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_SPLITK_FIXUP");
    return e && e[0] == '1';
  }();
  return g_fixup_override >= 0 ? g_fixup_override != 0 : on;
}

// Arrival counters of the in-kernel split-K fix-up: one zeroed pool per device, handed out round-robin,
// `tiles` counters per launch.  A launch's last arrivals re-zero their counters, so the pool is all zeros
// between launches, and two launches share counters only 2^20 tiles of later launches apart (never while
// both run).  Null (the caller reduces with a separate launch) when disabled, or when the pool would have
// to be created while `st` is capturing a graph.
int* splitk_tickets(int64_t tiles, hipStream_t st) {
  constexpr int64_t kPool = (int64_t)1 << 20;
  if (!splitk_fixup_on() || tiles <= 0 || tiles > kPool / 4) return nullptr;
  static std::mutex mu;
  static int* pool[64] = {};
  static int64_t next[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!pool[dev]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int* p = nullptr;
    if (hipMalloc(&p, kPool * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, kPool * sizeof(int), st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    pool[dev] = p;
  }
  if (next[dev] + tiles > kPool) next[dev] = 0;
  int* t = pool[dev] + next[dev];
  next[dev] += tiles;
  return t;
}

// returns hipErrorNotSupported when the pipelined kernel cannot take the shape (the caller falls back)
template <class LA, class LB>
hipError_t launch_pp_plain(const LA& la, const LB& lb, int64_t M, int64_t N, int64_t K, Epi epi, hipStream_t st,
                           int splits, float* slab, int* used_out = nullptr) {
  Epi e = epi;
  if (splits > 1) {
    e.slab = slab;
    // MN-major x MN-major (weight gradients): the kernel's last split of each tile reduces in place
    if constexpr (!LA::kMajor && !LB::kMajor) e.tickets = splitk_tickets(((M + 255) / 256) * ((N + 255) / 256), st);
  }
  int used = splits;
  const hipError_t r = gemm_pp(la.p, LA::kMajor, la.ld, lb.p, LB::kMajor, lb.ld, M, N, K, e, splits, -1, st, &used);
  if (used_out) *used_out = used;
  if (r == hipErrorInvalidValue) return hipErrorNotSupported;
  if (r != hipSuccess || used <= 1 || e.tickets) return r;
  int ll = 0;
  while (ll < 4 && (used >> ll) > 16) ++ll;
  const int64_t per_block = 256 >> ll;
  const int64_t g = (M * N / 4 + per_block - 1) / per_block;
  const int64_t rb = (epi.rowsum_out && epi.rowsum_mode == 4) ? (M + 255) / 256 : 0;
  splitk_reduce_kernel<<<(unsigned)(g + rb), 256, 0, st>>>(slab, used, M, N, ll, epi);
  return hipGetLastError();
}

template <template <int> class TA, template <int> class TB, class MakeA, class MakeB>
hipError_t dispatch_bn(int64_t M, int64_t N, int64_t K, const Plan& p, Epi epi, float* slab, hipStream_t st,
                       MakeA make_a, MakeB make_b) {
  if constexpr (IsPlain<TA<64>>::value && IsPlain<TB<64>>::value) {
    if (pp_mode()) {
      int ws = 0;
      if (use_wide(M, N, K, p, epi)) ws = 1;
      else if (slab) ws = wide_splits(M, N, K, p, epi);
      if (ws > 0) {
        const hipError_t r = launch_pp_plain(make_a(TA<64>{}), make_b(TB<64>{}), M, N, K, epi, st, ws, slab);
        if (r != hipErrorNotSupported) return r;
      }
    }
  }
  if (use_wide(M, N, K, p, epi) && ((WideBst<TA<64>>::value && WideBst<TB<64>>::value) || !epi.bst_z))
    return launch_wide(make_a(TA<64>{}), make_b(TB<64>{}), M, N, K, epi, st);
  if (slab) {
    const int ws = wide_splits(M, N, K, p, epi);
    if (ws > 0) return launch_wide(make_a(TA<64>{}), make_b(TB<64>{}), M, N, K, epi, st, ws, slab);
  }
  if constexpr (TA<128>::kMajor && TB<64>::kMajor) {
    if (use_big(M, N, K, p, epi)) return launch_big(make_a(TA<128>{}), make_b(TB<64>{}), M, N, K, epi, st);
  }
  if (p.bm == 64) {
    if (p.bn == 64) return launch<64, 64>(make_a(TA<64>{}), make_b(TB<64>{}), M, N, K, p, epi, slab, st);
    return launch<64, 128>(make_a(TA<64>{}), make_b(TB<128>{}), M, N, K, p, epi, slab, st);
  }
  if (p.bn == 64) return launch<128, 64>(make_a(TA<128>{}), make_b(TB<64>{}), M, N, K, p, epi, slab, st);
  return launch<128, 128>(make_a(TA<128>{}), make_b(TB<128>{}), M, N, K, p, epi, slab, st);
}

ConvGeom make_geom(int H, int W, int C, int P, int Q, int R, int S, int st, int pad, int dil, int Cg) {
  ConvGeom g;
  g.H = H; g.W = W; g.C = C; g.P = P; g.Q = Q; g.R = R; g.S = S; g.st = st; g.pad = pad; g.dil = dil; g.Cg = Cg;
  g.fC = make_fastdiv((uint32_t)Cg);
  g.fS = make_fastdiv((uint32_t)S);
  g.fQ = make_fastdiv((uint32_t)Q);
  g.fP = make_fastdiv((uint32_t)P);
  g.fW = make_fastdiv((uint32_t)W);
  g.fH = make_fastdiv((uint32_t)H);
  return g;
}

bool dgrad_phased(int stride, int dil) { return stride == 1 || dil == 1; }

}  // namespace

// (ping-pong schedules of the wide kernel — the two wave groups alternating MFMA and load sections —
// measured slower on every plain GEMM and most convs: profiles/r3_wide_pingpong_DROPPED.jsonl)
// (a register-direct wide epilogue — 8-byte stores from the accumulators, no LDS staging — measured
// 6 % slower on the headline step than the staged 16-byte row stores: profiles/
// r3_epi_direct_DROPPED_and_transformers.jsonl)
void set_gemm_paths(int wide) { g_wide_override = wide; }
void set_gemm_pp(int on) { g_pp_override = on; }
void set_splitk_fixup(int on) { g_fixup_override = on; }

// slab sizing covers both the 128-tile plan and the wide tile's (possibly deeper) split
int64_t split_slab_floats(int64_t M, int64_t N, int64_t K, const Plan& p) {
  if (p.splits <= 1) return 0;
  int s = p.splits;
  const int w = wide_split_count(M, N, K);
  if (w > s) s = w;
  return (int64_t)s * M * N;
}

int64_t gemm_slab_floats(int64_t M, int64_t N, int64_t K, bool allow_split) {
  return split_slab_floats(M, N, K, plan_gemm(M, N, K, allow_split, 512));
}

// C[M,N] = A[M,K] * B[K,N].  a_kmajor: A(m,k)=A[m*lda+k] else A[k*lda+m];
// b_kmajor: B(k,n)=B[n*ldb+k] else B[k*ldb+n].  K, N must be multiples of 8 (N of 4 for the store).
hipError_t gemm_bf16(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                     void* C, bool c_f32, int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                     bool bias_f32, bool relu, float* slab, bool allow_split, hipStream_t st) {
  Plan p = plan_gemm(M, N, K, allow_split && slab != nullptr, 512);
  Epi epi{C, ldc, c_f32 ? 1 : 0, bias, bias_f32 ? 1 : 0, relu ? 1 : 0, nullptr};
  auto mk_ak = [&](auto t) { t.p = A; t.rows = M; t.K = K; t.ld = lda; return t; };
  auto mk_amn = [&](auto t) { t.p = A; t.K = K; t.cols = M; t.ld = lda; return t; };
  auto mk_bk = [&](auto t) { t.p = B; t.rows = N; t.K = K; t.ld = ldb; return t; };
  auto mk_bmn = [&](auto t) { t.p = B; t.K = K; t.cols = N; t.ld = ldb; return t; };
  if (a_kmajor && b_kmajor) return dispatch_bn<PlainK, PlainK>(M, N, K, p, epi, slab, st, mk_ak, mk_bk);
  if (a_kmajor) return dispatch_bn<PlainK, PlainMN>(M, N, K, p, epi, slab, st, mk_ak, mk_bmn);
  if (b_kmajor) return dispatch_bn<PlainMN, PlainK>(M, N, K, p, epi, slab, st, mk_amn, mk_bk);
  return dispatch_bn<PlainMN, PlainMN>(M, N, K, p, epi, slab, st, mk_amn, mk_bmn);
}

// db[i] = sum over the split-K launches' row sums src[s][i]
__global__ void __launch_bounds__(256) rowsum_cast_kernel(const float* __restrict__ src, void* dst, int bf16_out,
                                                          int64_t n, int splits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += src[(int64_t)s * n + i];
  if (bf16_out) ((bf16_t*)dst)[i] = f2bf(v);
  else ((float*)dst)[i] = v;
}

// Weight gradient with the bias gradient folded in: dw[M, N] = dy^T x with dy [K, M] and x
// [K, N] (both MN-major, K = tokens), and db[M] = column sums of dy = row sums of the A operand, computed
// by the pipelined kernel's extra MFMAs when the GEMM takes the 256 x 256 path (*db_done = 1); otherwise
// *db_done = 0 and only dw is written.  Split-K launches store their partial sums at `rs_scratch`
// [split][M] (sized by the caller for the slab's split count; no zeroing pass) and a pass sums them
// into db.
hipError_t gemm_bf16_wgrad_db(const bf16_t* dy, int64_t ld_dy, const bf16_t* x, int64_t ld_x, void* dw, bool dw_f32,
                              int64_t ldc, int64_t M, int64_t N, int64_t K, void* db, bool db_bf16, float* slab,
                              float* rs_scratch, hipStream_t st, int* db_done) {
  *db_done = 0;
  Plan p = plan_gemm(M, N, K, slab != nullptr, 512);
  Epi epi{dw, ldc, dw_f32 ? 1 : 0, nullptr, 0, 0, nullptr};
  auto mk_amn = [&](auto t) { t.p = dy; t.K = K; t.cols = M; t.ld = ld_dy; return t; };
  auto mk_bmn = [&](auto t) { t.p = x; t.K = K; t.cols = N; t.ld = ld_x; return t; };
  if (pp_mode()) {
    int ws = 0;
    if (use_wide(M, N, K, p, epi)) ws = 1;
    else if (slab) ws = wide_splits(M, N, K, p, epi);
    if (ws > 0) {
      Epi e = epi;
      static const bool fused_cast = [] {  // PDA_ROWSUM_FUSED=0: the separate rowsum_cast launch (A/B)
        const char* v = getenv("PDA_ROWSUM_FUSED");
        return !(v && v[0] == '0');
      }();
      if (ws > 1) {
        e.rowsum = rs_scratch;
        e.rowsum_mode = 4;
        if (fused_cast) {
          e.rowsum_out = db;
          e.rowsum_out_bf16 = db_bf16 ? 1 : 0;
        }
      } else {
        e.rowsum = db;
        e.rowsum_mode = db_bf16 ? 2 : 1;
      }
      int used = 1;
      const hipError_t r =
          launch_pp_plain(mk_amn(PlainMN<64>{}), mk_bmn(PlainMN<64>{}), M, N, K, e, st, ws, slab, &used);
      if (r != hipErrorNotSupported) {
        if (r != hipSuccess) return r;
        if (ws > 1 && (!e.rowsum_out || used <= 1)) {  // (used == 1: no reduce launch carried the sums)
          rowsum_cast_kernel<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(rs_scratch, db, db_bf16 ? 1 : 0, M,
                                                                          used);
          PDA_CHECK_HIP(hipGetLastError());
        }
        *db_done = 1;
        return hipSuccess;
      }
    }
  }
  return dispatch_bn<PlainMN, PlainMN>(M, N, K, p, epi, slab, st, mk_amn, mk_bmn);
}

// gemm_bf16 with a fused GELU epilogue (Epi::act): bf16 C, no split-K (the activation lives in the
// staged epilogues of the 128 / 256x128 / 256x256 tiles, not in splitk_reduce_kernel).
hipError_t gemm_bf16_act(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                         bf16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias, bool bias_f32,
                         int act, bf16_t* act_aux, hipStream_t st) {
  if ((act != 1 && act != 2) || !act_aux || N % 8 || ldc % 8) return hipErrorInvalidValue;
  Plan p = plan_gemm(M, N, K, false, 512);
  Epi epi{C, ldc, 0, bias, bias_f32 ? 1 : 0, 0, nullptr};
  epi.act = act;
  epi.act_aux = act_aux;
  auto mk_ak = [&](auto t) { t.p = A; t.rows = M; t.K = K; t.ld = lda; return t; };
  auto mk_amn = [&](auto t) { t.p = A; t.K = K; t.cols = M; t.ld = lda; return t; };
  auto mk_bk = [&](auto t) { t.p = B; t.rows = N; t.K = K; t.ld = ldb; return t; };
  auto mk_bmn = [&](auto t) { t.p = B; t.K = K; t.cols = N; t.ld = ldb; return t; };
  if (a_kmajor && b_kmajor) return dispatch_bn<PlainK, PlainK>(M, N, K, p, epi, nullptr, st, mk_ak, mk_bk);
  if (a_kmajor) return dispatch_bn<PlainK, PlainMN>(M, N, K, p, epi, nullptr, st, mk_ak, mk_bmn);
  if (b_kmajor) return dispatch_bn<PlainMN, PlainK>(M, N, K, p, epi, nullptr, st, mk_amn, mk_bk);
  return dispatch_bn<PlainMN, PlainMN>(M, N, K, p, epi, nullptr, st, mk_amn, mk_bmn);
}



// 3x3 halo path (conv3x3_halo_kernel): a 3x3 / pad-1 / stride-1 / dil-1 conv whose source has
// channels % 64 == 0 and whose band (rows spanned by 128 consecutive output pixels + 2 halo rows, full
// width) fits in LDS beside the two weight stages at two workgroups per CU.  PDA_CONV_HALO=0 disables it.
constexpr int kHaloLdsCap = 80 * 1024;

int halo_band_px(int H, int W) {
  // 128 consecutive pixels span at most ceil(127 / W) + 1 rows; + 1 halo row each side; + 1 zero pixel
  // (the target of taps outside the image); rounded up to the 32 pixels of one loader round
  const int rows = (127 + W - 1) / W + 1 + 2;
  return (rows * W + 1 + 31) / 32 * 32;
}

bool halo_mode_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_HALO");
    return !(e && e[0] == '0');
  }();
  return on;
}

int halo_lds_bytes(int H, int W, int BN) {
  int b = halo_band_px(H, W) * 128 + halo_stages(BN) * BN * BK * 2;
  const int epi_b = 128 * (BN + 8) * 2 + (NT / 64) * BN * 2 * 4;
  return b > epi_b ? b : epi_b;
}

bool use_halo(int H, int W, int Cg, int Nout, int R, int S, int stride, int pad, int dil, const Epi& epi) {
  if (!halo_mode_on() || R != 3 || S != 3 || stride != 1 || pad != 1 || dil != 1) return false;
  // 128-channel outputs only (measured, bench_conv bs 512, same box): 28^2 128->128 fwd 158 -> 144 us,
  // dgrad 162 -> 147 us.  At Nout >= 256 the 256x256 implicit-GEMM tile streams as many weight bytes
  // per FLOP as a 128-channel halo tile and ties it (14^2 256, 7^2 512: +-2 %); at Nout = 64 (56^2
  // 64->64) the 77-KB band + 4-stage workgroup fits 2 per CU against the 128x64 implicit-GEMM tile's
  // 3, and the layer is latency- rather than L2-bound there: +6 %.
  if (Cg % 64 || Nout != 128 || epi.c_f32 || epi.slab || epi.rm_on) return false;
  return halo_lds_bytes(H, W, 128) <= kHaloLdsCap;
}

template <int BN>
hipError_t launch_halo_bn(const bf16_t* src, const bf16_t* B, int Nimg, int H, int W, int Cg, int Nout, bool flip,
                          const Epi& epi, hipStream_t st) {
  const int lds = halo_lds_bytes(H, W, BN);
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_halo_kernel<BN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kHaloLdsCap);
    return true;
  }();
  (void)attr;
  HaloGeom hg;
  hg.H = H; hg.W = W; hg.Cg = Cg;
  hg.fW = make_fastdiv((uint32_t)W);
  hg.fH = make_fastdiv((uint32_t)H);
  hg.band_px = halo_band_px(H, W);
  hg.flip = flip ? 1 : 0;
  const int64_t M = (int64_t)Nimg * H * W, K = 9LL * Cg;
  PlainK<BN> lb;
  lb.p = B; lb.rows = Nout; lb.K = K; lb.ld = K;
  const int tiles_n = (Nout + BN - 1) / BN;
  const int tiles = (int)((M + 127) / 128) * tiles_n;
  conv3x3_halo_kernel<BN><<<tiles, NT, lds, st>>>(src, hg, lb, M, Nout, tiles_n, epi);
  return hipGetLastError();
}

// PDA_CONV_RES64=0: the 64 -> 64 channel 3x3 convs stay on the implicit GEMM (A/B)
bool res64_mode_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_RES64");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool use_res64(int H, int W, int Cg, int Nout, int R, int S, int stride, int pad, int dil, const Epi& epi) {
  if (!res64_mode_on() || R != 3 || S != 3 || stride != 1 || pad != 1 || dil != 1) return false;
  if (Cg != 64 || Nout != 64 || W != R64_QW || H % 4 != 0) return false;
  if (epi.slab || epi.c_f32 || epi.act || epi.rm_on) return false;
  return true;
}

hipError_t launch_res64(const bf16_t* src, const bf16_t* B, int Nimg, int H, int W, bool flip, const Epi& epi,
                        hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_res64_kernel<0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, R64_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_res64_kernel<1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, R64_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_res64_kernel<2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, R64_LDS);
    return true;
  }();
  (void)attr;
  (void)W;
  const int64_t M = (int64_t)Nimg * H * R64_QW;
  const int ntiles = Nimg * H / 4;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = ntiles < cus ? ntiles : cus;
  if (!epi.bst_z) conv3x3_res64_kernel<0><<<grid, NT, R64_LDS, st>>>(src, B, H, flip ? 1 : 0, M, ntiles, epi);
  else if (epi.addend || epi.bst_bits || epi.bst_z2)
    conv3x3_res64_kernel<1><<<grid, NT, R64_LDS, st>>>(src, B, H, flip ? 1 : 0, M, ntiles, epi);
  else conv3x3_res64_kernel<2><<<grid, NT, R64_LDS, st>>>(src, B, H, flip ? 1 : 0, M, ntiles, epi);
  return hipGetLastError();
}

hipError_t launch_halo(const bf16_t* src, const bf16_t* B, int Nimg, int H, int W, int Cg, int Nout, bool flip,
                       const Epi& epi, hipStream_t st) {
  return launch_halo_bn<128>(src, B, Nimg, H, W, Cg, Nout, flip, epi, st);
}

// PDA_WGRAD_PP_MIN_COUT: smallest Cout whose gathered weight gradient takes the pipelined tile (0: off)
int wgrad_pp_min_cout() {
  static const int v = [] {
    const char* e = getenv("PDA_WGRAD_PP_MIN_COUT");
    // off by default: 1.4-1.9x slower than the wide kernel's gather on every shape (the MN x MN gather
    // tile spills its LDS-read addresses inside the K loop; profiles/r4_wgrad_pp_gather_DROPPED.jsonl)
    const int x = e ? atoi(e) : 0;
    return x <= 0 ? (1 << 30) : x;
  }();
  return v;
}

// 3x3 all-taps weight gradient (conv3x3_wgrad_kernel): stride 1, pad 1, dil 1, C and Cout multiples of
// 64, W <= 64.  PDA_CONV_WG3=0 disables it.
bool wg3_mode_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_WG3");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool wg3_geom(int N, int H, int W, int C, int Cout, int R, int S, int stride, int pad, int dil, Wg3Geom& g) {
  if (!wg3_mode_on() || R != 3 || S != 3 || stride != 1 || pad != 1 || dil != 1) return false;
  // W >= 28 (the 56^2 and 28^2 layers: wgrad 367 -> 209 us and 233 -> 188 us at bs 512, bench_conv);
  // at 14^2 / 7^2 (4-7 rows per K-step, 16-64 output blocks re-reading each band) the implicit GEMM's
  // 256x256 split-K tile measured 7 % faster
  if (C % 64 || Cout % 64 || W > 64 || W < 28 || H < 1) return false;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Cout = Cout;
  g.rk = 64 / W;
  if (g.rk > H) g.rk = H;
  g.gpi = (H + g.rk - 1) / g.rk;
  g.groups = N * g.gpi;
  g.band_px = ((g.rk + 2) * (W + 2) + 31) / 32 * 32;
  g.fW2 = make_fastdiv((uint32_t)(W + 2));
  g.tiles_ci = C / 64;
  const int tiles = (Cout / 64) * g.tiles_ci;
  // ~512 workgroups (2 per CU), >= 4 row groups each, fp32 partial slabs capped at 96 MB
  int splits = 2 * wg3_wgrad_cus() / tiles;
  if (splits < 1) splits = 1;
  if (splits > g.groups / 4) splits = g.groups / 4 > 1 ? g.groups / 4 : 1;
  const int64_t per = (int64_t)Cout * 9 * C;
  const int64_t cap = ((int64_t)96 << 20) / (per * 4);
  if (splits > cap) splits = cap > 1 ? (int)cap : 1;
  g.gps = (g.groups + splits - 1) / splits;
  return 64 * BK * 2 + g.band_px * 128 <= WG3_STAGE;  // two stages, two workgroups per CU
}

int wg3_splits(const Wg3Geom& g) { return (g.groups + g.gps - 1) / g.gps; }

// conv3x3_wg_kernel (v2): every 3x3 / pad 1 / dil 1 layer with stride 1 or 2, C and Cout multiples of 64.
// PDA_CONV_WG3V2=0 keeps the round-4 kernels.
bool wg3v2_mode_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_WG3V2");
    return !(e && e[0] == '0');
  }();
  return on;
}

int wg3v2_co_tile(int Cout) { return Cout % 128 == 0 ? 128 : 64; }

bool wg3v2_geom(int N, int H, int W, int C, int Cout, int R, int S, int P, int Q, int stride, int pad, int dil,
                Wg3v2Geom& g) {
  if (!wg3v2_mode_on() || R != 3 || S != 3 || pad != 1 || dil != 1 || (stride != 1 && stride != 2)) return false;
  // Q >= 14: at 7-pixel output rows (7^2, and 14^2 -> 7^2 strided) a 49-pixel row group wastes 23 % of its
  // two halves and the implicit GEMM's split-K 256 x 256 tile measured 9 % faster
  // (profiles/r5_conv_wgrad_v2_table.jsonl)
  if (C % 64 || Cout % 64 || Q > 128 || Q < 14 || H < 1 || W < 1) return false;
  if (P != (H - 1) / stride + 1 || Q != (W - 1) / stride + 1) return false;
  // rows per K-step: the fewest 32-pixel halves per image among the rk whose dy (<= 128 px) and band
  // (<= 320 px) fit a stage; every step runs NH = ceil(rk Q / 32) halves (even for the 64-channel tile,
  // whose two wave groups take alternate halves)
  int w2p = 16;
  while (w2p < W + 2) w2p *= 2;
  if (w2p > 128) return false;
  int best = 0, best_halves = 1 << 30;
  for (int rk = 1; rk <= P && rk * Q <= 128; ++rk) {
    const int brows = (rk - 1) * stride + 3;
    if (brows * w2p > 320) break;
    const int full = P / rk, rem = P - full * rk;
    const int halves = full * ((rk * Q + 31) / 32) + (rem ? (rem * Q + 31) / 32 : 0);
    if (halves < best_halves || (halves == best_halves && rk > best)) {
      best_halves = halves;
      best = rk;
    }
  }
  if (best == 0) return false;
  g.N = N; g.H = H; g.W = W; g.P = P; g.Q = Q; g.C = C; g.Cout = Cout; g.st = stride;
  g.rk = best;
  g.gpi = (P + g.rk - 1) / g.rk;
  g.groups = N * g.gpi;
  g.band_rows = (g.rk - 1) * stride + 3;
  g.w2l = w2p == 16 ? 4 : (w2p == 32 ? 5 : (w2p == 64 ? 6 : 7));
  g.tiles_ci = C / 64;
  g.tiles_co = Cout / wg3v2_co_tile(Cout);
  g.fQ = make_fastdiv((uint32_t)Q);
  // one workgroup per CU: ~wgrad_cus() workgroups, >= 4 row groups each, fp32 slabs capped at 96 MB
  const int tiles = g.tiles_co * g.tiles_ci;
  const int per_split_slabs = wg3v2_co_tile(Cout) == 64 ? 2 : 1;
  int splits = wg3_wgrad_cus() / tiles;
  if (splits < 1) splits = 1;
  if (splits > g.groups / 4) splits = g.groups / 4 > 1 ? g.groups / 4 : 1;
  const int64_t per = (int64_t)Cout * 9 * C * per_split_slabs;
  const int64_t cap = ((int64_t)96 << 20) / (per * 4);
  if (splits > cap) splits = cap > 1 ? (int)cap : 1;
  g.gps = (g.groups + splits - 1) / splits;
  return true;
}

// slabs written by a v2 launch (the 64-channel tile's two pixel-half parities each write their own)
int wg3v2_slabs(const Wg3v2Geom& g) {
  const int splits = (g.groups + g.gps - 1) / g.gps;
  return wg3v2_co_tile(g.Cout) == 64 ? 2 * splits : splits;
}

// stem weight-gradient path (conv_stem_wgrad_kernel): 4x4 / stride 1 / pad 0 / dil 1 over 16 channels,
// Cout % 64 == 0, output rows of <= 128 pixels.  PDA_CONV_STEM_WG=0 disables it.
bool stem_wg_mode_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_STEM_WG");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool stem_geom(int N, int H, int W, int C, int Cout, int R, int S, int P, int Q, int stride, int pad, int dil,
               StemGeom& g) {
  if (!stem_wg_mode_on() || C != 16 || R != 4 || S != 4 || stride != 1 || pad != 0 || dil != 1) return false;
  if (Cout % 64 || Q > 128 || Q < 1 || P != H - 3 || Q != W - 3 || N < 1) return false;
  g.N = N; g.H = H; g.W = W; g.P = P; g.Q = Q; g.Cout = Cout;
  g.rows = N * P;
  // the last lane's tap read reaches band pixel 127 + 3 + 4 + 3 W; the band is always 4 DMA rounds of
  // 128 pixels (8 DMAs per row and thread: the counted waits assume it)
  const int need = 4 * W > 135 + 3 * W ? 4 * W : 135 + 3 * W;
  g.band_px = 512;
  if (need > g.band_px) return false;
  // two workgroups per CU over the whole chip: the stem's weight gradient is the last kernel of the
  // backward (nothing on the compute stream to leave CUs for)
  const int tiles = Cout / 64;
  int splits = 512 / tiles;
  if (splits < 1) splits = 1;
  if (splits > g.rows / 4) splits = g.rows / 4 > 1 ? g.rows / 4 : 1;
  const int64_t cap = ((int64_t)96 << 20) / ((int64_t)Cout * 256 * 4);
  if (splits > cap) splits = cap > 1 ? (int)cap : 1;
  g.rps = (g.rows + splits - 1) / splits;
  return true;
}

int stem_splits(const StemGeom& g) { return (g.rows + g.rps - 1) / g.rps; }

// stem forward path (conv_stem_fwd_kernel): the stem_geom shapes with Cout == 64 and a bf16 output.
// PDA_CONV_STEM_FWD=0 disables it.
bool stem_fwd_on(int Cout, bool y_f32, const StemGeom& g) {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_STEM_FWD");
    return !(e && e[0] == '0');
  }();
  return on && Cout == 64 && !y_f32 && g.Q <= 128;
}

// dgrad phases without taps as a fill kernel (dgrad_fill_phase_kernel).  PDA_DGRAD_FILL_PHASE=0 keeps
// the K = 0 GEMM launches.
bool fill_phase_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_DGRAD_FILL_PHASE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// ConvFwdKU / ConvDgradPhaseKU (tap-uniform K tiles) for 64-multiple gathered channel counts.
// PDA_CONV_TAP_UNIFORM=0 keeps ConvFwdK / ConvDgradPhaseK.
bool tap_uniform_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_TAP_UNIFORM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// 1x1 / stride-1 / pad-0 convs are plain GEMMs in NHWC: fwd and wgrad read x through the plain loaders
// (PlainK / PlainMN: a pointer add per row) instead of the im2col gathers (ConvFwdK / ConvWgradMN: two
// fast divisions, bounds checks and 64-bit offsets per 16-B chunk — VALU work that competes with the
// MFMA issue of the co-resident wave).  PDA_CONV_1X1_PLAIN=0 keeps the gathers.
bool conv_1x1_plain(int R, int S, int stride, int pad, int dil) {
  static const bool on = [] {
    const char* e = getenv("PDA_CONV_1X1_PLAIN");
    return !(e && e[0] == '0');
  }();
  return on && R == 1 && S == 1 && stride == 1 && pad == 0 && dil == 1;
}

// y[N,P,Q,Cout] = conv(x[N,H,W,C], w[Cout,R,S,C]) (+bias, relu)
hipError_t conv2d_fwd(const bf16_t* x, const bf16_t* w, void* y, bool y_f32, int N, int H, int W, int C, int Cout,
                      int R, int S, int P, int Q, int stride, int pad, int dil, const void* bias, bool bias_f32,
                      bool relu, float* stats, const float* stats_shift, int stats_rows, hipStream_t st) {
  const int64_t M = (int64_t)N * P * Q, Nn = Cout, K = (int64_t)R * S * C;
  if (y_f32 && stats) return hipErrorInvalidValue;  // epilogue statistics are a bf16-output feature
  Plan p = plan_gemm(M, Nn, K, false, 512);
  Epi epi{y, Cout, y_f32 ? 1 : 0, bias, bias_f32 ? 1 : 0, relu ? 1 : 0, nullptr};
  epi.stats = stats;
  epi.stats_shift = stats_shift;
  epi.stats_rows = stats_rows > 0 ? stats_rows : 1;

  if (use_res64(H, W, C, Cout, R, S, stride, pad, dil, epi)) return launch_res64(x, w, N, H, W, false, epi, st);
  if (use_halo(H, W, C, Cout, R, S, stride, pad, dil, epi)) return launch_halo(x, w, N, H, W, C, Cout, false, epi, st);
  StemGeom sg;
  if (stem_geom(N, H, W, C, Cout, R, S, P, Q, stride, pad, dil, sg) && stem_fwd_on(Cout, y_f32, sg)) {
    // two workgroups per CU, each walking a run of output rows; problems of <= 16 rows per table row
    // use at most R (= stats_rows) workgroups, so their BN sums are reproducible (one add per row)
    const int nb = (stats && sg.rows <= 16 * stats_rows) ? (stats_rows < 512 ? stats_rows : 512) : 512;
    sg.rps = (sg.rows + nb - 1) / nb;
    const int blocks = (sg.rows + sg.rps - 1) / sg.rps;
    conv_stem_fwd_kernel<<<blocks, NT, 0, st>>>(x, w, sg, epi);
    return hipGetLastError();
  }
  auto mk_b = [&](auto t) { t.p = w; t.rows = Nn; t.K = K; t.ld = K; return t; };
  if (conv_1x1_plain(R, S, stride, pad, dil)) {  // y[NHW, Cout] = x[NHW, C] w[Cout, C]^T
    // short K (the bottleneck expansions): the streaming kernel (HBM-bound shape, fwd_stream.hip)
    if (fwd_stream_ok(M, Nn, K, epi)) return fwd_stream(x, w, M, Nn, K, epi, st);
    auto mk_ap = [&](auto t) { t.p = x; t.rows = M; t.K = K; t.ld = C; return t; };
    return dispatch_bn<PlainK, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_ap, mk_b);
  }
  ConvGeom g = make_geom(H, W, C, P, Q, R, S, stride, pad, dil, C);
  auto mk_a = [&](auto t) { t.x = x; t.g = g; t.M = M; t.K = K; return t; };
  if (C % 64 == 0 && tap_uniform_on()) {
    // the 256 x 256 tile on the pipelined kernel (gathered A operand, gemm_pp.hip) where the wide tile
    // would be chosen; PDA_GEMM_PP=0 keeps the 2-stage wide kernel
    if (pp_mode() && pp_conv_mode() && use_wide(M, Nn, K, p, epi)) {
      const hipError_t r = gemm_pp_gather(x, N, H, W, C, P, Q, S, (int)K, stride, -pad, -pad, dil, dil, w, Cout, epi,
                                          st);
      if (r != hipErrorInvalidValue) return r;
    }
    return dispatch_bn<ConvFwdKU, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_b);
  }
  return dispatch_bn<ConvFwdK, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_b);
}

// dx[N,H,W,C] = dgrad(dy[N,P,Q,Cout], wt): one launch per stride phase with only the taps that reach
// it (wt phase-packed by conv_weight_transpose); folded single launch when stride > 1 and dil > 1.
bool conv_dgrad_needs_wt(int R, int S, int stride, int pad) { return !(R == 1 && S == 1 && stride == 1 && pad == 0); }

// 1x1 stride-1 dgrad on a transposed weight wt[C][Cout] (K-major B operand) instead of reading w
// [Cout][C] MN-major in place: the wide tile's K-major x K-major schedule avoids the two
// ds_read_b64_tr_b16 per B fragment (plain GEMMs: dgrad layout 0.72-0.86x the fwd layout,
// profiles/r3_wide_ring_DROPPED.jsonl two_stage arm).  Only where the GEMM is MFMA-heavy (C, Cout >= 256);
// the transpose is one small launch.  PDA_DGRAD_1X1_WT=0 keeps the in-place read.
bool conv_dgrad_1x1_wt(int R, int S, int stride, int pad, int C, int Cout) {
  static const bool on = [] {
    const char* e = getenv("PDA_DGRAD_1X1_WT");
    return !(e && e[0] == '0');
  }();
  return on && R == 1 && S == 1 && stride == 1 && pad == 0 && C >= 256 && Cout >= 256;
}

hipError_t conv2d_dgrad(const bf16_t* dy, const bf16_t* w, const bf16_t* wt, void* dx, bool dx_f32, int N, int H, int W,
                        int C, int Cout, int R, int S, int P, int Q, int stride, int pad, int dil, const bf16_t* addend,
                        const uint8_t* addend_bits, hipStream_t st, const BnBwdStats* bst) {
  const int cf = dx_f32 ? 1 : 0;
  // (a strided dgrad's fill-phase kernel writes the addend where no tap reaches: those elements would be
  // missing from the sums, so the statistics take an addend only at stride 1)
  if (bst && (dx_f32 || (addend && stride > 1) || !bst->z || !bst->mean || !bst->table || bst->rows < 1 ||
              (!bst->ss && !bst->bits) || (bst->z2 && (!bst->mean2 || !bst->table2))))
    return hipErrorInvalidValue;
  // every Epi below starts from this one: bf16 dx, the optional addend and the optional BN-backward sums
  auto base_epi = [&]() {
    Epi e{dx, C, cf, nullptr, 0, 0, nullptr};
    e.addend = addend;
    e.addend_bits = addend_bits;
    if (bst) {
      e.stats = bst->table;
      e.stats_shift = bst->mean;
      e.stats_rows = bst->rows;
      e.bst_z = bst->z;
      e.bst_ss = bst->ss;
      e.bst_bits = bst->bits;
      e.bst_z2 = bst->z2;
      e.bst_mean2 = bst->mean2;
      e.bst_table2 = bst->table2;
    }
    return e;
  };
  if (!conv_dgrad_needs_wt(R, S, stride, pad)) {
    // 1x1 stride 1: dx[NHW, C] = dy[NHW, Cout] * w[Cout, C] — dy rows are the K-major A operand and the
    // OHWI weight is already the MN-major B operand (k = co rows of C contiguous channels): no weight
    // transpose launch (36 of ResNet-50's 53 convs are 1x1, 32 of them stride 1)
    const int64_t M = (int64_t)N * H * W, Nn = C, K = Cout;
    Plan p = plan_gemm(M, Nn, K, false, 512);
    Epi epi = base_epi();
    // short K (64 / 128) with BN-backward sums: the streaming kernel (HBM-bound shape, dgrad_stream.hip)
    if (dgrad_stream_ok(M, Nn, K, epi)) return dgrad_stream(dy, w, M, Nn, K, epi, st);
    auto mk_a = [&](auto t) { t.p = dy; t.rows = M; t.K = K; t.ld = Cout; return t; };
    if (wt) {  // conv_dgrad_1x1_wt: B(k = co, n = ci) = wt[ci][co], K-major
      auto mk_bt = [&](auto t) { t.p = wt; t.rows = Nn; t.K = K; t.ld = Cout; return t; };
      return dispatch_bn<PlainK, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_bt);
    }
    auto mk_b = [&](auto t) { t.p = w; t.K = K; t.cols = Nn; t.ld = C; return t; };
    return dispatch_bn<PlainK, PlainMN>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_b);
  }
  ConvGeom g = make_geom(H, W, C, P, Q, R, S, stride, pad, dil, Cout);
  if (!dgrad_phased(stride, dil)) {
    const int64_t M = (int64_t)N * H * W, Nn = C, K = (int64_t)R * S * Cout;
    Plan p = plan_gemm(M, Nn, K, false, 512);
    Epi epi = base_epi();
    auto mk_a = [&](auto t) { t.dy = dy; t.g = g; t.M = M; t.K = K; return t; };
    auto mk_b = [&](auto t) { t.p = wt; t.rows = Nn; t.K = K; t.ld = K; return t; };
    return dispatch_bn<ConvDgradK, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_b);
  }
  if (stride == 1) {
    // stride-1 dgrad = the 3x3 conv of dy with the rotated transposed weights (halo path)
    Epi epi = base_epi();
    if (use_res64(H, W, Cout, C, R, S, stride, pad, dil, epi)) return launch_res64(dy, wt, N, H, W, true, epi, st);
    if (use_halo(H, W, Cout, C, R, S, stride, pad, dil, epi)) return launch_halo(dy, wt, N, H, W, Cout, C, true, epi, st);
  }
  const int nph = stride;  // phases per dim (1 for stride 1)
  for (int ph = 0; ph < nph; ++ph) {
    const TapPhase a = tap_phase(ph, R, stride, pad, dil);
    const int Hh = stride == 1 ? H : (H - ph + stride - 1) / stride;
    for (int pw = 0; pw < nph; ++pw) {
      const TapPhase b = tap_phase(pw, S, stride, pad, dil);
      const int Wh = stride == 1 ? W : (W - pw + stride - 1) / stride;
      if (Hh <= 0 || Wh <= 0) continue;
      PhaseGeom pg;
      pg.Hh = Hh; pg.Wh = Wh; pg.Sv = b.n > 0 ? b.n : 1;
      pg.base_r = a.base; pg.step_r = stride == 1 ? dil : 1;
      pg.base_s = b.base; pg.step_s = stride == 1 ? dil : 1;
      pg.fWh = make_fastdiv((uint32_t)Wh);
      pg.fHh = make_fastdiv((uint32_t)Hh);
      pg.fSv = make_fastdiv((uint32_t)pg.Sv);
      const int64_t M = (int64_t)N * Hh * Wh, Nn = C, K = (int64_t)a.n * b.n * Cout;
      if (K == 0 && fill_phase_on() && M * (C / 8) < ((int64_t)1 << 31) && C % 8 == 0) {
        const int64_t total = M * (C / 8);
        const int64_t blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
        dgrad_fill_phase_kernel<<<(unsigned)blocks, 256, 0, st>>>(
            dx, cf, addend, addend_bits, total, make_fastdiv((uint32_t)(C / 8)), make_fastdiv((uint32_t)Wh),
            make_fastdiv((uint32_t)Hh), H, W, C, stride, ph, pw);
        PDA_CHECK_HIP(hipGetLastError());
        continue;
      }
      const bf16_t* wph = wt + ((int64_t)a.cum * S + (int64_t)a.n * b.cum) * C * Cout;
      Plan p = plan_gemm(M, Nn, K, false, 512);
      Epi epi = base_epi();
      if (stride > 1) {
        if (M >= ((int64_t)1 << 32)) return hipErrorInvalidValue;  // epi_row's 32-bit row remap
        epi.rm_on = 1; epi.rm_Hh = Hh; epi.rm_Wh = Wh; epi.rm_st = stride; epi.rm_ph = ph; epi.rm_pw = pw;
        epi.rm_H = H; epi.rm_W = W;
      }
      auto mk_a = [&](auto t) { t.dy = dy; t.g = g; t.ph = pg; t.M = M; t.K = K; return t; };
      auto mk_b = [&](auto t) { t.p = wph; t.rows = Nn; t.K = K; t.ld = K > 0 ? K : 8; return t; };
      if (R == 1 && S == 1 && pad == 0 && Hh == P && Wh == Q && a.n * b.n == 1 && a.base == 0 && b.base == 0 &&
          conv_1x1_plain(1, 1, 1, 0, 1)) {
        // a strided 1x1 conv's one live phase: dx pixel (hh*st, ww*st) = dy[hh, ww] W, i.e. dy read as the
        // plain K-major [N*P*Q][Cout] operand (no gather), rows remapped by the epilogue
        auto mk_ap = [&](auto t) { t.p = dy; t.rows = M; t.K = K; t.ld = Cout; return t; };
        const hipError_t e = dispatch_bn<PlainK, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_ap, mk_b);
        if (e != hipSuccess) return e;
        continue;
      }
      const bool ku = Cout % 64 == 0 && R * S > 1 && tap_uniform_on();  // (strided 1x1: +3 %, kept gathered)
      if (ku && pp_mode() && pp_conv_mode() && use_wide(M, Nn, K, p, epi)) {
        // the phase's gather on the pipelined tile: dy pixel (hh + base_r - ri*step_r, ww + ...)
        const hipError_t r = gemm_pp_gather(dy, N, P, Q, Cout, Hh, Wh, pg.Sv, (int)K, 1, pg.base_r, pg.base_s,
                                            -pg.step_r, -pg.step_s, wph, C, epi, st);
        if (r != hipErrorInvalidValue) {
          if (r != hipSuccess) return r;
          continue;
        }
      }
      const hipError_t e = ku ? dispatch_bn<ConvDgradPhaseKU, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_b)
                              : dispatch_bn<ConvDgradPhaseK, PlainK>(M, Nn, K, p, epi, nullptr, st, mk_a, mk_b);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

int64_t conv_slab_floats(int mode, int N, int H, int W, int C, int Cout, int R, int S, int P, int Q) {
  if (mode != 2) return 0;  // only wgrad splits K
  const int64_t M = Cout, Nn = (int64_t)R * S * C, K = (int64_t)N * P * Q;
  int64_t n = split_slab_floats(M, Nn, K, plan_wgrad(M, Nn, K, true));
  Wg3Geom g;
  if (P == H && Q == W && wg3_geom(N, H, W, C, Cout, R, S, 1, 1, 1, g)) {
    const int64_t w3 = (int64_t)wg3_splits(g) * M * Nn;
    if (w3 > n) n = w3;
  }
  StemGeom sg;
  if (stem_geom(N, H, W, C, Cout, R, S, P, Q, 1, 0, 1, sg)) {
    const int64_t ws = (int64_t)stem_splits(sg) * M * Nn;
    if (ws > n) n = ws;
  }
  Wg3v2Geom gv;
  for (int sv = 1; sv <= 2; ++sv) {  // (the stride is not an argument: wg3v2_geom accepts at most one)
    if (wg3v2_geom(N, H, W, C, Cout, R, S, P, Q, sv, 1, 1, gv)) {
      const int64_t wv = (int64_t)wg3v2_slabs(gv) * M * Nn;
      if (wv > n) n = wv;
    }
  }
  return n;
}

// dw[Cout, R*S*C] = dy[NPQ, Cout]^T * im2col(x)[NPQ, R*S*C]   (fp32 or bf16 output)
hipError_t conv2d_wgrad(const bf16_t* dy, const bf16_t* x, void* dw, bool dw_f32, int N, int H, int W, int C,
                        int Cout, int R, int S, int P, int Q, int stride, int pad, int dil, float* slab,
                        hipStream_t st) {
  const int64_t M = Cout, Nn = (int64_t)R * S * C, K = (int64_t)N * P * Q;
  Epi epi{dw, Nn, dw_f32 ? 1 : 0, nullptr, 0, 0, nullptr};
  Wg3v2Geom gv;
  if (slab && wg3v2_geom(N, H, W, C, Cout, R, S, P, Q, stride, pad, dil, gv)) {
    const int splits = (gv.groups + gv.gps - 1) / gv.gps;
    const dim3 grid(gv.tiles_co * gv.tiles_ci, splits);
#define WG3V2_LAUNCH(CO)                                                                        \
  do {                                                                                          \
    if (gv.w2l == 4) conv3x3_wg_kernel<CO, 4><<<grid, WG3V2_NT, 0, st>>>(dy, x, gv, slab);      \
    else if (gv.w2l == 5) conv3x3_wg_kernel<CO, 5><<<grid, WG3V2_NT, 0, st>>>(dy, x, gv, slab); \
    else if (gv.w2l == 6) conv3x3_wg_kernel<CO, 6><<<grid, WG3V2_NT, 0, st>>>(dy, x, gv, slab); \
    else conv3x3_wg_kernel<CO, 7><<<grid, WG3V2_NT, 0, st>>>(dy, x, gv, slab);                 \
  } while (0)
    if (wg3v2_co_tile(Cout) == 128) WG3V2_LAUNCH(128);
    else WG3V2_LAUNCH(64);
#undef WG3V2_LAUNCH
    PDA_CHECK_HIP(hipGetLastError());
    const int slabs = wg3v2_slabs(gv);
    int ll = 0;
    while (ll < 4 && (slabs >> ll) > 16) ++ll;
    const int64_t per_block = 256 >> ll;
    const int64_t gr = (M * Nn / 4 + per_block - 1) / per_block;
    splitk_reduce_kernel<<<(unsigned)gr, 256, 0, st>>>(slab, slabs, M, Nn, ll, epi);
    return hipGetLastError();
  }
  Wg3Geom g3;
  if (slab && P == H && Q == W && wg3_geom(N, H, W, C, Cout, R, S, stride, pad, dil, g3)) {
    const int splits = wg3_splits(g3);
    conv3x3_wgrad_kernel<<<dim3((Cout / 64) * g3.tiles_ci, splits), NT, 0, st>>>(dy, x, g3, slab);
    PDA_CHECK_HIP(hipGetLastError());
    int ll = 0;
    while (ll < 4 && (splits >> ll) > 16) ++ll;
    const int64_t per_block = 256 >> ll;
    const int64_t gr = (M * Nn / 4 + per_block - 1) / per_block;
    splitk_reduce_kernel<<<(unsigned)gr, 256, 0, st>>>(slab, splits, M, Nn, ll, epi);
    return hipGetLastError();
  }
  StemGeom sg;
  if (slab && stem_geom(N, H, W, C, Cout, R, S, P, Q, stride, pad, dil, sg)) {
    const int splits = stem_splits(sg);
    conv_stem_wgrad_kernel<<<dim3(Cout / 64, splits), NT, 0, st>>>(dy, x, sg, slab);
    PDA_CHECK_HIP(hipGetLastError());
    int ll = 0;
    while (ll < 4 && (splits >> ll) > 16) ++ll;
    const int64_t per_block = 256 >> ll;
    const int64_t gr = (M * Nn / 4 + per_block - 1) / per_block;
    splitk_reduce_kernel<<<(unsigned)gr, 256, 0, st>>>(slab, splits, M, Nn, ll, epi);
    return hipGetLastError();
  }
  Plan p = plan_wgrad(M, Nn, K, slab != nullptr);
  // gathered convs with >= 256 output channels (a full 256-row tile): the pipelined tile with the
  // input gathered per k-row (gemm_pp.hip PPWg) instead of the 2-stage wide kernel's gather
  if (slab && pp_conv_mode() && wgrad_pp_min_cout() <= Cout && !conv_1x1_plain(R, S, stride, pad, dil)) {
    const int ws = wide_split_count(M, Nn, K);
    Epi e = epi;
    e.slab = slab;
    int used = 1;
    const hipError_t r = gemm_pp_wgrad(dy, x, N, H, W, C, Cout, R, S, P, Q, stride, pad, dil, e, ws, st, &used);
    if (r == hipSuccess) {
      if (used <= 1) return hipGetLastError();
      int ll = 0;
      while (ll < 4 && (used >> ll) > 16) ++ll;
      const int64_t per_block = 256 >> ll;
      const int64_t gr = (M * Nn / 4 + per_block - 1) / per_block;
      splitk_reduce_kernel<<<(unsigned)gr, 256, 0, st>>>(slab, used, M, Nn, ll, epi);
      return hipGetLastError();
    }
    if (r != hipErrorInvalidValue) return r;
  }
  auto mk_a = [&](auto t) { t.p = dy; t.K = K; t.cols = M; t.ld = Cout; return t; };
  if (conv_1x1_plain(R, S, stride, pad, dil)) {  // dw[Cout, C] = dy[NHW, Cout]^T x[NHW, C]
    auto mk_bp = [&](auto t) { t.p = x; t.K = K; t.cols = Nn; t.ld = C; return t; };
    return dispatch_bn<PlainMN, PlainMN>(M, Nn, K, p, epi, slab, st, mk_a, mk_bp);
  }
  ConvGeom g = make_geom(H, W, C, P, Q, R, S, stride, pad, dil, C);
  auto mk_b = [&](auto t) { t.x = x; t.g = g; t.K = K; t.cols = Nn; return t; };
  return dispatch_bn<PlainMN, ConvWgradMN>(M, Nn, K, p, epi, slab, st, mk_a, mk_b);
}

hipError_t conv_weight_transpose(const bf16_t* w, bf16_t* wt, int Cout, int R, int S, int Cin, int stride, int pad,
                                 int dil, hipStream_t st) {
  dim3 grid((Cin + 31) / 32, (Cout + 31) / 32, R * S);
  conv_wt_transpose_kernel<<<grid, 256, 0, st>>>(w, wt, Cout, R, S, Cin, stride, pad, dgrad_phased(stride, dil) ? 1 : 0);
  return hipGetLastError();
}

}  // namespace pda
