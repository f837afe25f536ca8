// Causal / non-causal flash attention, forward and backward, bf16 in / fp32 accumulate, GQA
// (GPT-2 d_head 64, 16/25 heads, T=1024; Llama-3 d_head 128, 32 Q / 8 KV heads).
//
// Layout: q/k/v are [B, T, H, D] with arbitrary batch / time / head strides (so the q, k, v slices of a
// fused QKV projection are consumed in place) and a contiguous head dim; outputs likewise.
//
// MFMA structure (v_mfma_f32_16x16x32_bf16, wave64; cdna_hip_programming.md §3 "accumulator tile as
// the next MFMA's operand"):
//  * S = Q K^T is computed with K as the A operand and Q as the B operand, so each lane ends up owning
//    ONE query row (lane & 15) and 4 consecutive keys per 16-key sub-tile: row max / sum need only two
//    cross-lane shuffles and the O rescale is a per-lane scalar.
//  * P (bf16) feeds P*V directly from registers as the B operand, with the key order inside each 32-key
//    k-step permuted to match the S layout; V is the A operand, read with ds_read_b64_tr_b16 (T10) from
//    an LDS image swizzled per 32-B slot so the 8 rows a half-wave reads hit distinct banks.
//  * K tiles for the row-wise reads use a 16-B-chunk XOR swizzle (T2) -> conflict-free ds_read_b128.
// Backward = FA2 with recomputation: at D = 64 one key-stationary kernel computes dK, dV and dQ from a
// single P / dS per tile (dQ through an fp32 atomic accumulator, attn_bwd_dkdv2_kernel<..., FQ>); at
// D = 128 a dQ kernel (query-stationary) plus the dK/dV kernel, no atomics.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

typedef __bf16 mbf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int NT = 256;
constexpr int BQ = 64, BKV = 64;
constexpr float LOG2E = 1.4426950408889634f;
// finite "minus infinity" for running maxima: exp2(c * (m_old - m_new)) stays exact when a row has
// seen only masked keys so far (no inf - inf, no per-element "dead row" select)
constexpr float NEG_BIG = -1e30f;

// v_exp_f32 directly (HIP's exp2f adds a denormal-range fix-up: ldexp + compare + select per call);
// every argument here is a max-shifted log2-domain score <= 0, where the bare instruction is exact
// enough and underflows to 0 as wanted.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Reductions across the lanes l ^ 16 and l ^ 32 (the 4 lanes that hold one query's keys in the S
// accumulator layout) with the CDNA4 permlane swaps: each returns {own, partner} in some order, so a
// max / sum of the pair is the butterfly step without an LDS round trip (ds_bpermute).
__device__ __forceinline__ float max_x16_x32(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float sum_x16_x32(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// ---------------------------------------------------------------- LDS images (rows of D bf16)
// row image (for ds_read_b128 of 8 consecutive columns of one row)
template <int D>
__device__ __forceinline__ int row_off(int row, int chunk) {
  if constexpr (D == 128) return row * 256 + ((chunk ^ (row & 15)) << 4);
  else return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);  // 128-B rows: key on row pairs (16-row reads)
}
// transposed-read image (for ds_read_b64_tr_b16 of 4 consecutive rows x 16 columns)
template <int D>
__device__ __forceinline__ int tr_off(int row, int col) {
  if constexpr (D == 128) return row * 256 + ((((col >> 4) ^ (row & 7)) & 7) << 5) + ((col & 15) << 1);
  else return row * 128 + ((((col >> 4) ^ ((row >> 1) & 3)) & 3) << 5) + ((col & 15) << 1);
}

__device__ __forceinline__ u16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const u16x8*>(p); }
__device__ __forceinline__ u16x8 zero16() {
  u16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = 0;
  return z;
}

// Stage a [64 rows][D] tile of X (rows row0.., row stride `rs` elements) into LDS images, optionally
// applying the rotary embedding of row position gr (rotate-half: pairs (d, d + D/2)).
template <int D, bool ROW, bool TR>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ X, int64_t rs, int row0, int T, char* row_img,
                                           char* tr_img, const float* __restrict__ rc = nullptr,
                                           const float* __restrict__ rsn = nullptr) {
  constexpr int CPR = D / 8;  // 16-B chunks per row
  if (rc == nullptr) {
#pragma unroll
    for (int i = 0; i < (64 * CPR) / NT; ++i) {
      const int c = threadIdx.x + NT * i;
      const int r = c / CPR, ch = c % CPR;
      const int gr = row0 + r;
      const u16x8 v = gr < T ? ld16(X + (int64_t)gr * rs + ch * 8) : zero16();
      if (ROW) *reinterpret_cast<u16x8*>(row_img + row_off<D>(r, ch)) = v;
      if (TR) *reinterpret_cast<u16x8*>(tr_img + tr_off<D>(r, ch * 8)) = v;
    }
    return;
  }
  constexpr int HALF = CPR / 2;
#pragma unroll
  for (int i = 0; i < (64 * HALF) / NT; ++i) {
    const int c = threadIdx.x + NT * i;
    const int r = c / HALF, ch = c % HALF;
    const int gr = row0 + r;
    u16x8 a = zero16(), b = zero16();
    if (gr < T) {
      a = ld16(X + (int64_t)gr * rs + ch * 8);
      b = ld16(X + (int64_t)gr * rs + (ch + HALF) * 8);
      const float* cr = rc + (int64_t)gr * (D / 2) + ch * 8;
      const float* sr = rsn + (int64_t)gr * (D / 2) + ch * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x1 = bf2f(a[j]), x2 = bf2f(b[j]);
        a[j] = f2bf(x1 * cr[j] - x2 * sr[j]);
        b[j] = f2bf(x2 * cr[j] + x1 * sr[j]);
      }
    }
    if (ROW) {
      *reinterpret_cast<u16x8*>(row_img + row_off<D>(r, ch)) = a;
      *reinterpret_cast<u16x8*>(row_img + row_off<D>(r, ch + HALF)) = b;
    }
    if (TR) {
      *reinterpret_cast<u16x8*>(tr_img + tr_off<D>(r, ch * 8)) = a;
      *reinterpret_cast<u16x8*>(tr_img + tr_off<D>(r, (ch + HALF) * 8)) = b;
    }
  }
}

// Rotate register fragments f[ks] / f[ks + KS/2] (columns 32 ks + 8 g + j) of sequence position `row`.
template <int KS, int D>
__device__ __forceinline__ void rope_frags(mbf16x8 (&f)[KS], const float* rc, const float* rsn, int row, int T,
                                           int lane) {
  if (rc == nullptr || row >= T) return;
  const int g = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < KS / 2; ++ks) {
    const int d = 32 * ks + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cs = rc[(int64_t)row * (D / 2) + d + j], sn = rsn[(int64_t)row * (D / 2) + d + j];
      const float x1 = (float)f[ks][j], x2 = (float)f[ks + KS / 2][j];
      f[ks][j] = (__bf16)(x1 * cs - x2 * sn);
      f[ks + KS / 2][j] = (__bf16)(x2 * cs + x1 * sn);
    }
  }
}

// Gradient w.r.t. the pre-rotation input for an accumulator pair acc[dt] / acc[dt + DT/2]
// (lane holds columns 16 dt + 4 g + r of sequence position `row`).
template <int DT, int D>
__device__ __forceinline__ void rope_grad_acc(f32x4 (&acc)[DT], const float* rc, const float* rsn, int row, int T,
                                              int lane) {
  if (rc == nullptr || row >= T) return;
  const int g = lane >> 4;
#pragma unroll
  for (int dt = 0; dt < DT / 2; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 16 * dt + 4 * g + r;
      const float cs = rc[(int64_t)row * (D / 2) + d], sn = rsn[(int64_t)row * (D / 2) + d];
      const float g1 = acc[dt][r], g2 = acc[dt + DT / 2][r];
      acc[dt][r] = g1 * cs + g2 * sn;
      acc[dt + DT / 2][r] = g2 * cs - g1 * sn;
    }
}

// A/B fragment from a row image: lane l -> row (row0 + (l & 15)), columns 32 ks + 8 (l >> 4) + j
template <int D>
__device__ __forceinline__ mbf16x8 frag_row(const char* img, int row0, int ks, int lane) {
  const int r = row0 + (lane & 15);
  return *reinterpret_cast<const mbf16x8*>(img + row_off<D>(r, ks * 4 + (lane >> 4)));
}

// A fragment via transposed reads: lane l -> column (col0 + (l & 15)) of rows
// {k0 + 4g + q} (elements 0..3) and {k0 + 16 + 4g + q} (elements 4..7), g = l >> 4, i.e. the key
// order produced by an S / dS accumulator pair (sub-tiles 2c, 2c+1) with k0 = 32 c.
template <int D>
__device__ __forceinline__ mbf16x8 frag_tr(const char* img, int k0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int row = k0 + 4 * g + (i >> 2);
  const int col = col0 + 4 * (i & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + tr_off<D>(row, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + tr_off<D>(row + 16, col)));
  s16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return __builtin_bit_cast(mbf16x8, f);
}

// Pack two S-layout accumulators (sub-tiles 2c, 2c+1) into a bf16 B/A fragment with permuted key order.
__device__ __forceinline__ mbf16x8 pack_p(const f32x4& a, const f32x4& b) {
  mbf16x8 f;
  f[0] = (__bf16)a[0]; f[1] = (__bf16)a[1]; f[2] = (__bf16)a[2]; f[3] = (__bf16)a[3];
  f[4] = (__bf16)b[0]; f[5] = (__bf16)b[1]; f[6] = (__bf16)b[2]; f[7] = (__bf16)b[3];
  return f;
}

__device__ __forceinline__ mbf16x8 load_frag_global(const bf16_t* base, int64_t rs, int row, int T, int ks,
                                                    int lane) {
  if (row >= T) {
    s16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = 0;
    return __builtin_bit_cast(mbf16x8, z);
  }
  return *reinterpret_cast<const mbf16x8*>(base + (int64_t)row * rs + 32 * ks + 8 * (lane >> 4));
}

__device__ __forceinline__ f32x4 mfma(const mbf16x8& a, const mbf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- forward
template <int D>
__global__ void __launch_bounds__(NT, 2) attn_fwd_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BKV * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG];
  char* Ks = smem;
  char* Vs = smem + IMG;
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (p.Hq / p.Hkv);
  const int T = p.T;
  const int qrow = qt * BQ + w * 16 + (lane & 15);
  const bf16_t* qb = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  mbf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qf[ks] = load_frag_global(qb, p.q_st, qrow, T, ks, lane);
  rope_frags<KS, D>(qf, p.rope_cos, p.rope_sin, qrow, T, lane);
  const float c = p.scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kv_end = p.causal ? min(T, (qt + 1) * BQ) : T;
  for (int kv0 = 0; kv0 < kv_end; kv0 += BKV) {
    __syncthreads();
    stage_tile<D, true, false>(kb, p.k_st, kv0, T, Ks, nullptr, p.rope_cos, p.rope_sin);
    stage_tile<D, false, true>(vb, p.v_st, kv0, T, nullptr, Vs);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s[t] = mfma(frag_row<D>(Ks, 16 * t, ks, lane), qf[ks], s[t]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kv = kv0 + 16 * t + 4 * g + r;
        float v = s[t][r] * c;
        if (kv >= T || (p.causal && kv > qrow)) v = -INFINITY;
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = (m_new == -INFINITY) ? 1.f : exp2f(m - m_new);
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = (m_new == -INFINITY) ? 0.f : exp2f(s[t][r] - m_new);
        s[t][r] = e;
        rs += e;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = m_new;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const mbf16x8 pf = pack_p(s[2 * cc], s[2 * cc + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = mfma(frag_tr<D>(Vs, 32 * cc, 16 * dt, lane), pf, o[dt]);
    }
  }
  if (qrow < T) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* ob = p.o + b * p.o_sb + (int64_t)qrow * p.o_st + h * p.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[dt][r] * inv);
      *reinterpret_cast<u16x4*>(ob + 16 * dt + 4 * g) = v;
    }
    if (g == 0) p.lse[((int64_t)b * p.Hq + h) * T + qrow] = (m + log2f(l)) / LOG2E;
  }
}

// ---------------------------------------------------------------- backward: delta = rowsum(dO * O)
// DRPT rows per thread group, all loads issued before the first use (one-shot threads are latency
// bound: a lone 16-B load pair per thread kept this pass near 2 TB/s).  With the fused dQ path it also
// zeroes the rows of the fp32 dQ accumulator.
constexpr int DRPT = 4;
template <int D>
__global__ void __launch_bounds__(NT) attn_bwd_delta_kernel(AttnParams p) {
  constexpr int TPR = D / 8;  // threads per row
  constexpr int RPB = NT / TPR;  // rows per block per pass
  const int64_t rows = (int64_t)p.B * p.Hq * p.T;
  const int part = threadIdx.x % TPR;
  float a[DRPT][8], o[DRPT][8];
  int64_t rr[DRPT];
#pragma unroll
  for (int i = 0; i < DRPT; ++i) {
    const int64_t row = ((int64_t)blockIdx.x * DRPT + i) * RPB + threadIdx.x / TPR;
    rr[i] = row;
    if (row < rows) {
      const int t = (int)(row % p.T);
      const int h = (int)((row / p.T) % p.Hq);
      const int b = (int)(row / ((int64_t)p.T * p.Hq));
      load8(p.dout + b * p.do_sb + (int64_t)t * p.do_st + h * p.do_sh + part * 8, a[i]);
      load8(p.o + b * p.o_sb + (int64_t)t * p.o_st + h * p.o_sh + part * 8, o[i]);
    }
  }
  if (p.dq_acc != nullptr) {  // fused-dQ accumulator rows start at zero
#pragma unroll
    for (int i = 0; i < DRPT; ++i)
      if (rr[i] < rows) {
        float4* z = reinterpret_cast<float4*>(p.dq_acc + rr[i] * D + part * 8);
        z[0] = z[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
  }
#pragma unroll
  for (int i = 0; i < DRPT; ++i) {
    float acc = 0.f;
    if (rr[i] < rows) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += a[i][j] * o[i][j];
    }
#pragma unroll
    for (int off = TPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (rr[i] < rows && part == 0) p.delta[rr[i]] = acc;
  }
}

// dq = scale * dq_acc ([B][Hq][T][D] fp32 from the fused dK/dV/dQ kernel), 8 columns per thread
__global__ void __launch_bounds__(NT) attn_dq_convert_kernel(AttnParams p) {
  const int D = p.D, T = p.T;
  const int64_t n8 = (int64_t)p.B * p.Hq * T * (D / 8);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  constexpr int U = 4;  // chunks in flight per thread
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n8; i0 += U * stride) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * stride < n8) load8(p.dq_acc + (i0 + u * stride) * 8, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n8) break;
      const int c8 = (int)(i % (D / 8));
      int64_t r = i / (D / 8);
      const int t = (int)(r % T);
      r /= T;
      const int h = (int)(r % p.Hq);
      const int b = (int)(r / p.Hq);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[u][j] *= p.scale;
      store8(p.dq + b * p.dq_sb + (int64_t)t * p.dq_st + h * p.dq_sh + c8 * 8, v[u]);
    }
  }
}

// ---------------------------------------------------------------- backward: dQ (query-stationary)
template <int D>
__global__ void __launch_bounds__(NT, 2) attn_bwd_dq_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BKV * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[3 * IMG];
  char* Kr = smem;
  char* Kt = smem + IMG;
  char* Vr = smem + 2 * IMG;
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (p.Hq / p.Hkv);
  const int T = p.T;
  const int qrow = qt * BQ + w * 16 + (lane & 15);
  const bf16_t* qb = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* dob = p.dout + b * p.do_sb + h * p.do_sh;
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  mbf16x8 qf[KS], df[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = load_frag_global(qb, p.q_st, qrow, T, ks, lane);
    df[ks] = load_frag_global(dob, p.do_st, qrow, T, ks, lane);
  }
  rope_frags<KS, D>(qf, p.rope_cos, p.rope_sin, qrow, T, lane);
  const int64_t rowid = ((int64_t)b * p.Hq + h) * T + qrow;
  const float lse2 = qrow < T ? p.lse[rowid] * LOG2E : 0.f;
  const float dl = qrow < T ? p.delta[rowid] : 0.f;
  const float c = p.scale * LOG2E;
  f32x4 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kv_end = p.causal ? min(T, (qt + 1) * BQ) : T;
  for (int kv0 = 0; kv0 < kv_end; kv0 += BKV) {
    __syncthreads();
    stage_tile<D, true, true>(kb, p.k_st, kv0, T, Kr, Kt, p.rope_cos, p.rope_sin);
    stage_tile<D, true, false>(vb, p.v_st, kv0, T, Vr, nullptr);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s[t] = mfma(frag_row<D>(Kr, 16 * t, ks, lane), qf[ks], s[t]);
        dp[t] = mfma(frag_row<D>(Vr, 16 * t, ks, lane), df[ks], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kv = kv0 + 16 * t + 4 * g + r;
        const bool ok = qrow < T && kv < T && !(p.causal && kv > qrow);
        const float pr = ok ? exp2f(s[t][r] * c - lse2) : 0.f;
        s[t][r] = pr * (dp[t][r] - dl);  // dS (unscaled)
      }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const mbf16x8 sf = pack_p(s[2 * cc], s[2 * cc + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) dq[dt] = mfma(frag_tr<D>(Kt, 32 * cc, 16 * dt, lane), sf, dq[dt]);
    }
  }
  rope_grad_acc<DT, D>(dq, p.rope_cos, p.rope_sin, qrow, T, lane);
  if (qrow < T) {
    bf16_t* out = p.dq + b * p.dq_sb + (int64_t)qrow * p.dq_st + h * p.dq_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(dq[dt][r] * p.scale);
      *reinterpret_cast<u16x4*>(out + 16 * dt + 4 * g) = v;
    }
  }
}

// ---------------------------------------------------------------- backward: dK, dV (key-stationary)
template <int D>
__global__ void __launch_bounds__(NT, 1) attn_bwd_dkdv_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BQ * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG + 2 * BQ * 4];
  char* Qr = smem;
  char* Qt = smem + IMG;
  char* Dr = smem + 2 * IMG;
  char* Dt = smem + 3 * IMG;
  float* s_lse = reinterpret_cast<float*>(smem + 4 * IMG);
  float* s_dl = s_lse + BQ;
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int kt = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int T = p.T, G = p.Hq / p.Hkv;
  const int kvrow = kt * BKV + w * 16 + (lane & 15);
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  mbf16x8 kf[KS], vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    kf[ks] = load_frag_global(kb, p.k_st, kvrow, T, ks, lane);
    vf[ks] = load_frag_global(vb, p.v_st, kvrow, T, ks, lane);
  }
  rope_frags<KS, D>(kf, p.rope_cos, p.rope_sin, kvrow, T, lane);
  const float c = p.scale * LOG2E;
  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q_begin = p.causal ? kt * BKV : 0;
  for (int hq = hk * G; hq < (hk + 1) * G; ++hq) {
    const bf16_t* qb = p.q + b * p.q_sb + hq * p.q_sh;
    const bf16_t* dob = p.dout + b * p.do_sb + hq * p.do_sh;
    const float* lse = p.lse + ((int64_t)b * p.Hq + hq) * T;
    const float* dlt = p.delta + ((int64_t)b * p.Hq + hq) * T;
    for (int q0 = q_begin; q0 < T; q0 += BQ) {
      __syncthreads();
      stage_tile<D, true, true>(qb, p.q_st, q0, T, Qr, Qt, p.rope_cos, p.rope_sin);
      stage_tile<D, true, true>(dob, p.do_st, q0, T, Dr, Dt);
      if (threadIdx.x < BQ) {
        const int q = q0 + threadIdx.x;
        s_lse[threadIdx.x] = q < T ? lse[q] * LOG2E : 0.f;
        s_dl[threadIdx.x] = q < T ? dlt[q] : 0.f;
      }
      __syncthreads();
      f32x4 s[4], dp[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          s[t] = mfma(frag_row<D>(Qr, 16 * t, ks, lane), kf[ks], s[t]);   // S^T: [q][kv = lane]
          dp[t] = mfma(frag_row<D>(Dr, 16 * t, ks, lane), vf[ks], dp[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = 16 * t + 4 * g + r;
          const int q = q0 + qi;
          const bool ok = q < T && kvrow < T && !(p.causal && kvrow > q);
          const float pr = ok ? exp2f(s[t][r] * c - s_lse[qi]) : 0.f;
          s[t][r] = pr;
          dp[t][r] = pr * (dp[t][r] - s_dl[qi]);  // dS
        }
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const mbf16x8 pf = pack_p(s[2 * cc], s[2 * cc + 1]);
        const mbf16x8 sf = pack_p(dp[2 * cc], dp[2 * cc + 1]);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dv[dt] = mfma(frag_tr<D>(Dt, 32 * cc, 16 * dt, lane), pf, dv[dt]);
          dk[dt] = mfma(frag_tr<D>(Qt, 32 * cc, 16 * dt, lane), sf, dk[dt]);
        }
      }
    }
  }
  rope_grad_acc<DT, D>(dk, p.rope_cos, p.rope_sin, kvrow, T, lane);
  if (kvrow < T) {
    bf16_t* dkp = p.dk + b * p.dk_sb + (int64_t)kvrow * p.dk_st + hk * p.dk_sh;
    bf16_t* dvp = p.dv + b * p.dv_sb + (int64_t)kvrow * p.dv_st + hk * p.dv_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 a, v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = f2bf(dk[dt][r] * p.scale);
        v[r] = f2bf(dv[dt][r]);
      }
      *reinterpret_cast<u16x4*>(dkp + 16 * dt + 4 * g) = a;
      *reinterpret_cast<u16x4*>(dvp + 16 * dt + 4 * g) = v;
    }
  }
}

// ================================================================ v2 kernels (no in-load RoPE)
// Same MFMA / LDS-image structure as above, plus:
//  * register-prefetched staging (T14): the K/V (or Q/dO) tile t+1 is loaded into VGPRs while tile t
//    is multiplied, and written to LDS between two barriers — global latency hides behind the MFMAs;
//  * forward: each wave owns two 16-row query groups (BQ = 128 per workgroup), so every K / V fragment
//    read from LDS feeds two MFMAs; causal masking math only on tiles that cross the diagonal, fully
//    masked tiles are skipped per wave, heavy (late) query tiles are scheduled first;
//  * dK/dV: one workgroup per (key tile, QUERY head) — 4x more workgroups than looping over the GQA
//    group inside a block — writing fp32 partials that a small kernel sums over the group.
template <int D>
struct TileRegs {
  static constexpr int CPR = D / 8, NCH = 64 * CPR / NT;
  u16x8 a[NCH], b[NCH];
};

template <int D>
__device__ __forceinline__ void fetch_tile(TileRegs<D>& tr, const bf16_t* __restrict__ A, int64_t ars,
                                           const bf16_t* __restrict__ B, int64_t brs, int row0, int T) {
  constexpr int CPR = TileRegs<D>::CPR;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::NCH; ++i) {
    const int c = threadIdx.x + NT * i;
    const int r = c / CPR, ch = c % CPR;
    const int gr = row0 + r;
    tr.a[i] = gr < T ? ld16(A + (int64_t)gr * ars + ch * 8) : zero16();
    tr.b[i] = gr < T ? ld16(B + (int64_t)gr * brs + ch * 8) : zero16();
  }
}

// write A to (row image a_row, optional tr image a_tr) and B likewise
template <int D>
__device__ __forceinline__ void store_tile(const TileRegs<D>& tr, char* a_row, char* a_tr, char* b_row, char* b_tr) {
  constexpr int CPR = TileRegs<D>::CPR;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::NCH; ++i) {
    const int c = threadIdx.x + NT * i;
    const int r = c / CPR, ch = c % CPR;
    if (a_row) *reinterpret_cast<u16x8*>(a_row + row_off<D>(r, ch)) = tr.a[i];
    if (a_tr) *reinterpret_cast<u16x8*>(a_tr + tr_off<D>(r, ch * 8)) = tr.a[i];
    if (b_row) *reinterpret_cast<u16x8*>(b_row + row_off<D>(r, ch)) = tr.b[i];
    if (b_tr) *reinterpret_cast<u16x8*>(b_tr + tr_off<D>(r, ch * 8)) = tr.b[i];
  }
}

// QG query groups of 16 rows per wave (query tile = 64 * QG): each K / V fragment read feeds QG MFMAs.
template <int D, int QG>
__global__ void __launch_bounds__(NT, 2) attn_fwd2_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BKV * D * 2, BQW = 64 * QG;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG];
  char* Ks = smem;
  char* Vs = smem + IMG;
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int qt = gridDim.x - 1 - blockIdx.x, h = blockIdx.y, b = blockIdx.z;  // heavy causal tiles first
  const int hk = h / (p.Hq / p.Hkv);
  const int T = p.T;
  const int qbase = qt * BQW + w * 16 * QG;  // this wave's queries: qbase + 16 qg + (lane & 15)
  const bf16_t* qb = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  mbf16x8 qf[QG][KS];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qg][ks] = load_frag_global(qb, p.q_st, qbase + 16 * qg + (lane & 15), T, ks, lane);
  const float c = p.scale * LOG2E;
  // m: running row max of the RAW scores (scale folded into the exponent's fma); l: this lane's
  // partial row sum (its 16 of every 64 keys) — the 4 lanes of a query are summed once at the end
  float m[QG], l[QG];
  f32x4 o[QG][DT];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    m[qg] = NEG_BIG;
    l[qg] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[qg][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int kv_end = p.causal ? min(T, (qt + 1) * BQW) : T;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  TileRegs<D> tr;
  fetch_tile<D>(tr, kb, p.k_st, vb, p.v_st, 0, T);
  for (int j = 0; j < ntiles; ++j) {
    const int kv0 = j * BKV;
    __syncthreads();
    store_tile<D>(tr, Ks, nullptr, nullptr, Vs);
    __syncthreads();
    if (j + 1 < ntiles) fetch_tile<D>(tr, kb, p.k_st, vb, p.v_st, kv0 + BKV, T);
    if (p.causal && kv0 > qbase + 16 * QG - 1) continue;  // every key of this tile is in this wave's future
    f32x4 s[QG][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) s[qg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const mbf16x8 kf = frag_row<D>(Ks, 16 * t, ks, lane);
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) s[qg][t] = mfma(kf, qf[qg][ks], s[qg][t]);
      }
    }
    const bool need_mask = kv0 + BKV > T || (p.causal && kv0 + BKV - 1 > qbase);
#pragma unroll
    for (int qg = 0; qg < QG; ++qg) {
      const int qrow = qbase + 16 * qg + (lane & 15);
      float mx = NEG_BIG;
      if (need_mask) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kv = kv0 + 16 * t + 4 * g + r;
            if (kv >= T || (p.causal && kv > qrow)) s[qg][t][r] = -INFINITY;
          }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[qg][t][r]);
      const float m_new = fmaxf(m[qg], max_x16_x32(mx));
      const float alpha = fast_exp2((m[qg] - m_new) * c);
      const float mc = m_new * c;
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = fast_exp2(fmaf(s[qg][t][r], c, -mc));
          s[qg][t][r] = e;
          rs += e;
        }
      l[qg] = fmaf(l[qg], alpha, rs);
      m[qg] = m_new;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[qg][dt] *= alpha;
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      mbf16x8 pf[QG];
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) pf[qg] = pack_p(s[qg][2 * cc], s[qg][2 * cc + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const mbf16x8 vf = frag_tr<D>(Vs, 32 * cc, 16 * dt, lane);
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) o[qg][dt] = mfma(vf, pf[qg], o[qg][dt]);
      }
    }
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const int qrow = qbase + 16 * qg + (lane & 15);
    const float lsum = sum_x16_x32(l[qg]);  // (all lanes take part: the swaps need a full EXEC)
    if (qrow >= T) continue;
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* ob = p.o + b * p.o_sb + (int64_t)qrow * p.o_st + h * p.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[qg][dt][r] * inv);
      *reinterpret_cast<u16x4*>(ob + 16 * dt + 4 * g) = v;
    }
    if (g == 0) p.lse[((int64_t)b * p.Hq + h) * T + qrow] = (m[qg] * c + log2f(lsum)) / LOG2E;
  }
}

// v3 forward: the K/V LDS images are double-buffered, so one barrier per key tile (v2: two — one
// before overwriting the single stage, one before reading it).  Iteration j multiplies tile j from
// stage j&1 while tile j+1 (prefetched into VGPRs during iteration j-1) is written into the other
// stage and tile j+2 is fetched; the only wait on global memory is for loads issued one whole
// iteration earlier.  Waves whose queries all precede a tile skip its math but not its barrier.
template <int D, int QG>
__global__ void __launch_bounds__(NT, 2) attn_fwd3_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BKV * D * 2, BQW = 64 * QG;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];  // [stage][K row image | V tr image]
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int qt = gridDim.x - 1 - blockIdx.x, h = blockIdx.y, b = blockIdx.z;  // heavy causal tiles first
  const int hk = h / (p.Hq / p.Hkv);
  const int T = p.T;
  const int qbase = qt * BQW + w * 16 * QG;
  const bf16_t* qb = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  const int kv_end = p.causal ? min(T, (qt + 1) * BQW) : T;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  TileRegs<D> tr;
  fetch_tile<D>(tr, kb, p.k_st, vb, p.v_st, 0, T);
  mbf16x8 qf[QG][KS];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qg][ks] = load_frag_global(qb, p.q_st, qbase + 16 * qg + (lane & 15), T, ks, lane);
  store_tile<D>(tr, smem, nullptr, nullptr, smem + IMG);
  if (ntiles > 1) fetch_tile<D>(tr, kb, p.k_st, vb, p.v_st, BKV, T);
  __syncthreads();
  const float c = p.scale * LOG2E;
  float m[QG], l[QG];
  f32x4 o[QG][DT];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    m[qg] = NEG_BIG;
    l[qg] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[qg][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int j = 0; j < ntiles; ++j) {
    const int kv0 = j * BKV;
    const char* Ks = smem + (j & 1) * 2 * IMG;
    const char* Vs = Ks + IMG;
    if (j + 1 < ntiles) {  // stage (j+1)&1 was last read in iteration j-1, before its barrier
      char* nk = smem + ((j + 1) & 1) * 2 * IMG;
      store_tile<D>(tr, nk, nullptr, nullptr, nk + IMG);
      if (j + 2 < ntiles) fetch_tile<D>(tr, kb, p.k_st, vb, p.v_st, kv0 + 2 * BKV, T);
    }
    if (!(p.causal && kv0 > qbase + 16 * QG - 1)) {
      f32x4 s[QG][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) s[qg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const mbf16x8 kf = frag_row<D>(Ks, 16 * t, ks, lane);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) s[qg][t] = mfma(kf, qf[qg][ks], s[qg][t]);
        }
      }
      const bool need_mask = kv0 + BKV > T || (p.causal && kv0 + BKV - 1 > qbase);
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) {
        const int qrow = qbase + 16 * qg + (lane & 15);
        float mx = NEG_BIG;
        if (need_mask) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int kv = kv0 + 16 * t + 4 * g + r;
              if (kv >= T || (p.causal && kv > qrow)) s[qg][t][r] = -INFINITY;
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[qg][t][r]);
        const float m_new = fmaxf(m[qg], max_x16_x32(mx));
        const float alpha = fast_exp2((m[qg] - m_new) * c);
        const float mc = m_new * c;
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = fast_exp2(fmaf(s[qg][t][r], c, -mc));
            s[qg][t][r] = e;
            rs += e;
          }
        l[qg] = fmaf(l[qg], alpha, rs);
        m[qg] = m_new;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[qg][dt] *= alpha;
      }
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        mbf16x8 pf[QG];
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) pf[qg] = pack_p(s[qg][2 * cc], s[qg][2 * cc + 1]);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const mbf16x8 vf = frag_tr<D>(Vs, 32 * cc, 16 * dt, lane);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) o[qg][dt] = mfma(vf, pf[qg], o[qg][dt]);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const int qrow = qbase + 16 * qg + (lane & 15);
    const float lsum = sum_x16_x32(l[qg]);
    if (qrow >= T) continue;
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* ob = p.o + b * p.o_sb + (int64_t)qrow * p.o_st + h * p.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[qg][dt][r] * inv);
      *reinterpret_cast<u16x4*>(ob + 16 * dt + 4 * g) = v;
    }
    if (g == 0) p.lse[((int64_t)b * p.Hq + h) * T + qrow] = (m[qg] * c + log2f(lsum)) / LOG2E;
  }
}

// ---------------------------------------------------------------- v4 forward: fewer VALU per MFMA
// The v3 loop issued ~5.5 VALU per MFMA (profiles/r5_attention_pmc.md: 16 % MFMA busy at D = 128) and
// about a third of them were bookkeeping: 64-bit address arithmetic and per-row bounds compares /
// selects of the register-staged K/V loads, 32 packed multiplies rescaling O every tile, and 32 adds of
// the row sums.  v4 keeps v3's structure (double-buffered K/V images, one barrier per key tile) and:
//   * loads the K/V tile through buffer descriptors rebased per tile in scalar registers: each lane's
//     byte offsets are loop-invariant (one VALU add per load), rows past T fall outside the descriptor
//     range and read as zero — no compare / select;
//   * defers the O rescale (the "RESCALE_THRESHOLD" idea): the running max used for the exponent moves
//     only when a row's max grows by more than 8 in the log2 domain (then P <= 2^8, exact in fp32 / bf16
//     range) — a wave-uniform branch that almost every tile after the first few skips;
//   * sums the rows on the matrix pipe: one extra MFMA per P fragment against an all-ones V^T fragment
//     accumulates l (the lane's query row sum) — 4 MFMAs per tile instead of 32 adds + 4 lane swaps.
template <int D>
struct TileOff {  // a thread's byte offsets of its chunks inside a 64-row tile of A and B
  static constexpr int CPR = D / 8, NCH = 64 * CPR / NT;
  uint32_t a0, b0, da, db;  // chunk i: a0 + i * da
};

template <int D>
__device__ __forceinline__ TileOff<D> tile_offsets(int64_t ars, int64_t brs) {
  constexpr int CPR = TileOff<D>::CPR;
  const int r = threadIdx.x / CPR, ch = threadIdx.x % CPR;  // chunk i: row r + (NT / CPR) i, same ch
  TileOff<D> t;
  t.a0 = (uint32_t)((r * ars + ch * 8) * 2);
  t.b0 = (uint32_t)((r * brs + ch * 8) * 2);
  t.da = (uint32_t)((NT / CPR) * ars * 2);
  t.db = (uint32_t)((NT / CPR) * brs * 2);
  return t;
}

template <int D>
__device__ __forceinline__ void fetch_tile_buf(TileRegs<D>& tr, const TileOff<D>& to, const bf16_t* __restrict__ A,
                                               int64_t ars, const bf16_t* __restrict__ B, int64_t brs, int row0,
                                               int T) {
  const int rows = T - row0;  // >= 1: rows past T are outside the descriptor range (read as zero)
  const int na = (int)((rows - 1) * ars * 2 + 2 * D), nb = (int)((rows - 1) * brs * 2 + 2 * D);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)row0 * ars), (short)0,
                                                                      na, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (int64_t)row0 * brs), (short)0,
                                                                      nb, 0x00020000);
#pragma unroll
  for (int i = 0; i < TileRegs<D>::NCH; ++i) {
    tr.a[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, to.a0 + i * to.da, 0, 0));
    tr.b[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, to.b0 + i * to.db, 0, 0));
  }
}

// the buffer-descriptor fetch needs every [T][row stride] span to fit a 31-bit byte offset (true for
// every training shape here: Llama-3-8B T = 4096 spans 48 MB); otherwise the pointer fetch
__device__ __forceinline__ bool attn_buf_ok(const AttnParams& p) {
  const int64_t lim = (int64_t)1 << 31, T = p.T;
  return T * p.k_st * 2 < lim && T * p.v_st * 2 < lim && T * p.q_st * 2 < lim &&
         (p.dout == nullptr || T * p.do_st * 2 < lim);
}

template <int D>
__device__ __forceinline__ void fetch_any(TileRegs<D>& tr, const TileOff<D>& to, bool buf, const bf16_t* __restrict__ A,
                                          int64_t ars, const bf16_t* __restrict__ B, int64_t brs, int row0, int T) {
  if (buf) fetch_tile_buf<D>(tr, to, A, ars, B, brs, row0, T);
  else fetch_tile<D>(tr, A, ars, B, brs, row0, T);
}

constexpr float RESCALE_LOG2 = 8.f;  // deferred-rescale threshold (log2 units): P <= 2^8

template <int D, int QG, int MINB = 2>
__global__ void __launch_bounds__(NT, MINB) attn_fwd4_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BKV * D * 2, BQW = 64 * QG;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];  // [stage][K row image | V tr image]
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int qt = gridDim.x - 1 - blockIdx.x, h = blockIdx.y, b = blockIdx.z;  // heavy causal tiles first
  const int hk = h / (p.Hq / p.Hkv);
  const int T = p.T;
  const int qbase = qt * BQW + w * 16 * QG;
  const bf16_t* qb = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  const int kv_end = p.causal ? min(T, (qt + 1) * BQW) : T;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  const TileOff<D> to = tile_offsets<D>(p.k_st, p.v_st);
  TileRegs<D> tr;
  fetch_tile_buf<D>(tr, to, kb, p.k_st, vb, p.v_st, 0, T);
  mbf16x8 qf[QG][KS];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qg][ks] = load_frag_global(qb, p.q_st, qbase + 16 * qg + (lane & 15), T, ks, lane);
  store_tile<D>(tr, smem, nullptr, nullptr, smem + IMG);
  if (ntiles > 1) fetch_tile_buf<D>(tr, to, kb, p.k_st, vb, p.v_st, BKV, T);
  __syncthreads();
  const float c = p.scale * LOG2E;
  mbf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  float m[QG];      // the max the exponents are taken against (moves only past the threshold)
  f32x4 lacc[QG];   // row sums from the matrix pipe (every element = the lane's query row sum)
  f32x4 o[QG][DT];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    m[qg] = NEG_BIG;
    lacc[qg] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[qg][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int j = 0; j < ntiles; ++j) {
    const int kv0 = j * BKV;
    const char* Ks = smem + (j & 1) * 2 * IMG;
    const char* Vs = Ks + IMG;
    if (j + 1 < ntiles) {  // stage (j+1)&1 was last read in iteration j-1, before its barrier
      char* nk = smem + ((j + 1) & 1) * 2 * IMG;
      store_tile<D>(tr, nk, nullptr, nullptr, nk + IMG);
      if (j + 2 < ntiles) fetch_tile_buf<D>(tr, to, kb, p.k_st, vb, p.v_st, kv0 + 2 * BKV, T);
    }
    if (!(p.causal && kv0 > qbase + 16 * QG - 1)) {
      f32x4 s[QG][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) s[qg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const mbf16x8 kf = frag_row<D>(Ks, 16 * t, ks, lane);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) s[qg][t] = mfma(kf, qf[qg][ks], s[qg][t]);
        }
      }
      const bool need_mask = kv0 + BKV > T || (p.causal && kv0 + BKV - 1 > qbase);
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) {
        const int qrow = qbase + 16 * qg + (lane & 15);
        if (need_mask) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int kv = kv0 + 16 * t + 4 * g + r;
              if (kv >= T || (p.causal && kv > qrow)) s[qg][t][r] = -INFINITY;
            }
        }
        float mx = NEG_BIG;
#pragma unroll
        for (int t = 0; t < 4; ++t) mx = fmaxf(mx, fmaxf(fmaxf(s[qg][t][0], s[qg][t][1]), fmaxf(s[qg][t][2], s[qg][t][3])));
        mx = max_x16_x32(mx);
        // deferred rescale: move the exponent's reference only when some row of the wave would see
        // P > 2^RESCALE_LOG2 (the first tile always moves it: m starts at NEG_BIG)
        if (__any((mx - m[qg]) * c > RESCALE_LOG2)) {
          const float m_new = fmaxf(m[qg], mx);
          const float alpha = fast_exp2((m[qg] - m_new) * c);
          m[qg] = m_new;
          lacc[qg] *= alpha;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[qg][dt] *= alpha;
        }
        const float mc = m[qg] * c;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[qg][t][r] = fast_exp2(fmaf(s[qg][t][r], c, -mc));
      }
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        mbf16x8 pf[QG];
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) {
          pf[qg] = pack_p(s[qg][2 * cc], s[qg][2 * cc + 1]);
          lacc[qg] = mfma(ones, pf[qg], lacc[qg]);
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const mbf16x8 vf = frag_tr<D>(Vs, 32 * cc, 16 * dt, lane);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) o[qg][dt] = mfma(vf, pf[qg], o[qg][dt]);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const int qrow = qbase + 16 * qg + (lane & 15);
    const float lsum = lacc[qg][0];
    if (qrow >= T) continue;
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* ob = p.o + b * p.o_sb + (int64_t)qrow * p.o_st + h * p.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[qg][dt][r] * inv);
      *reinterpret_cast<u16x4*>(ob + 16 * dt + 4 * g) = v;
    }
    if (g == 0) p.lse[((int64_t)b * p.Hq + h) * T + qrow] = (m[qg] * c + log2f(lsum)) / LOG2E;
  }
}

// dQ, query-stationary, prefetched K/V tiles; QG query groups of 16 rows per wave (query tile =
// 64 * QG): every K / V fragment read from LDS feeds QG MFMAs.
// DB: K/V images double-buffered (one barrier per key tile, as attn_fwd3_kernel) at twice the LDS.
// MINB: workgroups per CU the register budget is sized for (2: <= 256 registers per wave; 1: one wave per
// SIMD with up to 512, the accumulators in AGPRs — the D = 128 two-group variants)
template <int D, int QG, bool DB = false, int MINB = 2>
__global__ void __launch_bounds__(NT, MINB) attn_bwd_dq2_kernel(AttnParams p) {
  constexpr int KS = D / 32, DT = D / 16, IMG = BKV * D * 2, BQW = BQ * QG;
  constexpr int STAGE = 3 * IMG;
  __shared__ __attribute__((aligned(16))) char smem[(DB ? 2 : 1) * STAGE];
  // w wave-uniform (readfirstlane): its tests are scalar branches, not per-lane exec masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  const int qt = gridDim.x - 1 - blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (p.Hq / p.Hkv);
  const int T = p.T;
  const int qbase = qt * BQW + w * 16 * QG;  // this wave's queries: qbase + 16 qg + (lane & 15)
  const bf16_t* qb = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* dob = p.dout + b * p.do_sb + h * p.do_sh;
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  mbf16x8 qf[QG][KS], df[QG][KS];
  float lse2[QG], dl[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const int qrow = qbase + 16 * qg + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[qg][ks] = load_frag_global(qb, p.q_st, qrow, T, ks, lane);
      df[qg][ks] = load_frag_global(dob, p.do_st, qrow, T, ks, lane);
    }
    const int64_t rowid = ((int64_t)b * p.Hq + h) * T + qrow;
    lse2[qg] = qrow < T ? p.lse[rowid] * LOG2E : 0.f;
    dl[qg] = qrow < T ? p.delta[rowid] : 0.f;
  }
  const float c = p.scale * LOG2E;
  f32x4 dq[QG][DT];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dq[qg][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kv_end = p.causal ? min(T, (qt + 1) * BQW) : T;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  TileRegs<D> tr;
  const bool buf = attn_buf_ok(p);
  const TileOff<D> to = tile_offsets<D>(p.k_st, p.v_st);
  fetch_any<D>(tr, to, buf, kb, p.k_st, vb, p.v_st, 0, T);
  if constexpr (DB) {
    store_tile<D>(tr, smem, smem + IMG, smem + 2 * IMG, nullptr);
    if (ntiles > 1) fetch_any<D>(tr, to, buf, kb, p.k_st, vb, p.v_st, BKV, T);
    __syncthreads();
  }
  for (int j = 0; j < ntiles; ++j) {
    const int kv0 = j * BKV;
    char* Kr = smem + (DB ? (j & 1) * STAGE : 0);
    char* Kt = Kr + IMG;
    char* Vr = Kr + 2 * IMG;
    if constexpr (DB) {
      if (j + 1 < ntiles) {  // the other stage was last read before the previous barrier
        char* nx = smem + ((j + 1) & 1) * STAGE;
        store_tile<D>(tr, nx, nx + IMG, nx + 2 * IMG, nullptr);
        if (j + 2 < ntiles) fetch_any<D>(tr, to, buf, kb, p.k_st, vb, p.v_st, kv0 + 2 * BKV, T);
      }
    } else {
      __syncthreads();
      store_tile<D>(tr, Kr, Kt, Vr, nullptr);
      __syncthreads();
      if (j + 1 < ntiles) fetch_any<D>(tr, to, buf, kb, p.k_st, vb, p.v_st, kv0 + BKV, T);
    }
    // every key of this tile is in this wave's future (DB: skip the math, not the barrier)
    if (p.causal && kv0 > qbase + 16 * QG - 1) {
      if constexpr (DB) __syncthreads();
      continue;
    }
    f32x4 s[QG][4], dp[QG][4];
    // key sub-tiles in pairs: four independent accumulation chains per k-step (two chains left each
    // MFMA waiting on its predecessor's result and each fragment read waited for just in time)
#pragma unroll
    for (int tp = 0; tp < 4; tp += 2) {
#pragma unroll
      for (int t = tp; t < tp + 2; ++t)
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) s[qg][t] = dp[qg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        mbf16x8 kf[2], vf[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          kf[u] = frag_row<D>(Kr, 16 * (tp + u), ks, lane);
          vf[u] = frag_row<D>(Vr, 16 * (tp + u), ks, lane);
        }
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            s[qg][tp + u] = mfma(kf[u], qf[qg][ks], s[qg][tp + u]);
            dp[qg][tp + u] = mfma(vf[u], df[qg][ks], dp[qg][tp + u]);
          }
      }
    }
    const bool need_mask = kv0 + BKV > T || (p.causal && kv0 + BKV - 1 > qbase) || qbase + 16 * QG > T;
    // per 32-key half cc: P, the mask (masked tiles only: branch-free selects under one wave-uniform
    // branch), dS, the bf16 pack and the half's dQ MFMAs (the second half's exponentials can issue in the
    // shadow of the first half's MFMAs)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
#pragma unroll
      for (int qg = 0; qg < QG; ++qg)
#pragma unroll
        for (int t = 2 * cc; t < 2 * cc + 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[qg][t][r] = fast_exp2(fmaf(s[qg][t][r], c, -lse2[qg]));
      if (need_mask) {
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) {
          const int qrow = qbase + 16 * qg + (lane & 15);
#pragma unroll
          for (int t = 2 * cc; t < 2 * cc + 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int kv = kv0 + 16 * t + 4 * g + r;
              const bool dead = (qrow >= T) | (kv >= T) | (p.causal & (kv > qrow));
              s[qg][t][r] = dead ? 0.f : s[qg][t][r];
            }
        }
      }
      mbf16x8 sf[QG];
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) {
#pragma unroll
        for (int t = 2 * cc; t < 2 * cc + 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[qg][t][r] = s[qg][t][r] * (dp[qg][t][r] - dl[qg]);
        sf[qg] = pack_p(s[qg][2 * cc], s[qg][2 * cc + 1]);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const mbf16x8 ktf = frag_tr<D>(Kt, 32 * cc, 16 * dt, lane);
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) dq[qg][dt] = mfma(ktf, sf[qg], dq[qg][dt]);
      }
    }
    if constexpr (DB) __syncthreads();
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const int qrow = qbase + 16 * qg + (lane & 15);
    if (qrow >= T) continue;
    bf16_t* out = p.dq + b * p.dq_sb + (int64_t)qrow * p.dq_st + h * p.dq_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(dq[qg][dt][r] * p.scale);
      *reinterpret_cast<u16x4*>(out + 16 * dt + 4 * g) = v;
    }
  }
}

// Fused-dQ step of attn_bwd_dkdv2_kernel<..., FQ>: barrier (the dS image is complete), then wave w adds
// dS[q0 + 16 w .. +15][keys 0 .. kmax) * K into dq_acc.  kmax < BK only for causal diagonal tiles.
template <int D, int BK, bool ATOMIC>
__device__ __forceinline__ void fused_dq(const AttnParams& p, const char* DSt, const char* Kt, float* dqa, int q0,
                                         int kmax, int w, int lane) {
  constexpr int DT = D / 16;
  __syncthreads();
  const int nk = (kmax < BK ? kmax : BK) / 32;
  f32x4 acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int kc = 0; kc < nk; ++kc) {
    const mbf16x8 af = frag_tr<BQ>(DSt, 32 * kc, 16 * w, lane);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc[dt] = mfma(af, frag_tr<D>(Kt, 32 * kc, 16 * dt, lane), acc[dt]);
  }
  const int qb = q0 + 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (qb + r >= p.T) break;
    float* row = dqa + (int64_t)(qb + r) * D + (lane & 15);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      if constexpr (ATOMIC) unsafeAtomicAdd(row + 16 * dt, acc[dt][r]);
      else row[16 * dt] = acc[dt][r];  // lab only (PDA_ATTN_BWD_FUSED bit 4): prices the atomics, wrong dQ
    }
  }
}

// dK / dV for one (key tile, query head): prefetched Q / dO tiles; output bf16 directly (no GQA) or
// fp32 partials [2][B][Hq][T][D] summed over the group by attn_dkv_reduce_kernel.
// KG key groups of 16 per wave (key tile = 64 * KG): every Q / dO fragment read from LDS and every
// transposed Q / dO fragment feeds KG MFMAs, and each staged Q / dO tile serves 64 * KG keys.
//
// FQ (fused dQ, single-stage only): the workgroup also adds its keys' share of dQ = dS K for every query
// tile it visits, so no query-stationary dQ kernel recomputes S and dP.  The waves' dS fragments go to
// an LDS image transposed to [key][query] (4 consecutive queries per 8-byte store), the key tile sits in
// LDS once as a transposed-read image, and after one extra barrier wave w multiplies query rows
// 16 w .. 16 w + 15 of dS by K (A and B both by ds_read_b64_tr_b16, the key order permuted alike) and
// adds the fp32 result into p.dq_acc ([B][Hq][T][D], zeroed by the delta kernel) with no-return
// atomics; attn_dq_convert_kernel scales it into dq.  Causal: a query tile only reads the key rows
// below its last query, which are exactly the rows of the waves that did not skip it.
template <int D, int KG, bool DB = false, int FQ = 0, int MINB = 2>
__global__ void __launch_bounds__(NT, MINB) attn_bwd_dkdv2_kernel(AttnParams p) {
  static_assert(!(DB && FQ), "fused dQ is single-stage");
  constexpr int KS = D / 32, DT = D / 16, IMG = BQ * D * 2, BK = BKV * KG;
  constexpr int STAGE = 4 * IMG + 2 * BQ * 4;  // Q row / Q tr / dO row / dO tr images + lse / delta
  constexpr int KIMG = FQ ? BK * D * 2 : 0, DSIMG = FQ ? BK * BQ * 2 : 0;
  __shared__ __attribute__((aligned(16))) char smem[(DB ? 2 : 1) * STAGE + KIMG + DSIMG];
  char* const Kt = smem + STAGE;        // [BK keys][D] transposed-read image (FQ)
  char* const DSt = smem + STAGE + KIMG;  // [BK keys][BQ queries] transposed-read image of dS (FQ)
  // w wave-uniform at D = 128 (scalar branches); per-lane at D = 64, where the readfirstlane form spills
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int w = D == 128 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6;
  const int kt = blockIdx.x, hq = blockIdx.y, b = blockIdx.z;
  const int T = p.T, G = p.Hq / p.Hkv, hk = hq / G;
  const int kvbase = kt * BK + w * 16 * KG;  // this wave's keys: kvbase + 16 kg + (lane & 15)
  const bf16_t* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vb = p.v + b * p.v_sb + hk * p.v_sh;
  mbf16x8 kf[KG][KS], vf[KG][KS];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[kg][ks] = load_frag_global(kb, p.k_st, kvbase + 16 * kg + (lane & 15), T, ks, lane);
      vf[kg][ks] = load_frag_global(vb, p.v_st, kvbase + 16 * kg + (lane & 15), T, ks, lane);
    }
  if constexpr (FQ) {  // visible after the first loop barrier
#pragma unroll
    for (int h = 0; h < KG; ++h) stage_tile<D, false, true>(kb, p.k_st, kt * BK + 64 * h, T, nullptr, Kt + h * 64 * D * 2);
  }
  const float c = p.scale * LOG2E;
  f32x4 dk[KG][DT], dv[KG][DT];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dk[kg][dt] = dv[kg][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q_begin = p.causal ? kt * BK : 0;
  float* const dqa = FQ ? p.dq_acc + ((int64_t)b * p.Hq + hq) * T * D : nullptr;
  const bf16_t* qb = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* dob = p.dout + b * p.do_sb + hq * p.do_sh;
  const float* lse = p.lse + ((int64_t)b * p.Hq + hq) * T;
  const float* dlt = p.delta + ((int64_t)b * p.Hq + hq) * T;
  TileRegs<D> tr;
  float nl = 0.f, nd = 0.f;
  auto fetch_stats = [&](int q0) {
    if (threadIdx.x < BQ) {
      const int q = q0 + threadIdx.x;
      nl = q < T ? lse[q] * LOG2E : 0.f;
      nd = q < T ? dlt[q] : 0.f;
    }
  };
  auto put = [&](char* st) {  // staged registers -> one stage's images and stats
    store_tile<D>(tr, st, st + IMG, st + 2 * IMG, st + 3 * IMG);
    if (threadIdx.x < BQ) {
      float* sl = reinterpret_cast<float*>(st + 4 * IMG);
      sl[threadIdx.x] = nl;
      sl[BQ + threadIdx.x] = nd;
    }
  };
  const bool buf = attn_buf_ok(p);
  const TileOff<D> to = tile_offsets<D>(p.q_st, p.do_st);
  if (q_begin < T) {
    fetch_any<D>(tr, to, buf, qb, p.q_st, dob, p.do_st, q_begin, T);
    fetch_stats(q_begin);
  }
  if constexpr (DB) {
    if (q_begin < T) {
      put(smem);
      if (q_begin + BQ < T) {
        fetch_any<D>(tr, to, buf, qb, p.q_st, dob, p.do_st, q_begin + BQ, T);
        fetch_stats(q_begin + BQ);
      }
    }
    __syncthreads();
  }
  for (int q0 = q_begin, j = 0; q0 < T; q0 += BQ, ++j) {
    char* st = smem + (DB ? (j & 1) * STAGE : 0);
    const char* Qr = st;
    const char* Qt = st + IMG;
    const char* Dr = st + 2 * IMG;
    const char* Dt = st + 3 * IMG;
    const float* s_lse = reinterpret_cast<const float*>(st + 4 * IMG);
    const float* s_dl = s_lse + BQ;
    if constexpr (DB) {
      if (q0 + BQ < T) {  // the other stage was last read before the previous barrier
        put(smem + ((j + 1) & 1) * STAGE);
        if (q0 + 2 * BQ < T) {
          fetch_any<D>(tr, to, buf, qb, p.q_st, dob, p.do_st, q0 + 2 * BQ, T);
          fetch_stats(q0 + 2 * BQ);
        }
      }
    } else {
      __syncthreads();
      put(st);
      __syncthreads();
      if (q0 + BQ < T) {
        fetch_any<D>(tr, to, buf, qb, p.q_st, dob, p.do_st, q0 + BQ, T);
        fetch_stats(q0 + BQ);
      }
    }
    // every query of this tile is before all of this wave's keys: nothing to add (wave-uniform)
    if (p.causal && q0 + BQ - 1 < kvbase) {
      if constexpr (FQ) {
        fused_dq<D, BK, FQ == 1>(p, DSt, Kt, dqa, q0, q0 + BQ - kt * BK, w, lane);
        continue;
      }
      if constexpr (DB) __syncthreads();
      continue;
    }
    f32x4 s[KG][4], dp[KG][4];
    // query sub-tiles in pairs when one key group leaves two chains per sub-tile (attn_bwd_dq2_kernel)
    constexpr int TP = KG == 1 ? 2 : 1;
#pragma unroll
    for (int tp = 0; tp < 4; tp += TP) {
#pragma unroll
      for (int t = tp; t < tp + TP; ++t)
#pragma unroll
        for (int kg = 0; kg < KG; ++kg) s[kg][t] = dp[kg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        mbf16x8 qf[TP], df[TP];
#pragma unroll
        for (int u = 0; u < TP; ++u) {
          qf[u] = frag_row<D>(Qr, 16 * (tp + u), ks, lane);
          df[u] = frag_row<D>(Dr, 16 * (tp + u), ks, lane);
        }
#pragma unroll
        for (int kg = 0; kg < KG; ++kg)
#pragma unroll
          for (int u = 0; u < TP; ++u) {
            s[kg][tp + u] = mfma(qf[u], kf[kg][ks], s[kg][tp + u]);  // S^T: [q][kv = lane]
            dp[kg][tp + u] = mfma(df[u], vf[kg][ks], dp[kg][tp + u]);
          }
      }
    }
    const bool need_mask = q0 + BQ > T || kvbase + 16 * KG - 1 >= T || (p.causal && kvbase + 16 * KG - 1 > q0);
    // Per 32-query half cc: P, the mask (masked tiles only: branch-free selects under one branch), dS,
    // the bf16 packs and the half's dV / dK MFMAs — the second half's exponentials are independent of the
    // first half's MFMAs, so they can issue in their shadow (a per-element masked test had compiled into
    // 32 scalar branches interleaved with the exponentials).
    mbf16x8 pf[2][KG], sf[2][KG];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
#pragma unroll
      for (int t = 2 * cc; t < 2 * cc + 2; ++t) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(s_lse + 16 * t + 4 * g);  // 4 consecutive queries
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) s[kg][t][r] = fast_exp2(fmaf(s[kg][t][r], c, -l4[r]));
      }
      if (need_mask) {
#pragma unroll
        for (int t = 2 * cc; t < 2 * cc + 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = q0 + 16 * t + 4 * g + r;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
              const int kvrow = kvbase + 16 * kg + (lane & 15);
              const bool dead = (q >= T) | (kvrow >= T) | (p.causal & (kvrow > q));
              s[kg][t][r] = dead ? 0.f : s[kg][t][r];
            }
          }
      }
#pragma unroll
      for (int t = 2 * cc; t < 2 * cc + 2; ++t) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(s_dl + 16 * t + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) dp[kg][t][r] = s[kg][t][r] * (dp[kg][t][r] - d4[r]);  // dS
      }
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        pf[cc][kg] = pack_p(s[kg][2 * cc], s[kg][2 * cc + 1]);
        sf[cc][kg] = pack_p(dp[kg][2 * cc], dp[kg][2 * cc + 1]);
      }
      if constexpr (FQ) {  // dS^T -> LDS: key row kl, queries 16 t + 4 g .. +3 (one 8-byte store each)
        const int kl = w * 16 * KG + (lane & 15);
        const int sw = (kl >> 1) & 3;
        char* const rowp = DSt + kl * (BQ * 2) + 8 * g;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          char* const a = rowp + (((2 * cc + h) ^ sw) << 5);
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            const s16x8 v = __builtin_bit_cast(s16x8, sf[cc][kg]);
            *reinterpret_cast<s16x4*>(a + kg * 16 * (BQ * 2)) =
                h ? s16x4{v[4], v[5], v[6], v[7]} : s16x4{v[0], v[1], v[2], v[3]};
          }
        }
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const mbf16x8 dtf = frag_tr<D>(Dt, 32 * cc, 16 * dt, lane);
        const mbf16x8 qtf = frag_tr<D>(Qt, 32 * cc, 16 * dt, lane);
#pragma unroll
        for (int kg = 0; kg < KG; ++kg) {
          dv[kg][dt] = mfma(dtf, pf[cc][kg], dv[kg][dt]);
          dk[kg][dt] = mfma(qtf, sf[cc][kg], dk[kg][dt]);
        }
      }
    }
    if constexpr (FQ) fused_dq<D, BK, FQ == 1>(p, DSt, Kt, dqa, q0, p.causal ? q0 + BQ - kt * BK : BK, w, lane);
    if constexpr (DB) __syncthreads();
  }
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    const int kvrow = kvbase + 16 * kg + (lane & 15);
    if (kvrow >= T) continue;
    if (G == 1) {
      bf16_t* dkp = p.dk + b * p.dk_sb + (int64_t)kvrow * p.dk_st + hk * p.dk_sh;
      bf16_t* dvp = p.dv + b * p.dv_sb + (int64_t)kvrow * p.dv_st + hk * p.dv_sh;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        u16x4 a, v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = f2bf(dk[kg][dt][r] * p.scale);
          v[r] = f2bf(dv[kg][dt][r]);
        }
        *reinterpret_cast<u16x4*>(dkp + 16 * dt + 4 * g) = a;
        *reinterpret_cast<u16x4*>(dvp + 16 * dt + 4 * g) = v;
      }
      continue;
    }
    const int64_t plane = (int64_t)p.B * p.Hq * T * D;
    float* pk = p.dkv_part + (((int64_t)b * p.Hq + hq) * T + kvrow) * D;
    float* pv = pk + plane;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      f32x4 a = dk[kg][dt] * p.scale;
      *reinterpret_cast<f32x4*>(pk + 16 * dt + 4 * g) = a;
      *reinterpret_cast<f32x4*>(pv + 16 * dt + 4 * g) = dv[kg][dt];
    }
  }
}

// dK/dV = sum over the G query heads of a KV head of the fp32 partials (8 columns per thread)
__global__ void __launch_bounds__(NT) attn_dkv_reduce_kernel(AttnParams p) {
  const int D = p.D, T = p.T, G = p.Hq / p.Hkv;
  const int64_t n8 = (int64_t)p.B * p.Hkv * T * (D / 8);
  const int64_t plane = (int64_t)p.B * p.Hq * T * D;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n8; i += stride) {
    const int which = i >= n8;  // 0: dK, 1: dV
    int64_t r = which ? i - n8 : i;
    const int c8 = (int)(r % (D / 8));
    r /= D / 8;
    const int t = (int)(r % T);
    r /= T;
    const int hk = (int)(r % p.Hkv);
    const int b = (int)(r / p.Hkv);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int gq = 0; gq < G; ++gq) {
      const float* src = p.dkv_part + which * plane + (((int64_t)b * p.Hq + hk * G + gq) * T + t) * D + c8 * 8;
      float v[8];
      load8(src, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    bf16_t* dst = which ? p.dv + b * p.dv_sb + (int64_t)t * p.dv_st + hk * p.dv_sh
                        : p.dk + b * p.dk_sb + (int64_t)t * p.dk_st + hk * p.dk_sh;
    store8(dst + c8 * 8, acc);
  }
}

// query groups per wave of the forward kernel (PDA_ATTN_FWD_QG=1|2 overrides).  Measured
// (profiles/r1_attn_microbench_v3.jsonl, profiles/r2_attn_fwd3.jsonl): 2 groups for both head dims —
// D = 64 287 vs 259 TFLOP/s; D = 128 with the double-buffered v3 kernel 406 vs 383 (v2: a tie).
int attn_fwd_groups(int D) {
  static const int env = [] {
    const char* e = getenv("PDA_ATTN_FWD_QG");
    return e ? atoi(e) : 0;
  }();
  if (env == 1 || env == 2 || env == 4) return env;
  (void)D;
  return 2;
}

// forward kernel generation: 3 (default) double-buffered K/V, one barrier per tile; 2 single stage
int attn_fwd_version() {
  static const int v = [] {
    const char* e = getenv("PDA_ATTN_FWD");
    return e ? atoi(e) : 4;
  }();
  return v;
}

}  // namespace

hipError_t attention_fwd(const AttnParams& p, hipStream_t st) {
  if (p.D != 64 && p.D != 128) return hipErrorInvalidValue;
  if (p.Hkv <= 0 || p.Hq % p.Hkv) return hipErrorInvalidValue;
  if (p.rope_cos == nullptr) {
    // v4 (default): buffer-descriptor K/V loads need the [T][row stride] spans to fit 31-bit offsets
    const bool v4_ok = (int64_t)p.T * p.k_st * 2 < ((int64_t)1 << 31) && (int64_t)p.T * p.v_st * 2 < ((int64_t)1 << 31);
    int qg = attn_fwd_groups(p.D);
    if (qg == 4 && !(attn_fwd_version() == 4 && v4_ok)) qg = 2;  // (4 groups: v4 only)
    dim3 grid((p.T + 64 * qg - 1) / (64 * qg), p.Hq, p.B);
    if (attn_fwd_version() == 2) {
      if (p.D == 128) {
        if (qg == 1) attn_fwd2_kernel<128, 1><<<grid, NT, 0, st>>>(p);
        else attn_fwd2_kernel<128, 2><<<grid, NT, 0, st>>>(p);
      } else {
        if (qg == 1) attn_fwd2_kernel<64, 1><<<grid, NT, 0, st>>>(p);
        else attn_fwd2_kernel<64, 2><<<grid, NT, 0, st>>>(p);
      }
      return hipGetLastError();
    }
    if (attn_fwd_version() == 4 && v4_ok) {
      if (qg == 4) {  // PDA_ATTN_FWD_QG=4: 64 query rows per wave at one wave per SIMD (half the K/V LDS
                      // reads per MFMA; O in AGPRs)
        const dim3 g4((p.T + 255) / 256, p.Hq, p.B);
        if (p.D == 128) attn_fwd4_kernel<128, 4, 1><<<g4, NT, 0, st>>>(p);
        else attn_fwd4_kernel<64, 4, 1><<<g4, NT, 0, st>>>(p);
        return hipGetLastError();
      }
      if (p.D == 128) {
        if (qg == 1) attn_fwd4_kernel<128, 1><<<grid, NT, 0, st>>>(p);
        else attn_fwd4_kernel<128, 2><<<grid, NT, 0, st>>>(p);
      } else {
        if (qg == 1) attn_fwd4_kernel<64, 1><<<grid, NT, 0, st>>>(p);
        else attn_fwd4_kernel<64, 2><<<grid, NT, 0, st>>>(p);
      }
      return hipGetLastError();
    }
    if (p.D == 128) {
      if (qg == 1) attn_fwd3_kernel<128, 1><<<grid, NT, 0, st>>>(p);
      else attn_fwd3_kernel<128, 2><<<grid, NT, 0, st>>>(p);
    } else {
      if (qg == 1) attn_fwd3_kernel<64, 1><<<grid, NT, 0, st>>>(p);
      else attn_fwd3_kernel<64, 2><<<grid, NT, 0, st>>>(p);
    }
    return hipGetLastError();
  }
  dim3 grid((p.T + BQ - 1) / BQ, p.Hq, p.B);
  if (p.D == 128) attn_fwd_kernel<128><<<grid, NT, 0, st>>>(p);
  else attn_fwd_kernel<64><<<grid, NT, 0, st>>>(p);
  return hipGetLastError();
}

int64_t attention_bwd_ws_floats(int B, int T, int Hq, int Hkv, int D, bool rope) {
  return (!rope && Hq > Hkv) ? (int64_t)2 * B * Hq * T * D : 0;
}

// PDA_ATTN_BWD_FUSED bit 0: fused dK/dV/dQ kernel at D = 64, bit 1: at D = 128 (else the dQ kernel +
// dK/dV kernel pair); bit 4: lab store mode (plain stores instead of the dQ atomics — wrong dQ, prices
// the atomics).  Measured (profiles/r5_attn_bwd_fused.jsonl): GPT-2-medium 326.1 / 321.8 k vs 315.3 /
// 318.1 k tok/s on one box; microbench backward 0.4065 vs 0.4176 ms (atomics ~0.05 ms of it).  At
// D = 128 the fused kernel needs 88.5 KB of LDS (one workgroup per CU): Llama-3-8B 16.9 k vs 18.6 k, off.
// Round 6: after the branch-free masking and the paired S / dP chains the pair overtook the fused kernel at
// D = 64 too (microbench 0.341 vs 0.379 ms, GPT-2-medium 322.5-322.7 k vs 321.4-321.5 k tok/s on one box,
// profiles/r6_attn_bwd_pair_vs_fused.jsonl), so the default is the pair — also atomic-free, i.e.
// run-to-run deterministic without PDA_DETERMINISTIC.
int& attention_bwd_fused_mode() {
  static int mode = [] {
    const char* e = getenv("PDA_ATTN_BWD_FUSED");
    return e ? atoi(e) : 0;
  }();
  return mode;
}
// PDA_DETERMINISTIC=1 (nn.py:deterministic, read per call so a process can switch) turns the fused kernel
// off: its dQ is summed by fp32 atomics in key-tile arrival order, the dQ + dK/dV pair has no atomics.
static bool deterministic_mode() {
  const char* e = getenv("PDA_DETERMINISTIC");
  return e != nullptr && e[0] == '1';
}
bool attention_bwd_fused(int D, bool rope) {
  return !rope && (attention_bwd_fused_mode() & (D == 64 ? 1 : 2)) != 0 && !deterministic_mode();
}

hipError_t attention_bwd(const AttnParams& p, hipStream_t st) {
  if (p.D != 64 && p.D != 128) return hipErrorInvalidValue;
  if (p.Hkv <= 0 || p.Hq % p.Hkv) return hipErrorInvalidValue;
  const int64_t rows = (int64_t)p.B * p.Hq * p.T;
  const int rows_per_block = DRPT * NT / (p.D / 8);
  const unsigned dgrid = (unsigned)((rows + rows_per_block - 1) / rows_per_block);
  if (p.D == 128) attn_bwd_delta_kernel<128><<<dgrid, NT, 0, st>>>(p);
  else attn_bwd_delta_kernel<64><<<dgrid, NT, 0, st>>>(p);
  PDA_CHECK_HIP(hipGetLastError());
  dim3 gq((p.T + BQ - 1) / BQ, p.Hq, p.B);
  if (p.rope_cos == nullptr) {
    dim3 gq2((p.T + 2 * BQ - 1) / (2 * BQ), p.Hq, p.B);
    if (p.Hq > p.Hkv && p.dkv_part == nullptr) return hipErrorInvalidValue;
    if (p.dq_acc != nullptr) {  // fused dK / dV / dQ (attention_bwd_fused)
      const bool lab_store = (attention_bwd_fused_mode() & 16) != 0;
      if (p.D == 128) {
        const dim3 gk((p.T + BKV - 1) / BKV, p.Hq, p.B);
        attn_bwd_dkdv2_kernel<128, 1, false, 1><<<gk, NT, 0, st>>>(p);
      } else {
        const dim3 gk((p.T + 2 * BKV - 1) / (2 * BKV), p.Hq, p.B);
        if (lab_store) attn_bwd_dkdv2_kernel<64, 2, false, 2><<<gk, NT, 0, st>>>(p);
        else attn_bwd_dkdv2_kernel<64, 2, false, 1><<<gk, NT, 0, st>>>(p);
      }
      PDA_CHECK_HIP(hipGetLastError());
      const int64_t n8 = (int64_t)p.B * p.Hq * p.T * (p.D / 8);
      int64_t g = (n8 + 4 * NT - 1) / (4 * NT);
      if (g > 4096) g = 4096;
      attn_dq_convert_kernel<<<(unsigned)g, NT, 0, st>>>(p);
      PDA_CHECK_HIP(hipGetLastError());
      if (p.Hq > p.Hkv) {
        const int64_t m8 = (int64_t)2 * p.B * p.Hkv * p.T * (p.D / 8);
        int64_t gm = (m8 + NT - 1) / NT;
        if (gm > 8192) gm = 8192;
        attn_dkv_reduce_kernel<<<(unsigned)gm, NT, 0, st>>>(p);
      }
      return hipGetLastError();
    }
    static const int db = [] {  // bit 0: dQ kernel double-buffered, bit 1: dK/dV kernel
      const char* e = getenv("PDA_ATTN_BWD_DB");
      return e ? atoi(e) : 0;
    }();
    static const int g128 = [] {  // PDA_ATTN_BWD128 bit 0: dQ kernel with 2 query groups, bit 1: dK/dV
      const char* e = getenv("PDA_ATTN_BWD128");  // kernel with 2 key groups (both at one wave per SIMD,
      return e ? atoi(e) : 0;                      // double-buffered: half the LDS bytes per MFMA)
    }();
    if (p.D == 128) {  // (two groups per wave exceed the 256-register budget of 2 waves per SIMD at D = 128)
      if (g128 & 1) attn_bwd_dq2_kernel<128, 2, true, 1><<<gq2, NT, 0, st>>>(p);
      else if (db & 1) attn_bwd_dq2_kernel<128, 1, true><<<gq, NT, 0, st>>>(p);
      else attn_bwd_dq2_kernel<128, 1><<<gq, NT, 0, st>>>(p);
      const dim3 gk((p.T + BKV - 1) / BKV, p.Hq, p.B);
      const dim3 gk2((p.T + 2 * BKV - 1) / (2 * BKV), p.Hq, p.B);
      if (g128 & 2) attn_bwd_dkdv2_kernel<128, 2, true, 0, 1><<<gk2, NT, 0, st>>>(p);
      else if (db & 2) attn_bwd_dkdv2_kernel<128, 1, true><<<gk, NT, 0, st>>>(p);
      else attn_bwd_dkdv2_kernel<128, 1><<<gk, NT, 0, st>>>(p);
    } else {
      // PDA_ATTN_BWD_G64=1: one query / key group per wave at D = 64 (140 / 159 VGPRs: 3 waves per SIMD
      // instead of 2, half the fragment reuse) — GPT-2-medium 323.3-324.6k vs 323.1-323.6k tok/s, a tie
      // (profiles/r4_attn_bwd_g64_ab.jsonl); A/B knob
      static const int g1 = [] {
        const char* e = getenv("PDA_ATTN_BWD_G64");
        return e && e[0] == '1' ? 1 : 0;
      }();
      if (g1) {
        attn_bwd_dq2_kernel<64, 1><<<gq, NT, 0, st>>>(p);
        const dim3 gk1((p.T + BKV - 1) / BKV, p.Hq, p.B);
        attn_bwd_dkdv2_kernel<64, 1><<<gk1, NT, 0, st>>>(p);
      } else {
        if (db & 1) attn_bwd_dq2_kernel<64, 2, true><<<gq2, NT, 0, st>>>(p);
        else attn_bwd_dq2_kernel<64, 2><<<gq2, NT, 0, st>>>(p);
        const dim3 gk((p.T + 2 * BKV - 1) / (2 * BKV), p.Hq, p.B);
        if (db & 2) attn_bwd_dkdv2_kernel<64, 2, true><<<gk, NT, 0, st>>>(p);
        else attn_bwd_dkdv2_kernel<64, 2><<<gk, NT, 0, st>>>(p);
      }
    }
    PDA_CHECK_HIP(hipGetLastError());
    if (p.Hq > p.Hkv) {
      const int64_t n8 = (int64_t)2 * p.B * p.Hkv * p.T * (p.D / 8);
      int64_t g = (n8 + NT - 1) / NT;
      if (g > 8192) g = 8192;
      attn_dkv_reduce_kernel<<<(unsigned)g, NT, 0, st>>>(p);
    }
    return hipGetLastError();
  }
  dim3 gk((p.T + BKV - 1) / BKV, p.Hkv, p.B);
  if (p.D == 128) {
    attn_bwd_dq_kernel<128><<<gq, NT, 0, st>>>(p);
    attn_bwd_dkdv_kernel<128><<<gk, NT, 0, st>>>(p);
  } else {
    attn_bwd_dq_kernel<64><<<gq, NT, 0, st>>>(p);
    attn_bwd_dkdv_kernel<64><<<gk, NT, 0, st>>>(p);
  }
  return hipGetLastError();
}

}  // namespace pda
