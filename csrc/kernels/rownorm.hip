// Row normalisations for the transformer configs (SURVEY §2.5 K19 LayerNorm — GPT-2, K20 RMSNorm —
// Llama-3) and the column reductions they need.  x: [rows, D] (fp32 or bf16, D % 8 == 0, D <= 8192),
// gamma/beta: [D].
//
// Layout on CDNA4: one 64-lane wavefront per row (4 rows per 256-thread workgroup), so every row
// reduction is a register/DPP shuffle reduction with no LDS and no barrier; lane l owns the 8-wide
// column vectors l, l+64, ... (VPL = ceil(D/512) of them, a template parameter).  The row stays in
// registers between the statistics and the output pass when VPL <= 4 (D <= 2048: GPT-2 medium/XL);
// wider rows re-read the (L2-resident) row instead of spilling.
//
// Parameter gradients (dgamma = sum_r dy*xhat, dbeta = sum_r dy) are NOT accumulated with atomics
// from the row kernel (2K-deep same-address contention): a column-strip kernel writes per-slab
// partials and a finalize kernel sums the slabs — the same slab scheme as the BatchNorm kernels.
#include "pda_common.h"
#include "pda_kernels.h"

#include <type_traits>

namespace pda {
namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerBlock = kThreads / 64;

template <typename T, typename P, bool RMS, int VPL>
__global__ void __launch_bounds__(kThreads) rownorm_fwd_kernel(const T* __restrict__ x, const P* __restrict__ gamma,
                                                               const P* __restrict__ beta, T* __restrict__ y,
                                                               float* __restrict__ mean_out,
                                                               float* __restrict__ rstd_out, int64_t rows, int64_t D,
                                                               float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * D;
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
      load8(xr + c, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = RMS ? 0.f : wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
      float g[8], b[8], o[8];
      load8(gamma + c, g);
      if (!RMS) load8(beta + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + (RMS ? 0.f : b[j]);
      store8(y + row * D + c, o);
    }
  }
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat))        (LayerNorm)
// dx = rstd * (g*dy - xhat * mean(g*dy*xhat))                      (RMSNorm)
template <typename T, typename P, bool RMS, int VPL>
__global__ void __launch_bounds__(kThreads) rownorm_bwd_dx_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                  const P* __restrict__ gamma,
                                                                  const float* __restrict__ mean_in,
                                                                  const float* __restrict__ rstd_in,
                                                                  T* __restrict__ dx, int64_t rows, int64_t D,
                                                                  const T* __restrict__ addend) {
  constexpr bool kKeep = VPL <= 4;
  constexpr int KV = kKeep ? VPL : 1;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float mean = RMS ? 0.f : mean_in[row], rstd = rstd_in[row];
  const T* xr = x + row * D;
  const T* dyr = dy + row * D;
  float xh[KV][8], gd[KV][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
      float xv[8], d[8], g[8];
      load8(xr + c, xv);
      load8(dyr + c, d);
      load8(gamma + c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (xv[j] - mean) * rstd, q = g[j] * d[j];
        s1 += q;
        s2 += q * h;
        if constexpr (kKeep) {
          xh[i][j] = h;
          gd[i][j] = q;
        }
      }
    }
  }
  const float m1 = RMS ? 0.f : wave_sum(s1) / (float)D;
  const float m2 = wave_sum(s2) / (float)D;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
      float o[8];
      if constexpr (kKeep) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (gd[i][j] - m1 - xh[i][j] * m2);
      } else {
        float xv[8], d[8], g[8];
        load8(xr + c, xv);
        load8(dyr + c, d);
        load8(gamma + c, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[j] * d[j] - m1 - (xv[j] - mean) * rstd * m2);
      }
      if (addend) {  // the residual stream's own gradient (fused add + norm): dx = norm_bwd(dy) + dh
        float a[8];
        load8(addend + row * D + c, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += a[j];
      }
      store8(dx + row * D + c, o);
    }
  }
}

// Fused backward (rows stay in registers, D <= 2048): workgroup = one row slab of ws_rows rows, each
// wave walks every 4th row of it writing dx, and the lanes keep the parameter-gradient partials of
// their own columns (sum dy * xhat, sum dy) across the slab — the column sums need no second pass over
// dy and x (colstrip_partial_kernel).  The 4 waves meet in LDS and write one slab partial per column.
template <typename T, typename P, bool RMS, int VPL>
__global__ void __launch_bounds__(kThreads) rownorm_bwd_fused_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                     const P* __restrict__ gamma,
                                                                     const float* __restrict__ mean_in,
                                                                     const float* __restrict__ rstd_in,
                                                                     T* __restrict__ dx, int64_t rows, int64_t D,
                                                                     const T* __restrict__ addend, float* __restrict__ ws,
                                                                     int64_t rows_per_slab, int nslab) {
  static_assert(VPL <= 4, "rows kept in registers");
  __shared__ float red[kRowsPerBlock - 1][2][2048];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_slab;
  const int64_t r1 = min(rows, r0 + rows_per_slab);
  float g[VPL][8], pg[VPL][8], pb[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) load8(gamma + c, g[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) pg[i][j] = pb[i][j] = 0.f;
  }
  for (int64_t row = r0 + w; row < r1; row += kRowsPerBlock) {
    const float mean = RMS ? 0.f : mean_in[row], rstd = rstd_in[row];
    const T* xr = x + row * D;
    const T* dyr = dy + row * D;
    float xh[VPL][8], gd[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int64_t c = ((int64_t)i * 64 + lane) * 8;
      if (c < D) {
        float xv[8], d[8];
        load8(xr + c, xv);
        load8(dyr + c, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float h = (xv[j] - mean) * rstd, q = g[i][j] * d[j];
          s1 += q;
          s2 += q * h;
          xh[i][j] = h;
          gd[i][j] = q;
          pg[i][j] = fmaf(d[j], h, pg[i][j]);
          pb[i][j] += d[j];
        }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / (float)D;
    const float m2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int64_t c = ((int64_t)i * 64 + lane) * 8;
      if (c < D) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (gd[i][j] - m1 - xh[i][j] * m2);
        if (addend) {
          float a[8];
          load8(addend + row * D + c, a);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += a[j];
        }
        store8(dx + row * D + c, o);
      }
    }
  }
  // waves 1..3 hand their partials to wave 0 through LDS; wave 0 writes the slab row
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red[w - 1][0][c + j] = pg[i][j];
          red[w - 1][1][c + j] = pb[i][j];
        }
      }
    }
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int k = 0; k < kRowsPerBlock - 1; ++k) {
            pg[i][j] += red[k][0][c + j];
            pb[i][j] += red[k][1][c + j];
          }
        }
        store8(ws + (int64_t)blockIdx.x * D + c, pg[i]);
        if (!RMS) store8(ws + ((int64_t)nslab + blockIdx.x) * D + c, pb[i]);
      }
    }
  }
}

// PDA_ROWNORM_FUSED_BWD=1 selects it.  Measured neutral on GPT-2-medium (311.3k vs 311.2k tok/s,
// profiles/r2_rownorm_fused_bwd_ab_v32.jsonl): the saved pass over dy and x is paid back by the fewer
// rows in flight per wave (512 slab workgroups instead of one workgroup per 4 rows), so the default
// stays the row kernel + column-strip pass.
bool rownorm_fused_bwd_on() {
  static const bool on = [] {
    const char* e = getenv("PDA_ROWNORM_FUSED_BWD");
    return e && e[0] == '1';
  }();
  return on;
}

// ------------------------------------------------------------------ column-strip reductions
// Block = 64 column vectors (512 columns) x 4 row lanes; blockIdx.y = row slab.  Each block writes
// its slab partial(s) to ws[k][slab][col]; colreduce_finalize sums the slabs.
constexpr int kStripCols = 512;

template <typename T, bool LN_GRAD, bool RMS>
__global__ void __launch_bounds__(kThreads) colstrip_partial_kernel(const T* __restrict__ a, const T* __restrict__ x,
                                                                    const float* __restrict__ mean_in,
                                                                    const float* __restrict__ rstd_in,
                                                                    float* __restrict__ ws, int64_t rows, int64_t D,
                                                                    int64_t rows_per_slab, int nslab) {
  __shared__ float red[2][4][kStripCols + 4];
  const int cv = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * kStripCols + cv * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
  const int64_t r1 = min(rows, r0 + rows_per_slab);
  float acc0[8], acc1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc0[j] = acc1[j] = 0.f;
  if (c < D) {
    for (int64_t r = r0 + rl; r < r1; r += 4) {
      float d[8];
      load8(a + r * D + c, d);
      if constexpr (LN_GRAD) {
        float xv[8];
        load8(x + r * D + c, xv);
        const float mean = RMS ? 0.f : mean_in[r], rstd = rstd_in[r];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc0[j] += d[j] * (xv[j] - mean) * rstd;
          acc1[j] += d[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc0[j] += d[j];
      }
    }
  }
  constexpr int NOUT = (LN_GRAD && !RMS) ? 2 : 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][rl][cv * 8 + j] = acc0[j];
    if (NOUT == 2) red[1][rl][cv * 8 + j] = acc1[j];
  }
  __syncthreads();
  // 256 threads finalize 512 columns x NOUT outputs
  for (int t = threadIdx.x; t < kStripCols * NOUT; t += kThreads) {
    const int k = t / kStripCols, col = t % kStripCols;
    const int64_t gc = (int64_t)blockIdx.x * kStripCols + col;
    if (gc >= D) continue;
    const float s = red[k][0][col] + red[k][1][col] + red[k][2][col] + red[k][3][col];
    ws[((int64_t)k * nslab + blockIdx.y) * D + gc] = s;
  }
}

// out_k[col] = sum_s ws[k][s][col].  A workgroup is 64 columns x 16 slab lanes with 8 loads in flight
// per lane: the slabs were just written (L2 / MALL hits), so depth of outstanding loads, not bytes,
// sets the time.  (One thread per column walking ~512 slabs 4 loads deep took ~30 us per call on the
// GPT-2 bias / LayerNorm gradients.)
constexpr int kFinCols = 64, kFinLanes = 16;
// (out_bf16: the outputs are written as bf16 — straight into a bf16 parameter's gradient slot)
__global__ void __launch_bounds__(kFinCols * kFinLanes) colreduce_finalize_kernel(const float* __restrict__ ws,
                                                                                  int nslab, int64_t D, int nout,
                                                                                  void* __restrict__ out0,
                                                                                  void* __restrict__ out1,
                                                                                  int out_bf16) {
  __shared__ float red[kFinLanes][kFinCols];
  const int cl = threadIdx.x % kFinCols, lane = threadIdx.x / kFinCols;
  const int64_t t = (int64_t)blockIdx.x * kFinCols + cl;  // output index over nout x D
  const bool ok = t < D * nout;
  const int k = ok ? (int)(t / D) : 0;
  const int64_t col = ok ? t % D : 0;
  const float* p = ws + (int64_t)k * nslab * D + col;
  float a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = 0.f;
  if (ok) {
    int s = lane;
    for (; s + 7 * kFinLanes < nslab; s += 8 * kFinLanes) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += p[(int64_t)(s + u * kFinLanes) * D];
    }
    for (; s < nslab; s += kFinLanes) a[0] += p[(int64_t)s * D];
  }
  red[lane][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (lane != 0 || !ok) return;
  float r = 0.f;
#pragma unroll
  for (int l = 0; l < kFinLanes; ++l) r += red[l][cl];
  void* o = k == 0 ? out0 : out1;
  if (out_bf16) static_cast<bf16_t*>(o)[col] = f2bf(r);
  else static_cast<float*>(o)[col] = r;
}

inline unsigned fin_grid(int64_t n) { return (unsigned)((n + kFinCols - 1) / kFinCols); }

int plan_slabs(int64_t rows, int64_t D) {
  const int64_t strips = (D + kStripCols - 1) / kStripCols;
  int64_t nslab = 1024 / strips;                 // ~4 workgroups per CU
  const int64_t max_by_rows = (rows + 31) / 32;  // >= 32 rows (8 per row lane) per slab
  if (nslab > max_by_rows) nslab = max_by_rows;
  if (nslab < 1) nslab = 1;
  return (int)nslab;
}

// Residual add fused into the next norm — h = x + r (rounded to bf16, as the unfused add would store
// it) is written once and normalised from registers (one HBM pass instead of add + norm).  Serving
// passes no statistics buffers; training stores mean / rstd of h for the backward.
template <bool RMS, int VPL>
__global__ void __launch_bounds__(kThreads) add_rownorm_fwd_kernel(const bf16_t* __restrict__ x,
                                                                   const bf16_t* __restrict__ r,
                                                                   const bf16_t* __restrict__ gamma,
                                                                   const bf16_t* __restrict__ beta,
                                                                   bf16_t* __restrict__ h, bf16_t* __restrict__ y,
                                                                   int64_t rows, int64_t D, float eps,
                                                                   float* __restrict__ mean_out,
                                                                   float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
      float a[8], b[8];
      load8(x + row * D + c, a);
      load8(r + row * D + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f(f2bf(a[j] + b[j]));
        s += v[i][j];
      }
      store8(h + row * D + c, v[i]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = RMS ? 0.f : wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int64_t c = ((int64_t)i * 64 + lane) * 8;
    if (c < D) {
      float g[8], b[8], o[8];
      load8(gamma + c, g);
      if (!RMS) load8(beta + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + (RMS ? 0.f : b[j]);
      store8(y + row * D + c, o);
    }
  }
  if (rstd_out && lane == 0) {  // training: the backward's statistics of h
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <typename F>
void dispatch_vpl(int64_t D, F&& f) {
  const int64_t vpl = (D + 511) / 512;
  if (vpl <= 1) f(std::integral_constant<int, 1>{});
  else if (vpl <= 2) f(std::integral_constant<int, 2>{});
  else if (vpl <= 4) f(std::integral_constant<int, 4>{});
  else if (vpl <= 8) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}

}  // namespace

hipError_t add_rownorm_fwd(const bf16_t* x, const bf16_t* r, const bf16_t* gamma, const bf16_t* beta, bf16_t* h,
                           bf16_t* y, int64_t rows, int64_t D, float eps, bool rms, hipStream_t st, float* mean,
                           float* rstd) {
  if (rows == 0) return hipSuccess;
  const unsigned grid = (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  dispatch_vpl(D, [&](auto vc) {
    constexpr int V = decltype(vc)::value;
    if (rms) add_rownorm_fwd_kernel<true, V><<<grid, kThreads, 0, st>>>(x, r, gamma, beta, h, y, rows, D, eps, mean, rstd);
    else add_rownorm_fwd_kernel<false, V><<<grid, kThreads, 0, st>>>(x, r, gamma, beta, h, y, rows, D, eps, mean, rstd);
  });
  return hipGetLastError();
}

int64_t colreduce_ws_floats(int64_t rows, int64_t D, int nout) { return (int64_t)nout * plan_slabs(rows, D) * D; }

hipError_t rownorm_fwd(const void* x, bool x_bf16, const void* gamma, const void* beta, bool p_bf16, void* y,
                       float* mean, float* rstd, int64_t rows, int64_t D, float eps, bool rms, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  const unsigned grid = (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  dispatch_vpl(D, [&](auto vc) {
    constexpr int V = decltype(vc)::value;
#define L(T, P, R) \
  rownorm_fwd_kernel<T, P, R, V><<<grid, kThreads, 0, st>>>((const T*)x, (const P*)gamma, (const P*)beta, (T*)y, mean, rstd, rows, D, eps)
    if (rms) {
      if (x_bf16 && p_bf16) L(bf16_t, bf16_t, true);
      else if (x_bf16) L(bf16_t, float, true);
      else if (p_bf16) L(float, bf16_t, true);
      else L(float, float, true);
    } else {
      if (x_bf16 && p_bf16) L(bf16_t, bf16_t, false);
      else if (x_bf16) L(bf16_t, float, false);
      else if (p_bf16) L(float, bf16_t, false);
      else L(float, float, false);
    }
#undef L
  });
  return hipGetLastError();
}

hipError_t rownorm_bwd(const void* dy, const void* x, bool x_bf16, const void* gamma, bool p_bf16, const float* mean,
                       const float* rstd, void* dx, void* dgamma, void* dbeta, bool dparam_bf16, int64_t rows,
                       int64_t D, bool rms, float* ws, hipStream_t st, const void* addend) {
  const int ob = dparam_bf16 ? 1 : 0;
  const size_t osz = dparam_bf16 ? 2 : 4;
  if (rows == 0) {
    PDA_CHECK_HIP(hipMemsetAsync(dgamma, 0, D * osz, st));
    if (!rms) PDA_CHECK_HIP(hipMemsetAsync(dbeta, 0, D * osz, st));
    return hipSuccess;
  }
  const int nslab = plan_slabs(rows, D);
  const int64_t rps = (rows + nslab - 1) / nslab;
  if (rownorm_fused_bwd_on() && D <= 2048) {
    // one pass: dx plus the slab partials of dgamma / dbeta (ws sized by colreduce_ws_floats)
    dispatch_vpl(D, [&](auto vc) {
      constexpr int V = decltype(vc)::value;
      if constexpr (V <= 4) {
#define L(T, P, R) \
  rownorm_bwd_fused_kernel<T, P, R, V><<<(unsigned)nslab, kThreads, 0, st>>>((const T*)dy, (const T*)x, (const P*)gamma, mean, rstd, (T*)dx, rows, D, (const T*)addend, ws, rps, nslab)
        if (rms) {
          if (x_bf16 && p_bf16) L(bf16_t, bf16_t, true);
          else if (x_bf16) L(bf16_t, float, true);
          else if (p_bf16) L(float, bf16_t, true);
          else L(float, float, true);
        } else {
          if (x_bf16 && p_bf16) L(bf16_t, bf16_t, false);
          else if (x_bf16) L(bf16_t, float, false);
          else if (p_bf16) L(float, bf16_t, false);
          else L(float, float, false);
        }
#undef L
      }
    });
    PDA_CHECK_HIP(hipGetLastError());
    const int nout = rms ? 1 : 2;
    colreduce_finalize_kernel<<<fin_grid(D * nout), kFinCols * kFinLanes, 0, st>>>(ws, nslab, D, nout, dgamma, dbeta, ob);
    return hipGetLastError();
  }
  const unsigned grid = (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  dispatch_vpl(D, [&](auto vc) {
    constexpr int V = decltype(vc)::value;
#define L(T, P, R) \
  rownorm_bwd_dx_kernel<T, P, R, V><<<grid, kThreads, 0, st>>>((const T*)dy, (const T*)x, (const P*)gamma, mean, rstd, (T*)dx, rows, D, (const T*)addend)
    if (rms) {
      if (x_bf16 && p_bf16) L(bf16_t, bf16_t, true);
      else if (x_bf16) L(bf16_t, float, true);
      else if (p_bf16) L(float, bf16_t, true);
      else L(float, float, true);
    } else {
      if (x_bf16 && p_bf16) L(bf16_t, bf16_t, false);
      else if (x_bf16) L(bf16_t, float, false);
      else if (p_bf16) L(float, bf16_t, false);
      else L(float, float, false);
    }
#undef L
  });
  PDA_CHECK_HIP(hipGetLastError());
  dim3 pg((unsigned)((D + kStripCols - 1) / kStripCols), (unsigned)nslab);
#define P(T, R) \
  colstrip_partial_kernel<T, true, R><<<pg, kThreads, 0, st>>>((const T*)dy, (const T*)x, mean, rstd, ws, rows, D, rps, nslab)
  if (x_bf16) {
    if (rms) P(bf16_t, true); else P(bf16_t, false);
  } else {
    if (rms) P(float, true); else P(float, false);
  }
#undef P
  PDA_CHECK_HIP(hipGetLastError());
  const int nout = rms ? 1 : 2;
  colreduce_finalize_kernel<<<fin_grid(D * nout), kFinCols * kFinLanes, 0, st>>>(ws, nslab, D, nout, dgamma, dbeta, ob);
  return hipGetLastError();
}

// Column sums of a [rows, cols] matrix (bias gradients): out[c] = sum_r x[r, c] (fp32 or bf16 out), cols % 8 == 0.
hipError_t colsum(const void* x, bool bf16, void* out, bool out_bf16, int64_t rows, int64_t cols, float* ws,
                  hipStream_t st) {
  if (rows == 0) return hipMemsetAsync(out, 0, cols * (out_bf16 ? 2 : 4), st);
  const int nslab = plan_slabs(rows, cols);
  const int64_t rps = (rows + nslab - 1) / nslab;
  dim3 pg((unsigned)((cols + kStripCols - 1) / kStripCols), (unsigned)nslab);
  if (bf16)
    colstrip_partial_kernel<bf16_t, false, false><<<pg, kThreads, 0, st>>>((const bf16_t*)x, nullptr, nullptr, nullptr,
                                                                           ws, rows, cols, rps, nslab);
  else
    colstrip_partial_kernel<float, false, false><<<pg, kThreads, 0, st>>>((const float*)x, nullptr, nullptr, nullptr,
                                                                          ws, rows, cols, rps, nslab);
  PDA_CHECK_HIP(hipGetLastError());
  colreduce_finalize_kernel<<<fin_grid(cols), kFinCols * kFinLanes, 0, st>>>(ws, nslab, cols, 1, out, nullptr, out_bf16 ? 1 : 0);
  return hipGetLastError();
}

}  // namespace pda
