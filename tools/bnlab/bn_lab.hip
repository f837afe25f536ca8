// Standalone lab for the BatchNorm reduction kernels (stats / backward reduce): compares the
// contiguous-chunk row partition against an interleaved one and the ReLU-mask variants, on
// ResNet-50 bs256 shapes, with buffers rotated so every pass streams from HBM.
//   hipcc -O3 --offload-arch=gfx950 -I csrc/include tools/bnlab/bn_lab.hip -o /tmp/bn_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "pda_common.h"
using namespace pda;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NT = 256;

__device__ __forceinline__ void colsum_store(float (&a)[8], float (&b)[8], int tx, int ty, int cols, int rpi, int vcol,
                                             int C, float* sa, float* sb) {
  __shared__ float s_a[NT * 8], s_b[NT * 8];
  for (int j = 0; j < 8; ++j) { s_a[threadIdx.x * 8 + j] = a[j]; s_b[threadIdx.x * 8 + j] = b[j]; }
  __syncthreads();
  if (ty == 0 && vcol * 8 < C) {
    for (int k = 1; k < rpi; ++k) {
      const int t = k * cols + tx;
      for (int j = 0; j < 8; ++j) { a[j] += s_a[t * 8 + j]; b[j] += s_b[t * 8 + j]; }
    }
    store8(sa + (int64_t)blockIdx.x * C + vcol * 8, a);
    store8(sb + (int64_t)blockIdx.x * C + vcol * 8, b);
  }
}

// ILV = 0: block owns rows [b*rpb, (b+1)*rpb); ILV = 1: block takes chunks of U*rpi rows round-robin.
template <int ILV, int U>
__global__ void __launch_bounds__(NT) stats_k(const bf16_t* __restrict__ x, int64_t M, int C, int cols, int rpi,
                                               int64_t rpb, float* __restrict__ slab) {
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  float s1[8], s2[8], piv[8];
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    load8(x + vcol * 8, piv);
    const int64_t chunk = (int64_t)U * rpi;
    int64_t r, r1, step;
    if (ILV) { r = (int64_t)blockIdx.x * chunk + ty; r1 = M; step = (int64_t)gridDim.x * chunk; }
    else { r = (int64_t)blockIdx.x * rpb + ty; r1 = min((int64_t)(blockIdx.x + 1) * rpb, M); step = chunk; }
    for (; r + (U - 1) * rpi < r1; r += step) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) load8(x + (r + u * rpi) * C + vcol * 8, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[u][j] - piv[j]; s1[j] += d; s2[j] = fmaf(d, d, s2[j]); }
    }
    for (; r < r1; r += rpi) {  // tail rows (ILV: only the last partial chunk, r < M)
      float v[8];
      load8(x + r * C + vcol * 8, v);
      for (int j = 0; j < 8; ++j) { const float d = v[j] - piv[j]; s1[j] += d; s2[j] = fmaf(d, d, s2[j]); }
      if (ILV && ((r - ty) % chunk) + rpi >= chunk) break;
    }
  }
  colsum_store(s1, s2, tx, ty, cols, rpi, vcol, C, slab, slab + (int64_t)gridDim.x * C);
}

// backward reduce: MASK 2 = recompute from x*scale+shift (PRE: scale/shift in registers), 3 = bits
template <int ILV, int MASK, bool PRE>
__global__ void __launch_bounds__(NT) red_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                             const uint8_t* __restrict__ bits, const float* __restrict__ ss,
                                             const float* __restrict__ mean, int64_t M, int C, int cols, int rpi,
                                             int64_t rpb, float* __restrict__ slab) {
  constexpr int U = 4;
  const int tx = threadIdx.x % cols, ty = threadIdx.x / cols;
  const int vcol = blockIdx.y * cols + tx;
  const bool active = ty < rpi && vcol * 8 < C;
  const int c0 = vcol * 8;
  float sa[8], sb[8], mu[8], sc[8], sh[8];
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.f;
  if (active) {
    load8(mean + c0, mu);
    if (PRE && MASK == 2) { load8(ss + c0, sc); load8(ss + C + c0, sh); }
    const int64_t chunk = (int64_t)U * rpi;
    int64_t r, r1, step;
    if (ILV) { r = (int64_t)blockIdx.x * chunk + ty; r1 = M; step = (int64_t)gridDim.x * chunk; }
    else { r = (int64_t)blockIdx.x * rpb + ty; r1 = min((int64_t)(blockIdx.x + 1) * rpb, M); step = chunk; }
    for (; r + (U - 1) * rpi < r1; r += step) {
      float g[U][8], xv[U][8];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = (r + u * rpi) * C + c0;
        load8(dy + off, g[u]);
        load8(x + off, xv[u]);
        if (MASK == 3) mb[u] = bits[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          bool keep;
          if (MASK == 3) keep = (mb[u] >> j) & 1u;
          else if (PRE) keep = fmaf(xv[u][j], sc[j], sh[j]) > 0.f;
          else keep = xv[u][j] * ss[c0 + j] + ss[C + c0 + j] > 0.f;
          const float gg = keep ? g[u][j] : 0.f;
          sa[j] += gg;
          sb[j] = fmaf(gg, xv[u][j] - mu[j], sb[j]);
        }
      }
    }
  }
  colsum_store(sa, sb, tx, ty, cols, rpi, vcol, C, slab, slab + (int64_t)gridDim.x * C);
}

__global__ void copy_k(const u16x8* __restrict__ a, u16x8* __restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) b[i] = a[i];
}

struct Geo { int cols, rpi, gy; };
Geo geo(int C) { Geo g; int cv = C / 8; if (cv >= NT) { g.cols = NT; g.rpi = 1; g.gy = (cv + NT - 1) / NT; } else { g.cols = cv; g.rpi = NT / cv; g.gy = 1; } return g; }

int main() {
  const int64_t shapes[][2] = {{3211264, 64}, {802816, 64}, {802816, 256}, {200704, 128}, {200704, 512},
                               {50176, 256}, {50176, 1024}, {12544, 512}, {12544, 2048}};
  const int NB = 4;  // rotate buffers: >= 4 x 100+ MB keeps the 256 MB MALL from serving re-reads
  size_t maxe = 3211264ull * 64;
  std::vector<bf16_t*> X(NB), DY(NB);
  std::vector<uint8_t*> BI(NB);
  for (int i = 0; i < NB; ++i) {
    CK(hipMalloc(&X[i], maxe * 2)); CK(hipMalloc(&DY[i], maxe * 2)); CK(hipMalloc(&BI[i], maxe / 8));
    CK(hipMemset(X[i], 0x3f, maxe * 2)); CK(hipMemset(DY[i], 0x3f, maxe * 2)); CK(hipMemset(BI[i], 0x55, maxe / 8));
  }
  float *slab, *ss, *mean;
  CK(hipMalloc(&slab, 64 << 20)); CK(hipMalloc(&ss, 4 * 4096)); CK(hipMalloc(&mean, 4 * 4096));
  CK(hipMemset(ss, 0, 4 * 4096)); CK(hipMemset(mean, 0, 4 * 4096));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int IT = 24;
  for (auto& s : shapes) {
    const int64_t M = s[0]; const int C = (int)s[1];
    const double bytes = (double)M * C * 2;
    Geo g = geo(C);
    auto run = [&](const char* name, double passes, auto launch) {
      for (int w = 0; w < 4; ++w) launch(w % NB);
      CK(hipEventRecord(e0));
      for (int i = 0; i < IT; ++i) launch(i % NB);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / IT;
      printf("{\"M\": %ld, \"C\": %d, \"kernel\": \"%s\", \"us\": %.2f, \"TBps\": %.2f}\n", (long)M, C, name, us,
             passes * bytes / us / 1e6);
    };
    for (int nb : {512, 1024}) {
      const int target = nb / g.gy;
      int64_t rpb = (M + target - 1) / target; if (rpb < 64) rpb = 64;
      const int nrb = (int)((M + rpb - 1) / rpb);
      char nm[64];
      snprintf(nm, 64, "stats_chunk_nb%d", nb);
      run(nm, 1, [&](int b) { stats_k<0, 8><<<dim3(nrb, g.gy), NT>>>(X[b], M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "stats_ilv8_nb%d", nb);
      run(nm, 1, [&](int b) { stats_k<1, 8><<<dim3(nrb, g.gy), NT>>>(X[b], M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "stats_ilv4_nb%d", nb);
      run(nm, 1, [&](int b) { stats_k<1, 4><<<dim3(nrb, g.gy), NT>>>(X[b], M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "red3_chunk_nb%d", nb);
      run(nm, 2, [&](int b) { red_k<0, 3, false><<<dim3(nrb, g.gy), NT>>>(DY[b], X[b], BI[b], ss, mean, M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "red3_ilv_nb%d", nb);
      run(nm, 2, [&](int b) { red_k<1, 3, false><<<dim3(nrb, g.gy), NT>>>(DY[b], X[b], BI[b], ss, mean, M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "red2_chunk_nb%d", nb);
      run(nm, 2, [&](int b) { red_k<0, 2, false><<<dim3(nrb, g.gy), NT>>>(DY[b], X[b], BI[b], ss, mean, M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "red2pre_chunk_nb%d", nb);
      run(nm, 2, [&](int b) { red_k<0, 2, true><<<dim3(nrb, g.gy), NT>>>(DY[b], X[b], BI[b], ss, mean, M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "red2pre_ilv_nb%d", nb);
      run(nm, 2, [&](int b) { red_k<1, 2, true><<<dim3(nrb, g.gy), NT>>>(DY[b], X[b], BI[b], ss, mean, M, C, g.cols, g.rpi, rpb, slab); });
      snprintf(nm, 64, "red0_chunk_nb%d", nb);
      run(nm, 2, [&](int b) { red_k<0, 0, false><<<dim3(nrb, g.gy), NT>>>(DY[b], X[b], BI[b], ss, mean, M, C, g.cols, g.rpi, rpb, slab); });
    }
    run("copy", 2, [&](int b) { copy_k<<<2048, 256>>>((const u16x8*)X[b], (u16x8*)DY[(b + 1) % NB], M * C / 8); });
  }
  printf("done\n");
  return 0;
}
