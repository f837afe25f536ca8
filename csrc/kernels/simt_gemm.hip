// General-stride SIMT GEMM (fp32 or bf16 operands, fp32 accumulate): the path for matmuls the MFMA
// kernel cannot take — fp32 models (the reference's fp32 Linear(20,1) DDP demo `PY1:77`, the
// DataParallel MLP 10-20-20-20-5 `NB01:94-107`) and widths that are not multiples of 8.  SURVEY §2.5
// K01 calls this the "skinny path": at [32,20]x[20,1] an MFMA tile would be >90 % idle.
// 64x64 block tile, 256 threads x (4x4) outputs, K staged through LDS 16 at a time.
#include "pda_common.h"
#include "pda_kernels.h"

namespace pda {
namespace {

constexpr int TB = 64, TK = 16;

template <typename TA, typename TB_, typename TC>
__global__ void __launch_bounds__(256) simt_gemm_kernel(const TA* __restrict__ A, int64_t sam, int64_t sak,
                                                        const TB_* __restrict__ B, int64_t sbk, int64_t sbn,
                                                        TC* __restrict__ C, int64_t scm, int64_t scn, int64_t M,
                                                        int64_t N, int64_t K, const float* __restrict__ bias,
                                                        int relu, float beta) {
  __shared__ float As[TK][TB + 1];
  __shared__ float Bs[TK][TB + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t m0 = (int64_t)blockIdx.y * TB, n0 = (int64_t)blockIdx.x * TB;
  float acc[4][4] = {};
  for (int64_t k0 = 0; k0 < K; k0 += TK) {
    for (int i = threadIdx.x; i < TK * TB; i += 256) {
      const int kk = i / TB, mm = i % TB;
      const int64_t m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < M && k < K) ? Elem<TA>::load(A, m * sam + k * sak) : 0.f;
      const int64_t n = n0 + mm;
      Bs[kk][mm] = (n < N && k < K) ? Elem<TB_>::load(B, k * sbk + n * sbn) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + tx * 4 + j;
      if (n >= N) continue;
      float v = acc[i][j];
      if (bias) v += bias[n];
      if (beta != 0.f) v += beta * Elem<TC>::load(C, m * scm + n * scn);
      if (relu) v = fmaxf(v, 0.f);
      Elem<TC>::store(C, m * scm + n * scn, v);
    }
  }
}

}  // namespace

// dtype codes: 0 fp32, 1 bf16
hipError_t simt_gemm(const void* A, int a_dt, int64_t sam, int64_t sak, const void* B, int b_dt, int64_t sbk,
                     int64_t sbn, void* C, int c_dt, int64_t scm, int64_t scn, int64_t M, int64_t N, int64_t K,
                     const float* bias, bool relu, float beta, hipStream_t st) {
  dim3 grid((unsigned)((N + TB - 1) / TB), (unsigned)((M + TB - 1) / TB));
#define PDA_SIMT(TA_, TB__, TC_)                                                                                 \
  simt_gemm_kernel<TA_, TB__, TC_><<<grid, 256, 0, st>>>((const TA_*)A, sam, sak, (const TB__*)B, sbk, sbn,   \
                                                         (TC_*)C, scm, scn, M, N, K, bias, relu ? 1 : 0, beta)
  const int code = a_dt * 4 + b_dt * 2 + c_dt;
  switch (code) {
    case 0: PDA_SIMT(float, float, float); break;
    case 1: PDA_SIMT(float, float, bf16_t); break;
    case 2: PDA_SIMT(float, bf16_t, float); break;
    case 3: PDA_SIMT(float, bf16_t, bf16_t); break;
    case 4: PDA_SIMT(bf16_t, float, float); break;
    case 5: PDA_SIMT(bf16_t, float, bf16_t); break;
    case 6: PDA_SIMT(bf16_t, bf16_t, float); break;
    default: PDA_SIMT(bf16_t, bf16_t, bf16_t); break;
  }
#undef PDA_SIMT
  return hipGetLastError();
}

}  // namespace pda
