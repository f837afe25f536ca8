// Host-callable launchers of the pytorchdistributed_amd HIP kernels.  Pure HIP: no torch headers,
// so kernel translation units compile in seconds and the bindings layer owns tensor validation.
// Every launcher is asynchronous on `st`, performs no allocation and no synchronisation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pda {
typedef uint16_t bf16_t;

// attention tensors are [B, T, H, D] with element strides (sb, st, sh) and a contiguous head dim
struct AttnParams {
  const bf16_t *q, *k, *v;
  bf16_t* o;
  float* lse;  // [B, Hq, T] (natural log)
  int64_t q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh;
  int B, T, Hq, Hkv, D, causal;
  float scale;
  // optional fused rotary embedding (rotate-half convention) of q and k: tables [T, D/2]
  const float *rope_cos, *rope_sin;
  // backward
  const bf16_t* dout;
  int64_t do_sb, do_st, do_sh;
  float* delta;  // [B, Hq, T] workspace
  bf16_t *dq, *dk, *dv;
  int64_t dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh, dv_sb, dv_st, dv_sh;
  // GQA dK/dV partials per query head, fp32 [2][B][Hq][T][D] (only when Hq > Hkv; attn_bwd_ws_floats)
  float* dkv_part;
  // fused dK/dV/dQ backward: fp32 dQ accumulator [B][Hq][T][D] (attention_bwd_fused), else null
  float* dq_acc;
};

// ---- xgmi.hip (one-shot / two-shot all-reduce over IPC-mapped peer buffers)
constexpr int kXgmiMaxRanks = 8;
constexpr int kXgmiMaxBlocks = 128;
constexpr int kXgmiPhases = 3;
// XgmiArgs::algo: all-reduce one-shot / two-shot / ring, all-gather, reduce-scatter
constexpr int kXgmiOneShot = 0, kXgmiTwoShot = 1, kXgmiRing = 2, kXgmiAllGather = 3, kXgmiReduceScatter = 4;
struct XgmiArgs {
  void* data[kXgmiMaxRanks];       // exchange buffer of every rank (own + IPC-mapped peers)
  uint32_t* flags[kXgmiMaxRanks];  // flag array of every rank: [kXgmiPhases][kXgmiMaxBlocks][kXgmiMaxRanks]
  void* out;
  int64_t n;                       // elements, multiple of 8
  int rank, world;
  float scale;
  uint32_t epoch;
  long long timeout_ticks;         // wall_clock64 ticks before a spin gives up
  int* err;
  int algo;                        // kXgmi* below
};
hipError_t xgmi_alloc(void** p, size_t bytes);
hipError_t xgmi_free(void* p);
hipError_t xgmi_alloc_error_word(int** host, int** dev);  // pinned, host-coherent, zeroed
hipError_t xgmi_free_error_word(int* host);
hipError_t xgmi_get_handle(void* p, char* out64);
hipError_t xgmi_open_handle(const char* in64, void** p);
hipError_t xgmi_close_handle(void* p);
hipError_t xgmi_allreduce(const XgmiArgs& a, bool bf16, hipStream_t st);

// ---- optim.hip
hipError_t sgd_step(float* master, bf16_t* param_bf16, const void* grad, bool grad_bf16, float* mom, int64_t n,
                    float lr, float momentum, float dampening, float wd, bool nesterov, bool first, float gscale,
                    const float* gscale_ptr, const float* lr_ptr, hipStream_t st);
hipError_t adam_step(float* master, bf16_t* param_bf16, const void* grad, bool grad_bf16, float* m, float* v,
                     int64_t n, float lr, float beta1, float beta2, float eps, float wd, bool adamw, int64_t step,
                     float gscale, const float* gscale_ptr, const float* lr_ptr, const float* step_ptr,
                     hipStream_t st);
int grad_norm_partials();
hipError_t grad_norm(const void* grad, bool grad_bf16, int64_t n, float pre, float max_norm, float* partial,
                     float* out, hipStream_t st);
hipError_t cast_scale(const void* src, bool src_bf16, void* dst, bool dst_bf16, int64_t n, float scale,
                      const float* scale_ptr, hipStream_t st);

// ---- cross_entropy.hip
hipError_t cross_entropy_fwd(const void* logits, bool logits_bf16, int64_t M, int64_t C, int64_t Cv,
                             const int64_t* target_idx,
                             const float* target_prob, int64_t ignore_index, float smoothing, float* loss, float* lse,
                             hipStream_t st);
hipError_t cross_entropy_bwd(const void* logits, bool logits_bf16, int64_t M, int64_t C, int64_t Cv,
                             const int64_t* target_idx,
                             const float* target_prob, int64_t ignore_index, float smoothing, const float* lse,
                             const float* gscale_ptr, float gscale, void* dlogits, hipStream_t st);

// ---- batchnorm.hip (x, y: [M, C] channels-last, C % 8 == 0)
int64_t bn_workspace_floats(int64_t M, int64_t C);
hipError_t bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                        const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, float* running_mean,
                        float* running_var, float momentum, float eps, bool relu, float* save_mean,
                        float* save_invstd, float* save_ss, float* ws, uint8_t* relu_bits, int64_t* num_batches,
                        hipStream_t st);
// num_batches (optional): int64 counter incremented once on the stream (BN num_batches_tracked)
// relu_bits (optional, with relu): [M*C/8] bytes, bit j of byte v = ReLU mask of element 8v+j
// training forward from a conv epilogue's statistics table [table_rows][2][C]: rows hold partial
// sum(x - K) and sum((x - K)^2), K = shift; finalize (which re-zeroes the table) + apply only — no
// statistics pass over x
hipError_t bn_fwd_train_sums(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, float* table,
                             int table_rows, const float* shift, const float* gamma_f, const bf16_t* gamma_b,
                             const float* beta_f, const bf16_t* beta_b, float* running_mean, float* running_var,
                             float momentum, float eps, bool relu, float* save_mean, float* save_invstd,
                             float* save_ss, uint8_t* relu_bits, int64_t* num_batches, hipStream_t st);
// one BN of bn_fwd_train_sums_dual: its statistics table / shift, affine params, running stats and
// outputs (save_ss: [2, C] scale then shift)
struct BnSumsArgs {
  float* table;
  int table_rows;
  const float* shift;
  const float* gamma_f;
  const bf16_t* gamma_b;
  const float* beta_f;
  const bf16_t* beta_b;
  float* running_mean;
  float* running_var;
  float* save_mean;
  float* save_invstd;
  float* save_ss;
  int64_t* num_batches;
};
// finalize only (no apply): mean, invstd, scale / shift (save_ss [2, C]) and the running statistics from a
// conv epilogue's statistics table, which it re-zeroes
hipError_t bn_finalize_sums(const bf16_t* x, int64_t M, int64_t C, const BnSumsArgs& a, float momentum, float eps,
                            hipStream_t st);
// ResNet stem backward of maxpool(3, 2, 1) over relu(bn(z)): dp [N,P,Q,C] + argmax bytes -> dz [N,H,W,C],
// dgamma / dbeta; the pooled-input gradient is gathered in registers (never stored)
bool stem_pool_bn_bwd_ok(int H, int W, int C, int P, int Q, int k, int s, int pad);
int64_t stem_pool_bn_bwd_ws_floats(int64_t C);
hipError_t stem_pool_bn_bwd(const bf16_t* dp, const uint8_t* idx, const bf16_t* z, const float* ss,
                            const float* mean, const float* invstd, const float* gamma_f, const bf16_t* gamma_b,
                            int N, int H, int W, int C, int P, int Q, bf16_t* dz, float* dgamma_f, bf16_t* dgamma_b,
                            float* dbeta_f, bf16_t* dbeta_b, float* ws, hipStream_t st);
bool bn_dual_ok(int64_t C);
// one BN of bn_bwd_dual: input, saved statistics, affine weight, outputs, workspace (bn_workspace_floats)
struct BnBwdSide {
  float* table;  // optional: [rows][2][C] sums from a dgrad epilogue (no reduce pass; re-zeroed)
  int rows;
  const bf16_t* x;
  const float* mean;
  const float* invstd;
  const float* gamma_f;
  const bf16_t* gamma_b;
  bf16_t* dx;
  float* dgamma_f;
  bf16_t* dgamma_b;
  float* dbeta_f;
  bf16_t* dbeta_b;
  float* ws;
};
bool bn_bwd_dual_ok(int64_t C);
// backward of y = relu(bn_a(x_a) + bn_b(x_b)) from dy and the forward's ReLU bits: one reduce pass over
// (dy, bits, x_a, x_b), two finalizes, one apply pass writing dx_a and dx_b
hipError_t bn_bwd_dual(const bf16_t* dy, const uint8_t* relu_bits, int64_t M, int64_t C, const BnBwdSide& a,
                       const BnBwdSide& b, hipStream_t st);
// y = relu(bn_a(x) + bn_b(x2)) from two conv-epilogue statistics tables; writes the 1-bit ReLU mask
hipError_t bn_fwd_train_sums_dual(const bf16_t* x, const bf16_t* x2, bf16_t* y, int64_t M, int64_t C,
                                  const BnSumsArgs& a, const BnSumsArgs& b, float momentum, float eps,
                                  uint8_t* relu_bits, hipStream_t st);
hipError_t bn_fwd_eval(const bf16_t* x, const bf16_t* res, bf16_t* y, int64_t M, int64_t C, const float* gamma_f,
                       const bf16_t* gamma_b, const float* beta_f, const bf16_t* beta_b, const float* running_mean,
                       const float* running_var, float eps, bool relu, float* ws, hipStream_t st);
// relu: the mask comes from relu_bits when given, else from y, else from x * ss[0:C] + ss[C:2C]
// (scale/shift saved by bn_fwd_train; BN+ReLU without residual never materialises y for the backward)
hipError_t bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const uint8_t* relu_bits, const float* ss,
                  int64_t M, int64_t C,
                  const float* save_mean, const float* save_invstd, const float* gamma_f, const bf16_t* gamma_b,
                  bool relu, bf16_t* dx, bf16_t* dres, float* dgamma_f, bf16_t* dgamma_b, float* dbeta_f,
                  bf16_t* dbeta_b, float* ws, float* fin_table, unsigned* fin_ticket, int fin_rows,
                  hipStream_t st);
// BN backward whose reduction sums were accumulated by the producing dgrad's epilogue (BnBwdStats): a
// finalize from `table` ([rows][2][C], re-zeroed) and the apply pass; no reduce pass over dy and x
hipError_t bn_bwd_table(const bf16_t* dy, const bf16_t* x, const uint8_t* relu_bits, const float* ss, int64_t M,
                        int64_t C, const float* save_mean, const float* save_invstd, const float* gamma_f,
                        const bf16_t* gamma_b, bool relu, bf16_t* dx, bf16_t* dres, float* dgamma_f, bf16_t* dgamma_b,
                        float* dbeta_f, bf16_t* dbeta_b, float* table, int rows, float* coef, hipStream_t st);
// fused finalize (fin_table != nullptr): the reduce kernel's last block finalizes in-launch from a
// persistent zeroed [fin_rows][2][C] table + ticket (left zero); rows for C channels:
int bn_bwd_table_rows(int64_t C);

// ---- pool.hip (NHWC, C % 8 == 0)
hipError_t maxpool2d_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int k,
                         int s, int pad, hipStream_t st);
// maxpool of relu(x * ss[0:C] + ss[C:2C]) (BatchNorm + ReLU applied on the fly), same outputs as maxpool2d_fwd
hipError_t maxpool2d_bn_fwd(const bf16_t* x, const float* ss, bf16_t* y, uint8_t* idx, int N, int H, int W, int C,
                            int P, int Q, int k, int s, int pad, hipStream_t st);
hipError_t maxpool2d_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int P, int Q,
                         int k, int s, int pad, hipStream_t st);
// stem space-to-depth: y[N, U, V, 16] from x[N, H, W, Cx] (first C <= 4 channels), 2x2 blocks, pad
hipError_t stem_space_to_depth(const bf16_t* x, bf16_t* y, int N, int H, int W, int Cx, int C, int U, int V, int pad,
                               hipStream_t st);
hipError_t avgpool_global_fwd(const bf16_t* x, void* y, bool y_bf16, int N, int HW, int C, hipStream_t st);
hipError_t avgpool_global_bwd(const void* dy, bool dy_bf16, bf16_t* dx, int N, int HW, int C, hipStream_t st);

// ---- synth.hip
hipError_t fill_random(void* out, int dtype /*0 f32, 1 bf16*/, int64_t n, uint64_t seed, uint64_t offset, int kind,
                       float a, float b, hipStream_t st);
hipError_t fill_randint(int64_t* out, int64_t n, uint64_t seed, uint64_t offset, int64_t low, int64_t high,
                        hipStream_t st);

// ---- gemm_conv.hip
// path override for the GEMM family: wide = -1 env default (PDA_GEMM_WIDE), 0 off, 1 heuristic, 2 force;
// variant >= 0 selects a wide-kernel schedule variant (bit 0 setprio, bit 1 MFMA/ds_read interleave)
void set_gemm_paths(int wide);
void set_gemm_pp(int on);  // -1: PDA_GEMM_PP (default on), 0 / 1: force
void set_splitk_fixup(int on);  // -1: PDA_SPLITK_FIXUP (default off), 0 / 1: force
int64_t gemm_slab_floats(int64_t M, int64_t N, int64_t K, bool allow_split);
hipError_t gemm_bf16(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                     void* C, bool c_f32, int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias,
                     bool bias_f32, bool relu, float* slab, bool allow_split, hipStream_t st);
// act 1: C = gelu_tanh(A B + bias), act_aux = A B + bias (pre-activation); act 2: C = (A B) * gelu_tanh'(act_aux)
hipError_t gemm_bf16_wgrad_db(const bf16_t* dy, int64_t ld_dy, const bf16_t* x, int64_t ld_x, void* dw, bool dw_f32,
                              int64_t ldc, int64_t M, int64_t N, int64_t K, void* db, bool db_bf16, float* slab,
                              float* rs_scratch, hipStream_t st, int* db_done);
hipError_t gemm_bf16_act(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                         bf16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, const void* bias, bool bias_f32,
                         int act, bf16_t* act_aux, hipStream_t st);
int64_t conv_slab_floats(int mode, int N, int H, int W, int C, int Cout, int R, int S, int P, int Q);
// stats (optional): BatchNorm sums of the output accumulated (atomically; must start zeroed) into a
// [stats_rows][2][Cout] fp32 table: sum(y - K) and sum((y - K)^2) with K = stats_shift (e.g. the running
// mean), each output tile adding into row (tile_m % stats_rows)
// y / dx: bf16, or fp32 with y_f32 / dx_f32 (the split-bf16 fp32 path, fp32x3.hip)
hipError_t conv2d_fwd(const bf16_t* x, const bf16_t* w, void* y, bool y_f32, int N, int H, int W, int C, int Cout,
                      int R, int S, int P, int Q, int stride, int pad, int dil, const void* bias, bool bias_f32,
                      bool relu, float* stats, const float* stats_shift, int stats_rows, hipStream_t st);
// addend (optional, bf16, dx's layout): dx = dgrad + addend, fused into the store; addend_bits (optional,
// [numel/8] bytes, bit j of byte v for element 8v + j): only the addend elements whose bit is set
// wt: the weight transposed by conv_weight_transpose — except for a 1x1 stride-1 unpadded conv
// (conv_dgrad_needs_wt() false), whose dgrad is a plain GEMM that reads w [Cout][C] MN-major in place.
bool conv_dgrad_needs_wt(int R, int S, int stride, int pad);
// 1x1 stride-1 dgrads that read a transposed weight wt[C][Cout] (K-major) instead (MFMA-heavy shapes)
bool conv_dgrad_1x1_wt(int R, int S, int stride, int pad, int C, int Cout);
// BatchNorm-backward statistics fused into the dgrad epilogue (bst, optional): dx is the dy of the BN whose
// ReLU output the conv consumed; the epilogues add sum(g) and sum(g (z - mean)), g = dx * relu_mask(z),
// into table[tile % rows][2][C] (zero on entry; bn_bwd_table reads and re-zeroes it).  Mask from
// ss = [2][C] scale / shift or from the forward's bit mask.  Not with an fp32 dx or an addend.
struct BnBwdStats {
  const bf16_t* z;
  const float* ss;
  const uint8_t* bits;
  const float* mean;
  float* table;
  int rows;
  // optional second BN of the same masked gradient (relu(bn(z) + bn2(z2))): its input, mean and table
  const bf16_t* z2;
  const float* mean2;
  float* table2;
};
hipError_t conv2d_dgrad(const bf16_t* dy, const bf16_t* w, const bf16_t* wt, void* dx, bool dx_f32, int N, int H, int W,
                        int C, int Cout, int R, int S, int P, int Q, int stride, int pad, int dil, const bf16_t* addend,
                        const uint8_t* addend_bits, hipStream_t st, const BnBwdStats* bst = nullptr);
// PDA_DGRAD_STREAM at run time (-1: back to the environment's value): 0 off, 1 BN-sums dgrads, 2 all short-K
void set_dgrad_stream(int mode);
void set_fwd_stream(int mode);  // -1: PDA_FWD_STREAM (default 1), 0 off, 1 K in {64, 128}, 2 also K = 256
hipError_t conv2d_wgrad(const bf16_t* dy, const bf16_t* x, void* dw, bool dw_f32, int N, int H, int W, int C,
                        int Cout, int R, int S, int P, int Q, int stride, int pad, int dil, float* slab,
                        hipStream_t st);
// wt = w transposed to [Cin][taps][Cout], phase-packed for the stride-decomposed dgrad
hipError_t conv_weight_transpose(const bf16_t* w, bf16_t* wt, int Cout, int R, int S, int Cin, int stride, int pad,
                                 int dil, hipStream_t st);


// ---- act.hip (op: 0 relu, 1 gelu_tanh)
hipError_t act_fwd(const void* x, void* y, bool bf16, int64_t n, int op, hipStream_t st);
hipError_t act_bwd(const void* dy, const void* ref, void* dx, bool bf16, int64_t n, int op, hipStream_t st);
hipError_t swiglu_fwd(const void* gu, void* y, bool bf16, int64_t rows, int64_t F, hipStream_t st);
hipError_t swiglu_bwd(const void* dy, const void* gu, void* dgu, bool bf16, int64_t rows, int64_t F, hipStream_t st);
hipError_t colsum_unaligned(const void* x, bool bf16, float* out, int64_t rows, int64_t cols, hipStream_t st);

// ---- gemm_pp.hip (pipelined 256x256 tile; lab entry)
hipError_t gemm_pp_lab(const bf16_t* A, bool a_kmajor, int64_t lda, const bf16_t* B, bool b_kmajor, int64_t ldb,
                       bf16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, const bf16_t* bias, int variant,
                       hipStream_t st);

// ---- simt_gemm.hip (dtype codes 0 fp32 / 1 bf16; arbitrary strides)
hipError_t simt_gemm(const void* A, int a_dt, int64_t sam, int64_t sak, const void* B, int b_dt, int64_t sbk,
                     int64_t sbn, void* C, int c_dt, int64_t scm, int64_t scn, int64_t M, int64_t N, int64_t K,
                     const float* bias, bool relu, float beta, hipStream_t st);

// ---- rownorm.hip (LayerNorm / RMSNorm over the last dim, D % 8 == 0, D <= 8192)
hipError_t add_rownorm_fwd(const bf16_t* x, const bf16_t* r, const bf16_t* gamma, const bf16_t* beta, bf16_t* h,
                           bf16_t* y, int64_t rows, int64_t D, float eps, bool rms, hipStream_t st,
                           float* mean = nullptr, float* rstd = nullptr);  // stats of h: training
hipError_t rownorm_fwd(const void* x, bool x_bf16, const void* gamma, const void* beta, bool p_bf16, void* y,
                       float* mean, float* rstd, int64_t rows, int64_t D, float eps, bool rms, hipStream_t st);
hipError_t rownorm_bwd(const void* dy, const void* x, bool x_bf16, const void* gamma, bool p_bf16, const float* mean,
                       const float* rstd, void* dx, void* dgamma, void* dbeta, bool dparam_bf16, int64_t rows,
                       int64_t D, bool rms, float* ws, hipStream_t st, const void* addend = nullptr);  // dx += addend (same layout)
// column sums via slab partials (cols % 8 == 0); ws holds colreduce_ws_floats(rows, cols, 1) floats
hipError_t colsum(const void* x, bool bf16, void* out, bool out_bf16, int64_t rows, int64_t cols, float* ws,
                  hipStream_t st);
int64_t colreduce_ws_floats(int64_t rows, int64_t D, int nout);

// ---- attention.hip (flash attention fwd / bwd, D in {64, 128}, GQA, causal or not)
hipError_t attention_fwd(const AttnParams& p, hipStream_t st);
hipError_t attention_bwd(const AttnParams& p, hipStream_t st);
int64_t attention_bwd_ws_floats(int B, int T, int Hq, int Hkv, int D, bool rope);
bool attention_bwd_fused(int D, bool rope);
int& attention_bwd_fused_mode();  // PDA_ATTN_BWD_FUSED bits (set_attn_bwd_fused)

// ---- decode_attn.hip (serving: one query token per sequence vs a bf16 KV cache, split over the sequence)
struct DecodeAttnParams {
  const bf16_t* q;  // [B, Hq, D] view (q_sb, q_sh strides), D contiguous
  const bf16_t* k;  // cache [B, Tmax, Hkv, D] view (k_sb, k_st, k_sh)
  const bf16_t* v;
  bf16_t* o;        // [B, Hq, D] contiguous
  float* ws_acc;    // [B, Hq, splits, D] fp32 (splits > 1)
  float* ws_ml;     // [B, Hq, splits, 2] fp32 (running max in log2 units, sum)
  int64_t q_sb, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh;
  int B, Hq, Hkv, D, L, splits, chunk;
  float scale_log2;  // softmax scale * log2(e)
  const int* L_dev;  // optional: attend *L_dev + 1 rows (graph-replayable decode; overrides L)
};
struct KvAppendParams {
  const bf16_t* qkv;  // new token [B, 1, Hq + 2*Hkv, D] view (x_sb, x_sh), D contiguous
  bf16_t* q_out;      // [B, Hq, D] contiguous, rotated q
  bf16_t* k_cache;    // [B, Tmax, Hkv, D] view
  bf16_t* v_cache;
  const float *cos, *sin;  // full-length rope tables [Tmax, D/2] or nullptr
  const int* pos;          // device position of the new token
  int64_t x_sb, x_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh;
  int B, Hq, Hkv, D;
};
hipError_t kv_append_rope(const KvAppendParams& p, hipStream_t st);

// ---- w8_gemm.hip (serving: weight-only int8 GEMM for decode steps, M <= 64)
struct W8GemmParams {
  const bf16_t* x;       // [M, K] rows of stride ldx
  const int8_t* w;       // [N, K] int8, row-major
  const float* scale;    // [N] per-row dequantisation scale
  bf16_t* y;             // [M, N] rows of stride ldy
  float* ws;             // [S, M, N] fp32 partial slabs (S > 1)
  int* tickets;          // [N / 64] int32, zero between calls (S > 1; reset by the kernel)
  int64_t ldx, ldy;
  int M, N, K, S;
};
int w8_gemm_splits(int N, int K);
int w8_gemm_rows();
hipError_t w8_gemm(const W8GemmParams& p, hipStream_t st);
int decode_attn_splits(int B, int Hkv, int L, int D);
hipError_t decode_attention(DecodeAttnParams p, hipStream_t st);

// ---- embed.hip
hipError_t embedding_fwd(const int64_t* idx, const bf16_t* table, bf16_t* out, int64_t n, int64_t D, hipStream_t st);
hipError_t embedding_bwd(const int64_t* idx, const bf16_t* dy, float* acc, int64_t n, int64_t D, hipStream_t st);
hipError_t embedding_bwd_sorted(const int64_t* sidx, const int64_t* order, const bf16_t* dy, float* acc, int64_t n,
                                int64_t D, hipStream_t st);
hipError_t rope_apply(const bf16_t* x, bf16_t* y, const float* cos, const float* sin, int B, int T, int H, int D,
                      int64_t sb, int64_t st_, int64_t sh, int64_t yb, int64_t yt, int64_t yh, bool inverse,
                      hipStream_t st);

// ---- fp32x3.hip (fp32 training path: split-bf16 GEMM operands + fp32 BN / pooling)
hipError_t split_bf16(const float* x, bf16_t* out, int64_t rows, int64_t C, int nseg, int lo_mask, int64_t seg_stride,
                      int64_t row_stride, hipStream_t st);
int bn_f32_partials(int64_t M, int C);
hipError_t bn_f32_fwd_train(const float* x, const float* res, const float* gamma, const float* beta,
                            float* running_mean, float* running_var, const float* shift, float momentum, float eps,
                            int relu, float* y, float* save_mean, float* save_invstd, float* ss, float* part,
                            int64_t* num_batches, int64_t M, int C, hipStream_t st);
hipError_t bn_f32_apply(const float* x, const float* res, const float* ss, float* y, int64_t M, int C, int relu,
                        hipStream_t st);
hipError_t bn_f32_bwd(const float* dy, const float* x, const float* y, const float* mean, const float* invstd,
                      const float* gamma, float* dx, float* gout, float* dgamma, float* dbeta, float* part, float* co,
                      int64_t M, int C, hipStream_t st);
hipError_t maxpool2d_f32_fwd(const float* x, float* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int k,
                             int s, int pad, hipStream_t st);
hipError_t maxpool2d_f32_bwd(const float* dy, const uint8_t* idx, float* dx, int N, int H, int W, int C, int P, int Q,
                             int k, int s, int pad, hipStream_t st);
hipError_t avgpool_f32_fwd(const float* x, float* y, int N, int HW, int C, hipStream_t st);
hipError_t avgpool_f32_bwd(const float* dy, float* dx, int N, int HW, int C, hipStream_t st);

}  // namespace pda
