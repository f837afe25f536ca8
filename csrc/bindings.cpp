// pybind11 / torch bindings of the native layer (module `pytorchdistributed_amd._C`).
//
// Kernel bindings validate shapes, dtypes and devices on the host BEFORE launching (a bad launch on
// a shared MI355X box can reset the node), run on the current HIP stream of the tensor's device,
// and raise on any HIP error.  Runtime bindings (TCP store, bucket reducer, host ring) are CPU-only.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <map>
#include <mutex>
#include <c10/core/DeviceGuard.h>

#include "pda_kernels.h"
#include "runtime.h"

namespace pda_rt {
void bind_runtime(pybind11::module& m);
}
namespace pda_comm {
void bind_comm(pybind11::module& m);
}

namespace py = pybind11;
using at::Tensor;

namespace {

#define CHECK_HIP_OK(expr)                                                                  \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e));      \
  } while (0)

hipStream_t stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_bf16(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
void check_f32(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}
bool is_bf16(const Tensor& t) { return t.scalar_type() == at::kBFloat16; }
void check_f32_or_bf16(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, name, " must be fp32 or bf16");
}
void check_aligned16(const Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

const pda::bf16_t* bp(const Tensor& t) { return reinterpret_cast<const pda::bf16_t*>(t.data_ptr()); }
pda::bf16_t* bpm(const Tensor& t) { return reinterpret_cast<pda::bf16_t*>(t.data_ptr()); }
const float* fopt(const c10::optional<Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }

// ------------------------------------------------------------------ optimizers
void sgd_step(Tensor master, c10::optional<Tensor> param_bf16, Tensor grad, Tensor mom, double lr, double momentum,
              double dampening, double wd, bool nesterov, bool first, double gscale,
              c10::optional<Tensor> gscale_t, c10::optional<Tensor> lr_t) {
  check_f32(master, "master");
  check_f32_or_bf16(grad, "grad");
  TORCH_CHECK(grad.numel() == master.numel(), "grad/master size mismatch");
  if (momentum != 0.0) {
    check_f32(mom, "momentum_buffer");
    TORCH_CHECK(mom.numel() == master.numel());
  }
  if (param_bf16) {
    check_bf16(*param_bf16, "param_bf16");
    TORCH_CHECK(param_bf16->numel() == master.numel());
  }
  for (auto* t : {&master, &grad}) check_aligned16(*t, "optimizer buffer");
  c10::DeviceGuard g(master.device());
  CHECK_HIP_OK(pda::sgd_step(master.data_ptr<float>(), param_bf16 ? bpm(*param_bf16) : nullptr, grad.data_ptr(),
                             is_bf16(grad), momentum != 0.0 ? mom.data_ptr<float>() : nullptr, master.numel(),
                             (float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, first, (float)gscale,
                             fopt(gscale_t), fopt(lr_t), stream_of(master)));
}

void adam_step(Tensor master, c10::optional<Tensor> param_bf16, Tensor grad, Tensor m, Tensor v, double lr,
               double beta1, double beta2, double eps, double wd, bool adamw, int64_t step, double gscale,
               c10::optional<Tensor> gscale_t, c10::optional<Tensor> lr_t, c10::optional<Tensor> step_t) {
  check_f32(master, "master");
  check_f32_or_bf16(grad, "grad");
  check_f32(m, "exp_avg");
  if (step_t) check_f32(*step_t, "step");
  check_f32(v, "exp_avg_sq");
  TORCH_CHECK(grad.numel() == master.numel() && m.numel() == master.numel() && v.numel() == master.numel());
  if (param_bf16) {
    check_bf16(*param_bf16, "param_bf16");
    TORCH_CHECK(param_bf16->numel() == master.numel());
  }
  TORCH_CHECK(step >= 1 || step_t, "adam step must be >= 1");
  c10::DeviceGuard g(master.device());
  CHECK_HIP_OK(pda::adam_step(master.data_ptr<float>(), param_bf16 ? bpm(*param_bf16) : nullptr, grad.data_ptr(),
                              is_bf16(grad), m.data_ptr<float>(), v.data_ptr<float>(), master.numel(), (float)lr,
                              (float)beta1, (float)beta2, (float)eps, (float)wd, adamw, step, (float)gscale,
                              fopt(gscale_t), fopt(lr_t), fopt(step_t), stream_of(master)));
}

// returns [norm, clip_coef] on device
Tensor grad_norm(Tensor grad, double pre, double max_norm) {
  check_f32_or_bf16(grad, "grad");
  c10::DeviceGuard g(grad.device());
  auto opts = grad.options().dtype(at::kFloat);
  Tensor partial = at::empty({pda::grad_norm_partials()}, opts);
  Tensor out = at::empty({2}, opts);
  CHECK_HIP_OK(pda::grad_norm(grad.data_ptr(), is_bf16(grad), grad.numel(), (float)pre, (float)max_norm,
                              partial.data_ptr<float>(), out.data_ptr<float>(), stream_of(grad)));
  return out;
}

void cast_scale(Tensor src, Tensor dst, double scale, c10::optional<Tensor> scale_t) {
  check_f32_or_bf16(src, "src");
  check_f32_or_bf16(dst, "dst");
  TORCH_CHECK(src.numel() == dst.numel());
  c10::DeviceGuard g(src.device());
  CHECK_HIP_OK(pda::cast_scale(src.data_ptr(), is_bf16(src), dst.data_ptr(), is_bf16(dst), src.numel(), (float)scale,
                               fopt(scale_t), stream_of(src)));
}

// ------------------------------------------------------------------ cross entropy
std::vector<Tensor> ce_fwd(Tensor logits, Tensor target, int64_t ignore_index, double smoothing, int64_t num_valid) {
  check_f32_or_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "logits must be [M, C]");
  const int64_t M = logits.size(0), C = logits.size(1);
  check_gpu(target, "target");
  const bool prob = target.is_floating_point();
  if (prob) {
    TORCH_CHECK(target.scalar_type() == at::kFloat && target.sizes() == logits.sizes(), "prob target must be fp32 [M,C]");
  } else {
    TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == M, "index target must be int64 [M]");
  }
  c10::DeviceGuard g(logits.device());
  auto opts = logits.options().dtype(at::kFloat);
  Tensor loss = at::empty({M}, opts), lse = at::empty({M}, opts);
  const int64_t Cv = num_valid > 0 ? std::min<int64_t>(num_valid, C) : C;
  CHECK_HIP_OK(pda::cross_entropy_fwd(logits.data_ptr(), is_bf16(logits), M, C, Cv,
                                      prob ? nullptr : target.data_ptr<int64_t>(),
                                      prob ? target.data_ptr<float>() : nullptr, ignore_index, (float)smoothing,
                                      loss.data_ptr<float>(), lse.data_ptr<float>(), stream_of(logits)));
  return {loss, lse};
}

Tensor ce_bwd(Tensor logits, Tensor target, Tensor lse, Tensor gscale_t, double gscale, int64_t ignore_index,
              double smoothing, int64_t num_valid) {
  check_f32_or_bf16(logits, "logits");
  const int64_t M = logits.size(0), C = logits.size(1);
  const bool prob = target.is_floating_point();
  check_f32(lse, "lse");
  check_f32(gscale_t, "gscale");
  c10::DeviceGuard g(logits.device());
  Tensor d = at::empty_like(logits);
  const int64_t Cv = num_valid > 0 ? std::min<int64_t>(num_valid, C) : C;
  CHECK_HIP_OK(pda::cross_entropy_bwd(logits.data_ptr(), is_bf16(logits), M, C, Cv,
                                      prob ? nullptr : target.data_ptr<int64_t>(),
                                      prob ? target.data_ptr<float>() : nullptr, ignore_index, (float)smoothing,
                                      lse.data_ptr<float>(), gscale_t.data_ptr<float>(), (float)gscale, d.data_ptr(),
                                      stream_of(logits)));
  return d;
}

// ------------------------------------------------------------------ batch norm (channels-last)
void bn_param_ptrs(const c10::optional<Tensor>& t, const float** f, const pda::bf16_t** b, int64_t C) {
  *f = nullptr;
  *b = nullptr;
  if (!t.has_value()) return;
  check_f32_or_bf16(*t, "bn affine parameter");
  TORCH_CHECK(t->numel() == C);
  if (is_bf16(*t)) *b = bp(*t);
  else *f = t->data_ptr<float>();
}

int64_t* nbt_ptr(const c10::optional<Tensor>& n, const Tensor& x) {
  if (!n || !n->defined()) return nullptr;
  TORCH_CHECK(n->scalar_type() == at::kLong && n->numel() == 1 && n->device() == x.device(),
              "num_batches must be a one-element int64 tensor on the input's device");
  return n->data_ptr<int64_t>();
}

std::vector<Tensor> bn_fwd_train(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> gamma,
                                 c10::optional<Tensor> beta, c10::optional<Tensor> running_mean,
                                 c10::optional<Tensor> running_var, double momentum, double eps, bool relu,
                                 bool relu_bits, c10::optional<Tensor> num_batches) {
  check_bf16(x, "x");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "channels must be a multiple of 8 and <= 2048");
  if (res) {
    check_bf16(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes());
  }
  const float *gf, *bfp;
  const pda::bf16_t *gb, *bb;
  bn_param_ptrs(gamma, &gf, &gb, C);
  bn_param_ptrs(beta, &bfp, &bb, C);
  if (running_mean) {
    check_f32(*running_mean, "running_mean");
    check_f32(*running_var, "running_var");
  }
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, fo), invstd = at::empty({C}, fo), ss = at::empty({2, C}, fo);
  Tensor ws = at::empty({pda::bn_workspace_floats(M, C)}, fo);
  Tensor bits = (relu && relu_bits) ? at::empty({M * C / 8}, x.options().dtype(at::kByte)) : Tensor();
  CHECK_HIP_OK(pda::bn_fwd_train(bp(x), res ? bp(*res) : nullptr, bpm(y), M, C, gf, gb, bfp, bb,
                                 running_mean ? running_mean->data_ptr<float>() : nullptr,
                                 running_var ? running_var->data_ptr<float>() : nullptr, (float)momentum, (float)eps,
                                 relu, mean.data_ptr<float>(), invstd.data_ptr<float>(), ss.data_ptr<float>(),
                                 ws.data_ptr<float>(), bits.defined() ? bits.data_ptr<uint8_t>() : nullptr,
                                 nbt_ptr(num_batches, x), stream_of(x)));
  return {y, mean, invstd, ss, bits};
}

// training BN forward from a conv epilogue's statistics table [R, 2, C] (conv_fwd_stats), which the
// finalize reads and leaves zeroed
std::vector<Tensor> bn_fwd_train_sums(Tensor x, Tensor table, Tensor shift, c10::optional<Tensor> res,
                                      c10::optional<Tensor> gamma, c10::optional<Tensor> beta,
                                      c10::optional<Tensor> running_mean, c10::optional<Tensor> running_var,
                                      double momentum, double eps, bool relu, bool relu_bits,
                                      c10::optional<Tensor> num_batches) {
  check_bf16(x, "x");
  check_f32(table, "table");
  check_f32(shift, "shift");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && shift.numel() == C);
  TORCH_CHECK(table.numel() % (2 * C) == 0 && table.numel() > 0 && table.is_contiguous(), "table must be [R, 2, C]");
  if (res) {
    check_bf16(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes());
  }
  const float *gf, *bfp;
  const pda::bf16_t *gb, *bb;
  bn_param_ptrs(gamma, &gf, &gb, C);
  bn_param_ptrs(beta, &bfp, &bb, C);
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, fo), invstd = at::empty({C}, fo), ss = at::empty({2, C}, fo);
  Tensor bits = (relu && relu_bits) ? at::empty({M * C / 8}, x.options().dtype(at::kByte)) : Tensor();
  CHECK_HIP_OK(pda::bn_fwd_train_sums(bp(x), res ? bp(*res) : nullptr, bpm(y), M, C, table.data_ptr<float>(),
                                      (int)(table.numel() / (2 * C)), shift.data_ptr<float>(), gf, gb, bfp, bb,
                                      running_mean ? running_mean->data_ptr<float>() : nullptr,
                                      running_var ? running_var->data_ptr<float>() : nullptr, (float)momentum,
                                      (float)eps, relu, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                      ss.data_ptr<float>(), bits.defined() ? bits.data_ptr<uint8_t>() : nullptr,
                                      nbt_ptr(num_batches, x), stream_of(x)));
  return {y, mean, invstd, ss, bits};
}

bool bn_dual_ok(int64_t C) { return pda::bn_dual_ok(C); }

// y = relu(bn(x) + bn2(x2)) (bottleneck output with a downsample shortcut), both BNs from their conv
// epilogues' statistics tables; returns {y, relu bits, mean, invstd, mean2, invstd2}
std::vector<Tensor> bn_fwd_train_sums_dual(Tensor x, Tensor table, Tensor shift, c10::optional<Tensor> gamma,
                                           c10::optional<Tensor> beta, Tensor running_mean, Tensor running_var,
                                           c10::optional<Tensor> num_batches, Tensor x2, Tensor table2,
                                           Tensor shift2, c10::optional<Tensor> gamma2, c10::optional<Tensor> beta2,
                                           Tensor running_mean2, Tensor running_var2,
                                           c10::optional<Tensor> num_batches2, double momentum, double eps) {
  check_bf16(x, "x");
  check_bf16(x2, "x2");
  TORCH_CHECK(x2.sizes() == x.sizes(), "dual BN: both inputs must have one shape");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(pda::bn_dual_ok(C), "dual BN apply needs the register-table path: C/8 dividing 64, or 64, 128 or 256 * 8");
  Tensor tabs[2] = {table, table2}, shifts[2] = {shift, shift2};
  for (int i = 0; i < 2; ++i) {
    check_f32(tabs[i], "table");
    check_f32(shifts[i], "shift");
    TORCH_CHECK(shifts[i].numel() == C && tabs[i].numel() % (2 * C) == 0 && tabs[i].numel() > 0 &&
                tabs[i].is_contiguous(), "table must be [R, 2, C]");
  }
  check_f32(running_mean, "running_mean");
  check_f32(running_var, "running_var");
  check_f32(running_mean2, "running_mean2");
  check_f32(running_var2, "running_var2");
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  Tensor stats = at::empty({2, 4, C}, fo);  // per BN: mean, invstd, scale, shift
  Tensor bits = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  pda::BnSumsArgs a[2];
  c10::optional<Tensor> gam[2] = {gamma, gamma2}, bet[2] = {beta, beta2}, nb[2] = {num_batches, num_batches2};
  Tensor rm[2] = {running_mean, running_mean2}, rv[2] = {running_var, running_var2};
  for (int i = 0; i < 2; ++i) {
    bn_param_ptrs(gam[i], &a[i].gamma_f, &a[i].gamma_b, C);
    bn_param_ptrs(bet[i], &a[i].beta_f, &a[i].beta_b, C);
    a[i].table = tabs[i].data_ptr<float>();
    a[i].table_rows = (int)(tabs[i].numel() / (2 * C));
    a[i].shift = shifts[i].data_ptr<float>();
    a[i].running_mean = rm[i].data_ptr<float>();
    a[i].running_var = rv[i].data_ptr<float>();
    float* st = stats.data_ptr<float>() + (int64_t)i * 4 * C;
    a[i].save_mean = st;
    a[i].save_invstd = st + C;
    a[i].save_ss = st + 2 * C;
    a[i].num_batches = nbt_ptr(nb[i], x);
  }
  CHECK_HIP_OK(pda::bn_fwd_train_sums_dual(bp(x), bp(x2), bpm(y), M, C, a[0], a[1], (float)momentum, (float)eps,
                                           bits.data_ptr<uint8_t>(), stream_of(x)));
  return {y, bits, stats[0][0], stats[0][1], stats[1][0], stats[1][1]};
}

bool bn_bwd_dual_ok(int64_t C) { return pda::bn_bwd_dual_ok(C); }

// backward of bn_fwd_train_sums_dual: {dx, dx2, dgamma, dbeta, dgamma2, dbeta2}; the parameter gradients
// go to the given outputs (flat-buffer slots) when passed, else are allocated in the parameter dtype
std::vector<Tensor> bn_bwd_dual(Tensor dy, Tensor bits, Tensor x, Tensor mean, Tensor invstd,
                                c10::optional<Tensor> gamma, Tensor x2, Tensor mean2, Tensor invstd2,
                                c10::optional<Tensor> gamma2, c10::optional<Tensor> dgamma_out,
                                c10::optional<Tensor> dbeta_out, c10::optional<Tensor> dgamma2_out,
                                c10::optional<Tensor> dbeta2_out, c10::optional<Tensor> table,
                                c10::optional<Tensor> table2) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  check_bf16(x2, "x2");
  TORCH_CHECK(dy.sizes() == x.sizes() && x2.sizes() == x.sizes(), "dual BN backward: one shape for dy, x, x2");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(pda::bn_bwd_dual_ok(C), "dual BN backward needs C with 1 or 2 register coefficient sets");
  check_gpu(bits, "relu_bits");
  TORCH_CHECK(bits.scalar_type() == at::kByte && bits.is_contiguous() && bits.numel() * 8 == x.numel(),
              "relu bit mask must hold numel/8 bytes");
  c10::DeviceGuard g(x.device());
  Tensor xs[2] = {x, x2}, means[2] = {mean, mean2}, invs[2] = {invstd, invstd2};
  c10::optional<Tensor> gam[2] = {gamma, gamma2}, dgo[2] = {dgamma_out, dgamma2_out}, dbo[2] = {dbeta_out, dbeta2_out};
  Tensor dxs[2], dgs[2], dbs[2], wss[2];
  pda::BnBwdSide side[2] = {};
  TORCH_CHECK(table.has_value() == table2.has_value(), "bn_bwd_dual: both tables or none");
  c10::optional<Tensor> tabs[2] = {table, table2};
  for (int i = 0; i < 2; ++i) {
    if (tabs[i].has_value()) {
      check_f32(*tabs[i], "table");
      TORCH_CHECK(tabs[i]->dim() == 3 && tabs[i]->size(1) == 2 && tabs[i]->size(2) == C && tabs[i]->is_contiguous());
      side[i].table = tabs[i]->data_ptr<float>();
      side[i].rows = (int)tabs[i]->size(0);
    }
    check_f32(means[i], "mean");
    check_f32(invs[i], "invstd");
    bn_param_ptrs(gam[i], &side[i].gamma_f, &side[i].gamma_b, C);
    const auto pdt = gam[i].has_value() ? gam[i]->scalar_type() : at::kFloat;
    dxs[i] = at::empty_like(x);
    dgs[i] = dgo[i].has_value() ? *dgo[i] : at::empty({C}, x.options().dtype(pdt));
    dbs[i] = dbo[i].has_value() ? *dbo[i] : at::empty({C}, x.options().dtype(pdt));
    TORCH_CHECK(dgs[i].numel() == C && dbs[i].numel() == C && dgs[i].scalar_type() == pdt &&
                dbs[i].scalar_type() == pdt);
    check_gpu(dgs[i], "dgamma");
    check_gpu(dbs[i], "dbeta");
    wss[i] = at::empty({pda::bn_workspace_floats(M, C)}, x.options().dtype(at::kFloat));
    const bool pb = pdt == at::kBFloat16;
    side[i].x = bp(xs[i]);
    side[i].mean = means[i].data_ptr<float>();
    side[i].invstd = invs[i].data_ptr<float>();
    side[i].dx = bpm(dxs[i]);
    side[i].dgamma_f = pb ? nullptr : dgs[i].data_ptr<float>();
    side[i].dgamma_b = pb ? bpm(dgs[i]) : nullptr;
    side[i].dbeta_f = pb ? nullptr : dbs[i].data_ptr<float>();
    side[i].dbeta_b = pb ? bpm(dbs[i]) : nullptr;
    side[i].ws = wss[i].data_ptr<float>();
  }
  CHECK_HIP_OK(pda::bn_bwd_dual(bp(dy), bits.data_ptr<uint8_t>(), M, C, side[0], side[1], stream_of(x)));
  return {dxs[0], dxs[1], dgs[0], dbs[0], dgs[1], dbs[1]};
}

Tensor bn_fwd_eval(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> gamma, c10::optional<Tensor> beta,
                   Tensor running_mean, Tensor running_var, double eps, bool relu) {
  check_bf16(x, "x");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "channels must be a multiple of 8 and <= 2048");
  if (res) check_bf16(*res, "residual");
  const float *gf, *bfp;
  const pda::bf16_t *gb, *bb;
  bn_param_ptrs(gamma, &gf, &gb, C);
  bn_param_ptrs(beta, &bfp, &bb, C);
  check_f32(running_mean, "running_mean");
  check_f32(running_var, "running_var");
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  Tensor ws = at::empty({2 * C}, x.options().dtype(at::kFloat));
  CHECK_HIP_OK(pda::bn_fwd_eval(bp(x), res ? bp(*res) : nullptr, bpm(y), M, C, gf, gb, bfp, bb,
                                running_mean.data_ptr<float>(), running_var.data_ptr<float>(), (float)eps, relu,
                                ws.data_ptr<float>(), stream_of(x)));
  return y;
}

// In-launch BN-backward finalize (batchnorm.hip:bwd_fused_finish) for C <= this threshold.  Default 0
// (off): measured on ResNet-50 bs 640 (profiles/r2_bn_bwd_fused_finalize_DROPPED.jsonl) it is neutral
// for C <= 256 and -1.2 % at 2048 (the atomic adds of ~1024 blocks into a few table rows contend at the
// memory side); the separate finalize launch's long dispatch waits beside the side-stream wgrads are
// time the GPU spends on those wgrads anyway.  PDA_BN_BWD_FUSED_MAXC or set_bn_bwd_fused_max_c().
int64_t& bn_bwd_fused_max_c() {
  static int64_t v = [] {
    const char* e = getenv("PDA_BN_BWD_FUSED_MAXC");
    return e ? (int64_t)atoll(e) : (int64_t)0;
  }();
  return v;
}
void set_bn_bwd_fused_max_c(int64_t c) { bn_bwd_fused_max_c() = c; }

std::vector<Tensor> bn_bwd(Tensor dy, Tensor x, c10::optional<Tensor> y, c10::optional<Tensor> ss, Tensor mean,
                           Tensor invstd, c10::optional<Tensor> gamma, bool relu, bool want_dres,
                           c10::optional<Tensor> dgamma_out, c10::optional<Tensor> dbeta_out) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes());
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "channels must be a multiple of 8 and <= 2048");
  const bool bits = relu && y.has_value() && y->scalar_type() == at::kByte;
  if (relu) {
    TORCH_CHECK(y.has_value() || ss.has_value(), "relu backward needs the saved output, its bit mask or scale/shift");
    if (bits) {
      check_gpu(*y, "relu_bits");
      TORCH_CHECK(y->is_contiguous() && y->numel() * 8 == x.numel(), "relu bit mask must hold numel/8 bytes");
    } else if (y.has_value()) check_bf16(*y, "y");
    else {
      check_f32(*ss, "ss");
      TORCH_CHECK(ss->numel() == 2 * C);
    }
  }
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  const float* gf;
  const pda::bf16_t* gb;
  bn_param_ptrs(gamma, &gf, &gb, C);
  c10::DeviceGuard g(x.device());
  Tensor dx = at::empty_like(x);
  Tensor dres = want_dres ? at::empty_like(x) : Tensor();
  // parameter gradients are produced directly in the parameter dtype (no cast kernels)
  const auto pdt = gamma.has_value() ? gamma->scalar_type() : at::kFloat;
  Tensor dgamma = dgamma_out.has_value() ? *dgamma_out : at::empty({C}, x.options().dtype(pdt));
  Tensor dbeta = dbeta_out.has_value() ? *dbeta_out : at::empty({C}, x.options().dtype(pdt));
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.scalar_type() == pdt && dbeta.scalar_type() == pdt);
  check_gpu(dgamma, "dgamma");
  check_gpu(dbeta, "dbeta");
  const bool pb = pdt == at::kBFloat16;
  // fused finalize for C <= PDA_BN_BWD_FUSED_MAXC (0 -> always the separate finalize launch): a persistent zeroed
  // table + ticket per (device, stream) — BN backwards on one stream are serialised, and every call
  // leaves both zero again
  const bool fused = C <= bn_bwd_fused_max_c();
  float* fin_table = nullptr;
  unsigned* fin_ticket = nullptr;
  const int fin_rows = pda::bn_bwd_table_rows(C);
  hipStream_t st = stream_of(x);
  if (fused) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, Tensor> tables;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair((int)x.device().index(), st);
    auto it = tables.find(key);
    if (it == tables.end()) {
      // [128 rows x 2 x 2048] floats covers every (rows, C) pair; + 16 floats for the ticket
      it = tables.emplace(key, at::zeros({128 * 2 * 2048 + 16}, x.options().dtype(at::kFloat))).first;
    }
    fin_table = it->second.data_ptr<float>();
    fin_ticket = reinterpret_cast<unsigned*>(fin_table + 128 * 2 * 2048);
    TORCH_CHECK((int64_t)fin_rows * 2 * C <= 128 * 2 * 2048);
  }
  Tensor ws = at::empty({fused ? 3 * C : pda::bn_workspace_floats(M, C)}, x.options().dtype(at::kFloat));
  const float* ssp = (relu && !y.has_value()) ? ss->data_ptr<float>() : nullptr;
  CHECK_HIP_OK(pda::bn_bwd(bp(dy), bp(x), (relu && y.has_value() && !bits) ? bp(*y) : nullptr,
                           bits ? y->data_ptr<uint8_t>() : nullptr, ssp, M, C, mean.data_ptr<float>(),
                           invstd.data_ptr<float>(), gf, gb, relu, bpm(dx), want_dres ? bpm(dres) : nullptr,
                           pb ? nullptr : dgamma.data_ptr<float>(), pb ? bpm(dgamma) : nullptr,
                           pb ? nullptr : dbeta.data_ptr<float>(), pb ? bpm(dbeta) : nullptr, ws.data_ptr<float>(),
                           fin_table, fin_ticket, fin_rows, st));
  return {dx, dres, dgamma, dbeta};
}

// BN backward from the sums a dgrad epilogue accumulated into `table` (conv_dgrad bst_*): finalize (re-zeroes
// the table) + apply; y = the forward's ReLU bit mask (uint8) or None with ss = scale / shift
std::vector<Tensor> bn_bwd_table(Tensor dy, Tensor x, c10::optional<Tensor> bits, c10::optional<Tensor> ss,
                                 Tensor mean, Tensor invstd, c10::optional<Tensor> gamma, bool relu, bool want_dres,
                                 Tensor table, c10::optional<Tensor> dgamma_out, c10::optional<Tensor> dbeta_out) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes());
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "channels must be a multiple of 8 and <= 2048");
  check_f32(table, "table");
  TORCH_CHECK(table.dim() == 3 && table.size(1) == 2 && table.size(2) == C && table.is_contiguous());
  if (relu) {
    TORCH_CHECK(bits.has_value() || ss.has_value(), "relu backward needs the bit mask or scale/shift");
    if (bits.has_value()) {
      check_gpu(*bits, "bits");
      TORCH_CHECK(bits->scalar_type() == at::kByte && bits->is_contiguous() && bits->numel() * 8 == x.numel());
    } else {
      check_f32(*ss, "ss");
      TORCH_CHECK(ss->numel() == 2 * C);
    }
  }
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  const float* gf;
  const pda::bf16_t* gb;
  bn_param_ptrs(gamma, &gf, &gb, C);
  c10::DeviceGuard g(x.device());
  Tensor dx = at::empty_like(x);
  Tensor dres = want_dres ? at::empty_like(x) : Tensor();
  const auto pdt = gamma.has_value() ? gamma->scalar_type() : at::kFloat;
  Tensor dgamma = dgamma_out.has_value() ? *dgamma_out : at::empty({C}, x.options().dtype(pdt));
  Tensor dbeta = dbeta_out.has_value() ? *dbeta_out : at::empty({C}, x.options().dtype(pdt));
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.scalar_type() == pdt && dbeta.scalar_type() == pdt);
  const bool pb = pdt == at::kBFloat16;
  Tensor coef = at::empty({3 * C}, x.options().dtype(at::kFloat));
  CHECK_HIP_OK(pda::bn_bwd_table(bp(dy), bp(x), (relu && bits.has_value()) ? bits->data_ptr<uint8_t>() : nullptr,
                                 (relu && !bits.has_value()) ? ss->data_ptr<float>() : nullptr, M, C,
                                 mean.data_ptr<float>(), invstd.data_ptr<float>(), gf, gb, relu, bpm(dx),
                                 want_dres ? bpm(dres) : nullptr, pb ? nullptr : dgamma.data_ptr<float>(),
                                 pb ? bpm(dgamma) : nullptr, pb ? nullptr : dbeta.data_ptr<float>(),
                                 pb ? bpm(dbeta) : nullptr, table.data_ptr<float>(), (int)table.size(0),
                                 coef.data_ptr<float>(), stream_of(x)));
  return {dx, dres, dgamma, dbeta};
}

// ------------------------------------------------------------------ pooling (NHWC)
std::vector<Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t s, int64_t pad) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "x must be [N,H,W,C]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k * k <= 255);
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, P, Q, C}, x.options());
  Tensor idx = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  CHECK_HIP_OK(pda::maxpool2d_fwd(bp(x), bpm(y), idx.data_ptr<uint8_t>(), N, H, W, C, P, Q, k, s, pad, stream_of(x)));
  return {y, idx};
}

// stem: BN finalize from the conv epilogue's table, then maxpool of relu(bn(x)) without storing the BN
// output; returns {y, idx, mean, invstd, ss}
std::vector<Tensor> bn_relu_maxpool_fwd(Tensor x, Tensor table, Tensor shift, c10::optional<Tensor> gamma,
                                        c10::optional<Tensor> beta, Tensor running_mean, Tensor running_var,
                                        c10::optional<Tensor> num_batches, double momentum, double eps, int64_t k,
                                        int64_t s, int64_t pad) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "x must be a contiguous [N,H,W,C] tensor");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && k * k <= 255);
  check_f32(table, "table");
  check_f32(shift, "shift");
  check_f32(running_mean, "running_mean");
  check_f32(running_var, "running_var");
  TORCH_CHECK(shift.numel() == C && table.numel() % (2 * C) == 0 && table.numel() > 0 && table.is_contiguous(),
              "table must be [R, 2, C]");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  c10::DeviceGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat);
  Tensor stats = at::empty({4, C}, fo);  // mean, invstd, scale, shift
  pda::BnSumsArgs a;
  bn_param_ptrs(gamma, &a.gamma_f, &a.gamma_b, C);
  bn_param_ptrs(beta, &a.beta_f, &a.beta_b, C);
  a.table = table.data_ptr<float>();
  a.table_rows = (int)(table.numel() / (2 * C));
  a.shift = shift.data_ptr<float>();
  a.running_mean = running_mean.data_ptr<float>();
  a.running_var = running_var.data_ptr<float>();
  a.save_mean = stats.data_ptr<float>();
  a.save_invstd = a.save_mean + C;
  a.save_ss = a.save_mean + 2 * C;
  a.num_batches = nbt_ptr(num_batches, x);
  hipStream_t st = stream_of(x);
  CHECK_HIP_OK(pda::bn_finalize_sums(bp(x), (int64_t)N * H * W, C, a, (float)momentum, (float)eps, st));
  Tensor y = at::empty({N, P, Q, C}, x.options());
  Tensor idx = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  CHECK_HIP_OK(pda::maxpool2d_bn_fwd(bp(x), a.save_ss, bpm(y), idx.data_ptr<uint8_t>(), N, H, W, C, P, Q, k, s, pad,
                                     st));
  return {y, idx, stats[0], stats[1], stats.narrow(0, 2, 2)};
}

bool stem_pool_bn_bwd_ok(int64_t H, int64_t W, int64_t C, int64_t k, int64_t s, int64_t pad) {
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  return pda::stem_pool_bn_bwd_ok((int)H, (int)W, (int)C, P, Q, (int)k, (int)s, (int)pad);
}

// backward of bn_relu_maxpool_fwd (3x3 / 2 / pad 1): {dz, dgamma, dbeta}
std::vector<Tensor> stem_pool_bn_bwd(Tensor dp, Tensor idx, Tensor z, Tensor ss, Tensor mean, Tensor invstd,
                                     c10::optional<Tensor> gamma, c10::optional<Tensor> dgamma_out,
                                     c10::optional<Tensor> dbeta_out) {
  check_bf16(dp, "dp");
  check_bf16(z, "z");
  TORCH_CHECK(z.dim() == 4 && dp.dim() == 4 && z.is_contiguous() && dp.is_contiguous());
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3), P = dp.size(1), Q = dp.size(2);
  TORCH_CHECK(dp.size(0) == N && dp.size(3) == C && idx.numel() == dp.numel() && idx.scalar_type() == at::kByte);
  TORCH_CHECK(pda::stem_pool_bn_bwd_ok(H, W, C, P, Q, 3, 2, 1), "stem pool+BN backward: 3x3/2/1 pool only");
  check_f32(ss, "ss");
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  TORCH_CHECK(ss.numel() == 2 * C && ss.is_contiguous());
  const float* gf;
  const pda::bf16_t* gb;
  bn_param_ptrs(gamma, &gf, &gb, C);
  c10::DeviceGuard g(z.device());
  const auto pdt = gamma.has_value() ? gamma->scalar_type() : at::kFloat;
  Tensor dz = at::empty_like(z);
  Tensor dgamma = dgamma_out.has_value() ? *dgamma_out : at::empty({C}, z.options().dtype(pdt));
  Tensor dbeta = dbeta_out.has_value() ? *dbeta_out : at::empty({C}, z.options().dtype(pdt));
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.scalar_type() == pdt && dbeta.scalar_type() == pdt);
  const bool pb = pdt == at::kBFloat16;
  Tensor ws = at::empty({pda::stem_pool_bn_bwd_ws_floats(C)}, z.options().dtype(at::kFloat));
  CHECK_HIP_OK(pda::stem_pool_bn_bwd(bp(dp), idx.data_ptr<uint8_t>(), bp(z), ss.data_ptr<float>(),
                                     mean.data_ptr<float>(), invstd.data_ptr<float>(), gf, gb, N, H, W, C, P, Q,
                                     bpm(dz), pb ? nullptr : dgamma.data_ptr<float>(), pb ? bpm(dgamma) : nullptr,
                                     pb ? nullptr : dbeta.data_ptr<float>(), pb ? bpm(dbeta) : nullptr,
                                     ws.data_ptr<float>(), stream_of(z)));
  return {dz, dgamma, dbeta};
}

// x [N,H,W,Cx] bf16 (first c channels used) -> [N, ceil((H+2pad)/2), ceil((W+2pad)/2), 16]
Tensor stem_s2d(Tensor x, int64_t c, int64_t pad) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "x must be a contiguous [N,H,W,C] tensor");
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cx = x.size(3);
  TORCH_CHECK(c >= 1 && c <= Cx && 4 * c <= 16, "stem_s2d: 1 <= c <= min(Cx, 4)");
  const int U = (H + 2 * pad + 1) / 2, V = (W + 2 * pad + 1) / 2;
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, U, V, 16}, x.options());
  CHECK_HIP_OK(pda::stem_space_to_depth(bp(x), bpm(y), N, H, W, Cx, (int)c, U, V, (int)pad, stream_of(x)));
  return y;
}

Tensor maxpool_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad) {
  check_bf16(dy, "dy");
  check_gpu(idx, "idx");
  TORCH_CHECK(idx.sizes() == dy.sizes());
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  c10::DeviceGuard g(dy.device());
  Tensor dx = at::empty({N, H, W, C}, dy.options());
  CHECK_HIP_OK(pda::maxpool2d_bwd(bp(dy), idx.data_ptr<uint8_t>(), bpm(dx), N, H, W, C, P, Q, k, s, pad,
                                  stream_of(dy)));
  return dx;
}

Tensor avgpool_fwd(Tensor x, bool out_bf16) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0);
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, C}, x.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  CHECK_HIP_OK(pda::avgpool_global_fwd(bp(x), y.data_ptr(), out_bf16, N, HW, C, stream_of(x)));
  return y;
}

Tensor avgpool_bwd(Tensor dy, int64_t H, int64_t W) {
  check_f32_or_bf16(dy, "dy");
  const int N = dy.size(0), C = dy.size(1);
  c10::DeviceGuard g(dy.device());
  Tensor dx = at::empty({N, H, W, C}, dy.options().dtype(at::kBFloat16));
  CHECK_HIP_OK(pda::avgpool_global_bwd(dy.data_ptr(), is_bf16(dy), bpm(dx), N, H * W, C, stream_of(dy)));
  return dx;
}

// ------------------------------------------------------------------ synthetic data
void fill_random(Tensor t, int64_t seed, int64_t offset, int64_t kind, double a, double b) {
  check_f32_or_bf16(t, "tensor");
  c10::DeviceGuard g(t.device());
  CHECK_HIP_OK(pda::fill_random(t.data_ptr(), is_bf16(t) ? 1 : 0, t.numel(), (uint64_t)seed, (uint64_t)offset,
                                (int)kind, (float)a, (float)b, stream_of(t)));
}
void fill_randint(Tensor t, int64_t seed, int64_t offset, int64_t low, int64_t high) {
  check_gpu(t, "tensor");
  TORCH_CHECK(t.scalar_type() == at::kLong && high > low);
  c10::DeviceGuard g(t.device());
  CHECK_HIP_OK(pda::fill_randint(t.data_ptr<int64_t>(), t.numel(), (uint64_t)seed, (uint64_t)offset, low, high,
                                 stream_of(t)));
}

// ------------------------------------------------------------------ GEMM / conv
// C = A * B with A(m,k) = A[m*lda+k] (a_kmajor) or A[k*lda+m]; B(k,n) = B[n*ldb+k] (b_kmajor) or B[k*ldb+n].
void gemm(Tensor A, bool a_kmajor, int64_t lda, Tensor B, bool b_kmajor, int64_t ldb, Tensor C, int64_t ldc,
          int64_t M, int64_t N, int64_t K, c10::optional<Tensor> bias, bool relu, bool allow_split) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_f32_or_bf16(C, "C");
  TORCH_CHECK(N % 8 == 0, "gemm needs N multiple of 8 (got N=", N, ")");
  TORCH_CHECK((!a_kmajor && !b_kmajor) || K % 8 == 0, "gemm with a K-major operand needs K % 8 == 0 (got K=", K, ")");
  TORCH_CHECK(a_kmajor || M % 8 == 0, "M-major A needs M % 8 == 0");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "leading dims must be 16-byte multiples");
  // bounds: the largest element each operand touches
  TORCH_CHECK((a_kmajor ? (M - 1) * lda + K : (K - 1) * lda + M) <= A.numel(), "A too small");
  TORCH_CHECK((b_kmajor ? (N - 1) * ldb + K : (K - 1) * ldb + N) <= B.numel(), "B too small");
  TORCH_CHECK((M - 1) * ldc + N <= C.numel(), "C too small");
  for (auto* t : {&A, &B, &C}) check_aligned16(*t, "gemm operand");
  if (bias) {
    check_f32_or_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N);
  }
  c10::DeviceGuard g(A.device());
  const int64_t slab_n = pda::gemm_slab_floats(M, N, K, allow_split);
  Tensor slab = slab_n > 0 ? at::empty({slab_n}, A.options().dtype(at::kFloat)) : Tensor();
  CHECK_HIP_OK(pda::gemm_bf16(bp(A), a_kmajor, lda, bp(B), b_kmajor, ldb, C.data_ptr(), C.scalar_type() == at::kFloat,
                              ldc, M, N, K, bias ? bias->data_ptr() : nullptr, bias ? !is_bf16(*bias) : false, relu,
                              slab_n > 0 ? slab.data_ptr<float>() : nullptr, slab_n > 0, stream_of(A)));
}

// Weight + bias gradient of a Linear in one pipelined GEMM: dw[N, K] = dy^T x (dy [M, N], x [M, K]) and
// db[N] = column sums of dy.  Returns whether db was written (false: the shape did not take the
// 256 x 256 pipelined path; the caller reduces dy itself).
bool gemm_wgrad_db(Tensor dy, Tensor x, Tensor dw, Tensor db) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  check_f32_or_bf16(dw, "dw");
  check_f32_or_bf16(db, "db");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0) && dy.is_contiguous() && x.is_contiguous());
  const int64_t T = dy.size(0), Nout = dy.size(1), Kin = x.size(1);
  TORCH_CHECK(Nout % 8 == 0 && Kin % 8 == 0, "gemm_wgrad_db needs in / out features multiples of 8");
  TORCH_CHECK(dw.numel() == Nout * Kin && dw.is_contiguous() && db.numel() == Nout && db.is_contiguous());
  for (auto* t : {&dy, &x, &dw}) check_aligned16(*t, "gemm_wgrad_db operand");
  c10::DeviceGuard g(dy.device());
  const int64_t slab_n = pda::gemm_slab_floats(Nout, Kin, T, true);
  // [splits][Nout] split-K row sums after the slab (its split count bounds the launch's)
  const int64_t rs_n = slab_n > 0 ? slab_n / Kin : Nout;
  Tensor scratch = at::empty({slab_n + rs_n}, dy.options().dtype(at::kFloat));
  int done = 0;
  CHECK_HIP_OK(pda::gemm_bf16_wgrad_db(bp(dy), Nout, bp(x), Kin, dw.data_ptr(), dw.scalar_type() == at::kFloat, Kin,
                                       Nout, Kin, T, db.data_ptr(), is_bf16(db),
                                       slab_n > 0 ? scratch.data_ptr<float>() : nullptr,
                                       scratch.data_ptr<float>() + slab_n, stream_of(dy), &done));
  return done != 0;
}

// GEMM with a fused GELU-tanh epilogue (bf16 C [M, ldc]):
//   act 1 (forward):  C = gelu(A B + bias) and aux = A B + bias (the pre-activation the backward needs)
//   act 2 (backward): C = (A B) * gelu'(aux), aux = that pre-activation
void gemm_act(Tensor A, bool a_kmajor, int64_t lda, Tensor B, bool b_kmajor, int64_t ldb, Tensor C, int64_t ldc,
              int64_t M, int64_t N, int64_t K, c10::optional<Tensor> bias, int64_t act, Tensor aux) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_bf16(C, "C");
  check_bf16(aux, "aux");
  TORCH_CHECK(act == 1 || act == 2, "act must be 1 (gelu fwd) or 2 (gelu bwd)");
  TORCH_CHECK(N % 8 == 0 && ldc % 8 == 0, "gemm_act needs N and ldc multiples of 8");
  TORCH_CHECK((!a_kmajor && !b_kmajor) || K % 8 == 0, "gemm with a K-major operand needs K % 8 == 0");
  TORCH_CHECK(a_kmajor || M % 8 == 0, "M-major A needs M % 8 == 0");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "leading dims must be 16-byte multiples");
  TORCH_CHECK((a_kmajor ? (M - 1) * lda + K : (K - 1) * lda + M) <= A.numel(), "A too small");
  TORCH_CHECK((b_kmajor ? (N - 1) * ldb + K : (K - 1) * ldb + N) <= B.numel(), "B too small");
  TORCH_CHECK((M - 1) * ldc + N <= C.numel() && (M - 1) * ldc + N <= aux.numel(), "C / aux too small");
  for (auto* t : {&A, &B, &C, &aux}) check_aligned16(*t, "gemm_act operand");
  if (bias) {
    check_f32_or_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && act == 1, "bias only with the forward activation");
  }
  c10::DeviceGuard g(A.device());
  CHECK_HIP_OK(pda::gemm_bf16_act(bp(A), a_kmajor, lda, bp(B), b_kmajor, ldb, bpm(C), ldc, M, N, K,
                                  bias ? bias->data_ptr() : nullptr, bias ? !is_bf16(*bias) : false, (int)act,
                                  bpm(aux), stream_of(A)));
}

// Pipelined 256x256 GEMM (gemm_pp.hip) lab entry: C[M,N] = A B (+ bias), bf16; operand majorness as
// gemm(): A(m,k) = A[m*lda+k] (a_kmajor) or A[k*lda+m]; B(k,n) = B[n*ldb+k] (b_kmajor) or B[k*ldb+n].
void gemm_pp_lab(Tensor A, bool a_kmajor, int64_t lda, Tensor B, bool b_kmajor, int64_t ldb, Tensor C, int64_t ldc,
                 int64_t M, int64_t N, int64_t K, c10::optional<Tensor> bias, int64_t variant) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_bf16(C, "C");
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0 && (a_kmajor || M % 8 == 0), "gemm_pp needs N, K (and M-major M) % 8 == 0");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0, "leading dims must be 16-byte multiples");
  TORCH_CHECK((a_kmajor ? (M - 1) * lda + K : (K - 1) * lda + M) <= A.numel(), "A too small");
  TORCH_CHECK((b_kmajor ? (N - 1) * ldb + K : (K - 1) * ldb + N) <= B.numel(), "B too small");
  TORCH_CHECK((M - 1) * ldc + N <= C.numel(), "C too small");
  for (auto* t : {&A, &B, &C}) check_aligned16(*t, "gemm_pp operand");
  if (bias) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N);
  }
  c10::DeviceGuard g(A.device());
  CHECK_HIP_OK(pda::gemm_pp_lab(bp(A), a_kmajor, lda, bp(B), b_kmajor, ldb, bpm(C), ldc, M, N, K,
                                bias ? bp(*bias) : nullptr, (int)variant, stream_of(A)));
}

void conv_check(const Tensor& x, const Tensor& w) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv tensors must be 4-D (NHWC activations, OHWI weights)");
  TORCH_CHECK(x.size(3) % 8 == 0, "input channels must be a multiple of 8");
  TORCH_CHECK(w.size(0) % 8 == 0, "output channels must be a multiple of 8");
  TORCH_CHECK(w.size(3) == x.size(3), "channel mismatch");
  TORCH_CHECK(x.numel() < (1LL << 31), "activation too large for 32-bit index math");
}

Tensor conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil, c10::optional<Tensor> bias, bool relu,
                bool out_f32) {
  conv_check(x, w);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Cout = w.size(0), R = w.size(1), S = w.size(2);
  const int P = (H + 2 * pad - dil * (R - 1) - 1) / stride + 1, Q = (W + 2 * pad - dil * (S - 1) - 1) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0);
  if (bias) TORCH_CHECK(bias->numel() == Cout);
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, P, Q, Cout}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  CHECK_HIP_OK(pda::conv2d_fwd(bp(x), bp(w), y.data_ptr(), out_f32, N, H, W, C, Cout, R, S, P, Q, stride, pad, dil,
                               bias ? bias->data_ptr() : nullptr, bias ? !is_bf16(*bias) : false, relu, nullptr,
                               nullptr, 0, stream_of(x)));
  return y;
}

// conv forward that also accumulates the BatchNorm sums of its output into `table` ([R, 2, Cout] fp32,
// zero on entry; the BN finalize that consumes it zeroes it again): table[r][0] += sum(y - shift),
// table[r][1] += sum((y - shift)^2) over the output tiles with tile_m % R == r (no statistics pass)
Tensor conv_fwd_stats(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil, Tensor shift, Tensor table) {
  conv_check(x, w);
  check_f32(shift, "shift");
  check_f32(table, "table");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Cout = w.size(0), R = w.size(1), S = w.size(2);
  TORCH_CHECK(shift.numel() == Cout);
  TORCH_CHECK(table.numel() % (2 * (int64_t)Cout) == 0 && table.numel() > 0 && table.is_contiguous(),
              "table must be [R, 2, Cout]");
  TORCH_CHECK(table.device() == x.device() && shift.device() == x.device());
  const int P = (H + 2 * pad - dil * (R - 1) - 1) / stride + 1, Q = (W + 2 * pad - dil * (S - 1) - 1) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0);
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, P, Q, Cout}, x.options());
  const int rows = (int)(table.numel() / (2 * (int64_t)Cout));
  CHECK_HIP_OK(pda::conv2d_fwd(bp(x), bp(w), bpm(y), false, N, H, W, C, Cout, R, S, P, Q, stride, pad, dil, nullptr, false,
                               false, table.data_ptr<float>(), shift.data_ptr<float>(), rows, stream_of(x)));
  return y;
}

// addend_bits: optional ReLU bit mask of the addend (numel/8 bytes): dx = dgrad + addend * mask
// bst_*: the BN-backward statistics of dx accumulated in the epilogue (pda::BnBwdStats): z = the BN's input
// (dx's shape), ss = its [2][C] scale / shift (ReLU mask recomputed) or bits = its forward ReLU bit mask,
// mean = its saved batch mean, table = [R][2][C] fp32 zero on entry (bn_bwd_table re-zeroes it)
Tensor conv_dgrad(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t stride, int64_t pad, int64_t dil,
                  c10::optional<Tensor> addend, c10::optional<Tensor> addend_bits, bool out_f32,
                  c10::optional<Tensor> bst_z, c10::optional<Tensor> bst_ss, c10::optional<Tensor> bst_bits,
                  c10::optional<Tensor> bst_mean, c10::optional<Tensor> bst_table, c10::optional<Tensor> bst_z2,
                  c10::optional<Tensor> bst_mean2, c10::optional<Tensor> bst_table2) {
  check_bf16(dy, "dy");
  check_bf16(w, "w");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), Cout = dy.size(3);
  const int R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(w.size(0) == Cout && C % 8 == 0 && Cout % 8 == 0);
  c10::DeviceGuard g(dy.device());
  Tensor wt;
  if (pda::conv_dgrad_needs_wt(R, S, (int)stride, (int)pad) ||
      pda::conv_dgrad_1x1_wt(R, S, (int)stride, (int)pad, C, Cout)) {
    wt = at::empty({C, R, S, Cout}, w.options());
    CHECK_HIP_OK(pda::conv_weight_transpose(bp(w), bpm(wt), Cout, R, S, C, stride, pad, dil, stream_of(dy)));
  }
  Tensor dx = at::empty({N, H, W, C}, dy.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  TORCH_CHECK(!(out_f32 && addend.has_value()), "conv_dgrad: an addend needs the bf16 output");
  if (addend.has_value()) {
    check_bf16(*addend, "addend");
    TORCH_CHECK(addend->sizes() == dx.sizes() && addend->is_contiguous(), "addend must have dx's shape");
  }
  if (addend_bits.has_value()) {
    TORCH_CHECK(addend.has_value(), "addend_bits without an addend");
    check_gpu(*addend_bits, "addend_bits");
    TORCH_CHECK(addend_bits->scalar_type() == at::kByte && addend_bits->is_contiguous() &&
                    addend_bits->numel() * 8 == dx.numel(),
                "addend_bits must be numel/8 contiguous bytes");
  }
  pda::BnBwdStats bst{};
  const bool want_bst = bst_z.has_value();
  if (want_bst) {
    TORCH_CHECK(!out_f32 && !(addend.has_value() && stride > 1),
                "conv_dgrad: BN-backward statistics need a bf16 dx (and no addend on a strided dgrad)");
    check_bf16(*bst_z, "bst_z");
    TORCH_CHECK(bst_z->sizes() == dx.sizes() && bst_z->is_contiguous(), "bst_z must have dx's shape");
    TORCH_CHECK(bst_mean.has_value() && bst_table.has_value(), "bst_z needs bst_mean and bst_table");
    check_f32(*bst_mean, "bst_mean");
    check_f32(*bst_table, "bst_table");
    TORCH_CHECK(bst_mean->numel() == C && bst_table->dim() == 3 && bst_table->size(1) == 2 && bst_table->size(2) == C &&
                    bst_table->is_contiguous(),
                "bst_table must be a contiguous [R, 2, C] fp32 table");
    TORCH_CHECK(bst_ss.has_value() != bst_bits.has_value(), "exactly one of bst_ss / bst_bits");
    bst.z = bp(*bst_z);
    bst.mean = bst_mean->data_ptr<float>();
    bst.table = bst_table->data_ptr<float>();
    bst.rows = (int)bst_table->size(0);
    if (bst_ss.has_value()) {
      check_f32(*bst_ss, "bst_ss");
      TORCH_CHECK(bst_ss->numel() == 2 * C);
      bst.ss = bst_ss->data_ptr<float>();
    } else {
      check_gpu(*bst_bits, "bst_bits");
      TORCH_CHECK(bst_bits->scalar_type() == at::kByte && bst_bits->is_contiguous() && bst_bits->numel() * 8 == dx.numel());
      bst.bits = bst_bits->data_ptr<uint8_t>();
    }
    if (bst_z2.has_value()) {
      check_bf16(*bst_z2, "bst_z2");
      TORCH_CHECK(bst_z2->sizes() == dx.sizes() && bst_z2->is_contiguous(), "bst_z2 must have dx's shape");
      TORCH_CHECK(bst_mean2.has_value() && bst_table2.has_value(), "bst_z2 needs bst_mean2 and bst_table2");
      check_f32(*bst_mean2, "bst_mean2");
      check_f32(*bst_table2, "bst_table2");
      TORCH_CHECK(bst_mean2->numel() == C && bst_table2->sizes() == bst_table->sizes() && bst_table2->is_contiguous());
      bst.z2 = bp(*bst_z2);
      bst.mean2 = bst_mean2->data_ptr<float>();
      bst.table2 = bst_table2->data_ptr<float>();
    }
  }
  CHECK_HIP_OK(pda::conv2d_dgrad(bp(dy), bp(w), wt.defined() ? bp(wt) : nullptr, dx.data_ptr(), out_f32, N, H, W, C, Cout, R, S, P, Q, stride, pad, dil,
                                 addend.has_value() ? bp(*addend) : nullptr,
                                 addend_bits.has_value() ? addend_bits->data_ptr<uint8_t>() : nullptr, stream_of(dy),
                                 want_bst ? &bst : nullptr));
  return dx;
}

Tensor conv_wgrad(Tensor dy, Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t dil, bool out_f32,
                  c10::optional<Tensor> out) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = dy.size(1), Q = dy.size(2), Cout = dy.size(3);
  TORCH_CHECK(dy.size(0) == N && C % 8 == 0 && Cout % 8 == 0);
  c10::DeviceGuard g(dy.device());
  Tensor dw;
  if (out.has_value()) {  // write straight into e.g. a DDP gradient-bucket view
    dw = *out;
    check_gpu(dw, "out");
    TORCH_CHECK(dw.numel() == (int64_t)Cout * R * S * C && dw.scalar_type() == (out_f32 ? at::kFloat : at::kBFloat16));
    check_aligned16(dw, "out");
  } else {
    dw = at::empty({Cout, R, S, C}, dy.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  }
  const int64_t slab_n = pda::conv_slab_floats(2, N, H, W, C, Cout, R, S, P, Q);
  Tensor slab = slab_n > 0 ? at::empty({slab_n}, dy.options().dtype(at::kFloat)) : Tensor();
  CHECK_HIP_OK(pda::conv2d_wgrad(bp(dy), bp(x), dw.data_ptr(), out_f32, N, H, W, C, Cout, R, S, P, Q, stride, pad, dil,
                                 slab_n > 0 ? slab.data_ptr<float>() : nullptr, stream_of(dy)));
  return dw;
}

// ------------------------------------------------------------------ activations / SIMT GEMM
Tensor act_fwd(Tensor x, int64_t op) {
  check_f32_or_bf16(x, "x");
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  CHECK_HIP_OK(pda::act_fwd(x.data_ptr(), y.data_ptr(), is_bf16(x), x.numel(), (int)op, stream_of(x)));
  return y;
}

Tensor act_bwd(Tensor dy, Tensor ref, int64_t op) {
  check_f32_or_bf16(dy, "dy");
  check_gpu(ref, "ref");
  TORCH_CHECK(ref.sizes() == dy.sizes() && ref.scalar_type() == dy.scalar_type());
  c10::DeviceGuard g(dy.device());
  Tensor dx = at::empty_like(dy);
  CHECK_HIP_OK(pda::act_bwd(dy.data_ptr(), ref.data_ptr(), dx.data_ptr(), is_bf16(dy), dy.numel(), (int)op,
                            stream_of(dy)));
  return dx;
}

Tensor relu_bwd(Tensor dy, Tensor y) { return act_bwd(dy, y, 0); }

Tensor swiglu_fwd(Tensor gu) {
  check_f32_or_bf16(gu, "gate_up");
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu width must be a multiple of 8");
  const int64_t rows = gu.numel() / F2, F = F2 / 2;
  c10::DeviceGuard g(gu.device());
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  Tensor y = at::empty(sizes, gu.options());
  CHECK_HIP_OK(pda::swiglu_fwd(gu.data_ptr(), y.data_ptr(), is_bf16(gu), rows, F, stream_of(gu)));
  return y;
}

Tensor swiglu_bwd(Tensor dy, Tensor gu) {
  check_f32_or_bf16(dy, "dy");
  check_gpu(gu, "gate_up");
  const int64_t F2 = gu.size(-1), rows = gu.numel() / F2, F = F2 / 2;
  TORCH_CHECK(dy.numel() == rows * F);
  c10::DeviceGuard g(gu.device());
  Tensor dgu = at::empty_like(gu);
  CHECK_HIP_OK(pda::swiglu_bwd(dy.data_ptr(), gu.data_ptr(), dgu.data_ptr(), is_bf16(gu), rows, F, stream_of(gu)));
  return dgu;
}

// column sums (bias gradients); ``out``: write straight into that tensor (e.g. a bf16 gradient slot),
// otherwise a new tensor of dtype ``out_bf16 ? bf16 : fp32``
Tensor colsum(Tensor x, c10::optional<Tensor> out, bool out_bf16) {
  check_f32_or_bf16(x, "x");
  const int64_t cols = x.size(-1), rows = x.numel() / cols;
  c10::DeviceGuard g(x.device());
  Tensor o;
  if (out.has_value()) {
    o = *out;
    check_f32_or_bf16(o, "out");
    TORCH_CHECK(o.numel() == cols && o.is_contiguous(), "colsum: out must be [cols] contiguous");
  } else {
    o = at::empty({cols}, x.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  }
  if (cols % 8 != 0 || !x.is_contiguous()) {
    Tensor xc = x.contiguous();
    Tensor f = o.scalar_type() == at::kFloat ? o : at::empty({cols}, x.options().dtype(at::kFloat));
    CHECK_HIP_OK(pda::colsum_unaligned(xc.data_ptr(), is_bf16(x), f.data_ptr<float>(), rows, cols, stream_of(x)));
    if (!f.is_same(o)) o.copy_(f);
    return o;
  }
  Tensor ws = at::empty({pda::colreduce_ws_floats(rows, cols, 1)}, x.options().dtype(at::kFloat));
  CHECK_HIP_OK(pda::colsum(x.data_ptr(), is_bf16(x), o.data_ptr(), is_bf16(o), rows, cols, ws.data_ptr<float>(),
                           stream_of(x)));
  return o;
}

// C[M,N] (+)= A[M,K] B[K,N] with explicit element strides (any alignment / dtype fp32|bf16)
void simt_gemm(Tensor A, int64_t sam, int64_t sak, Tensor B, int64_t sbk, int64_t sbn, Tensor C, int64_t scm,
               int64_t scn, int64_t M, int64_t N, int64_t K, c10::optional<Tensor> bias, bool relu, double beta) {
  for (auto* t : {&A, &B, &C}) {
    TORCH_CHECK(t->is_cuda(), "simt_gemm operands must be GPU tensors");
    TORCH_CHECK(t->scalar_type() == at::kFloat || t->scalar_type() == at::kBFloat16, "fp32/bf16 only");
  }
  auto span = [](int64_t a, int64_t sa, int64_t b, int64_t sb) { return (a - 1) * sa + (b - 1) * sb + 1; };
  TORCH_CHECK(M > 0 && N > 0 && K > 0);
  TORCH_CHECK(span(M, sam, K, sak) <= A.numel() && span(K, sbk, N, sbn) <= B.numel() &&
              span(M, scm, N, scn) <= C.numel(), "simt_gemm: operand too small for the given strides");
  if (bias) {
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() == N);
  }
  c10::DeviceGuard g(A.device());
  CHECK_HIP_OK(pda::simt_gemm(A.data_ptr(), is_bf16(A), sam, sak, B.data_ptr(), is_bf16(B), sbk, sbn, C.data_ptr(),
                              is_bf16(C), scm, scn, M, N, K, bias ? bias->data_ptr<float>() : nullptr, relu,
                              (float)beta, stream_of(A)));
}

// ------------------------------------------------------------------ LayerNorm / RMSNorm
std::vector<Tensor> rownorm_fwd(Tensor x, Tensor gamma, c10::optional<Tensor> beta, double eps, bool rms) {
  check_f32_or_bf16(x, "x");
  check_f32_or_bf16(gamma, "gamma");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "norm width must be a multiple of 8 and <= 8192");
  TORCH_CHECK(gamma.numel() == D);
  if (!rms) {
    TORCH_CHECK(beta.has_value() && beta->numel() == D && beta->scalar_type() == gamma.scalar_type());
    check_gpu(*beta, "beta");
  }
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({rms ? 1 : rows}, fo), rstd = at::empty({rows}, fo);
  CHECK_HIP_OK(pda::rownorm_fwd(x.data_ptr(), is_bf16(x), gamma.data_ptr(), rms ? nullptr : beta->data_ptr(),
                                is_bf16(gamma), y.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, D,
                                (float)eps, rms, stream_of(x)));
  return {y, mean, rstd};
}

// inference: (h = x + r, norm(h)) in one pass; all bf16, contiguous
std::vector<Tensor> add_rownorm_fwd(Tensor x, Tensor r, Tensor gamma, c10::optional<Tensor> beta, double eps, bool rms) {
  check_bf16(x, "x");
  check_bf16(r, "r");
  check_bf16(gamma, "gamma");
  TORCH_CHECK(x.is_contiguous() && r.is_contiguous() && x.sizes() == r.sizes(), "add_rownorm: x, r contiguous, same shape");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 8192 && gamma.numel() == D, "norm width must be a multiple of 8 and <= 8192");
  if (!rms) {
    TORCH_CHECK(beta.has_value() && beta->numel() == D);
    check_bf16(*beta, "beta");
  }
  c10::DeviceGuard g(x.device());
  Tensor h = at::empty_like(x), y = at::empty_like(x);
  CHECK_HIP_OK(pda::add_rownorm_fwd(bp(x), bp(r), bp(gamma), rms ? nullptr : bp(*beta), bpm(h), bpm(y), rows, D,
                                    (float)eps, rms, stream_of(x)));
  return {h, y};
}

// training: (h = x + r, norm(h), mean(h), rstd(h)); all bf16, contiguous
std::vector<Tensor> add_rownorm_fwd_train(Tensor x, Tensor r, Tensor gamma, c10::optional<Tensor> beta, double eps,
                                          bool rms) {
  check_bf16(x, "x");
  check_bf16(r, "r");
  check_bf16(gamma, "gamma");
  TORCH_CHECK(x.is_contiguous() && r.is_contiguous() && x.sizes() == r.sizes(), "add_rownorm: x, r contiguous, same shape");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 8192 && gamma.numel() == D, "norm width must be a multiple of 8 and <= 8192");
  if (!rms) {
    TORCH_CHECK(beta.has_value() && beta->numel() == D);
    check_bf16(*beta, "beta");
  }
  c10::DeviceGuard g(x.device());
  Tensor h = at::empty_like(x), y = at::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({rms ? 1 : rows}, fo), rstd = at::empty({rows}, fo);
  CHECK_HIP_OK(pda::add_rownorm_fwd(bp(x), bp(r), bp(gamma), rms ? nullptr : bp(*beta), bpm(h), bpm(y), rows, D,
                                    (float)eps, rms, stream_of(x), mean.data_ptr<float>(), rstd.data_ptr<float>()));
  return {h, y, mean, rstd};
}

// dgamma / dbeta in the parameter dtype, written into ``dgamma_out`` / ``dbeta_out`` when given (the
// parameters' gradient slots: no cast kernel, no copy)
std::vector<Tensor> rownorm_bwd(Tensor dy, Tensor x, Tensor gamma, Tensor mean, Tensor rstd, bool rms,
                                c10::optional<Tensor> addend, c10::optional<Tensor> dgamma_out,
                                c10::optional<Tensor> dbeta_out) {
  check_f32_or_bf16(dy, "dy");
  check_f32_or_bf16(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type());
  if (addend.has_value()) {
    TORCH_CHECK(addend->sizes() == x.sizes() && addend->scalar_type() == x.scalar_type() && addend->is_contiguous(),
                "rownorm_bwd: addend must match x");
    check_gpu(*addend, "addend");
  }
  const int64_t D = x.size(-1), rows = x.numel() / D;
  c10::DeviceGuard g(x.device());
  Tensor dx = at::empty_like(x);
  auto po = x.options().dtype(gamma.scalar_type());
  auto take = [&](const c10::optional<Tensor>& t, const char* name) {
    if (!t.has_value()) return at::empty({D}, po);
    TORCH_CHECK(t->scalar_type() == gamma.scalar_type() && t->numel() == D && t->is_contiguous(), name,
                ": must be a contiguous [D] tensor of the parameter dtype");
    return *t;
  };
  Tensor dgamma = take(dgamma_out, "dgamma_out");
  Tensor dbeta = rms ? at::empty({0}, po) : take(dbeta_out, "dbeta_out");
  Tensor ws = at::empty({pda::colreduce_ws_floats(rows, D, rms ? 1 : 2)}, x.options().dtype(at::kFloat));
  CHECK_HIP_OK(pda::rownorm_bwd(dy.data_ptr(), x.data_ptr(), is_bf16(x), gamma.data_ptr(), is_bf16(gamma),
                                rms ? nullptr : mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(),
                                dgamma.data_ptr(), rms ? nullptr : dbeta.data_ptr(), is_bf16(gamma), rows, D, rms,
                                ws.data_ptr<float>(), stream_of(x), addend.has_value() ? addend->data_ptr() : nullptr));
  return {dx, dgamma, dbeta};
}

// ------------------------------------------------------------------ flash attention
void attn_check(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, name, " must be [B, T, H, D] with contiguous D");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0, name,
              " strides must be multiples of 8 elements");
  check_aligned16(t, name);
}

void rope_tables(pda::AttnParams& p, const c10::optional<Tensor>& cs, const c10::optional<Tensor>& sn, int T, int D) {
  p.rope_cos = p.rope_sin = nullptr;
  if (!cs.has_value()) return;
  check_f32(*cs, "rope cos");
  check_f32(*sn, "rope sin");
  TORCH_CHECK(cs->numel() >= (int64_t)T * D / 2 && sn->numel() == cs->numel(), "rope tables must be [>=T, D/2]");
  p.rope_cos = cs->data_ptr<float>();
  p.rope_sin = sn->data_ptr<float>();
}

std::vector<Tensor> attn_fwd(Tensor q, Tensor k, Tensor v, double scale, bool causal, c10::optional<Tensor> rope_cos,
                             c10::optional<Tensor> rope_sin) {
  attn_check(q, "q");
  attn_check(k, "k");
  attn_check(v, "v");
  const int B = q.size(0), T = q.size(1), Hq = q.size(2), D = q.size(3), Hkv = k.size(2);
  TORCH_CHECK(D == 64 || D == 128, "head dim must be 64 or 128");
  TORCH_CHECK(k.size(0) == B && k.size(1) == T && k.size(3) == D && v.sizes() == k.sizes());
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "query heads must be a multiple of kv heads");
  c10::DeviceGuard g(q.device());
  Tensor o = at::empty({B, T, Hq, D}, q.options());
  Tensor lse = at::empty({B, Hq, T}, q.options().dtype(at::kFloat));
  pda::AttnParams p{};
  p.q = bp(q); p.k = bp(k); p.v = bp(v); p.o = bpm(o); p.lse = lse.data_ptr<float>();
  p.q_sb = q.stride(0); p.q_st = q.stride(1); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_st = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_st = v.stride(1); p.v_sh = v.stride(2);
  p.o_sb = o.stride(0); p.o_st = o.stride(1); p.o_sh = o.stride(2);
  p.B = B; p.T = T; p.Hq = Hq; p.Hkv = Hkv; p.D = D; p.causal = causal ? 1 : 0; p.scale = (float)scale;
  rope_tables(p, rope_cos, rope_sin, T, D);
  CHECK_HIP_OK(pda::attention_fwd(p, stream_of(q)));
  return {o, lse};
}

// Writes dq/dk/dv into the given tensors (any [B,T,H,D] strides, e.g. slices of a fused dQKV buffer).
void attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor dq, Tensor dk, Tensor dv,
              double scale, bool causal, c10::optional<Tensor> rope_cos, c10::optional<Tensor> rope_sin) {
  for (auto* t : {&dout, &q, &k, &v, &o, &dq, &dk, &dv}) attn_check(*t, "attention tensor");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && dq.sizes() == q.sizes());
  TORCH_CHECK(dk.sizes() == k.sizes() && dv.sizes() == v.sizes());
  check_f32(lse, "lse");
  const int B = q.size(0), T = q.size(1), Hq = q.size(2), D = q.size(3), Hkv = k.size(2);
  TORCH_CHECK(D == 64 || D == 128);
  c10::DeviceGuard g(q.device());
  Tensor delta = at::empty({B, Hq, T}, q.options().dtype(at::kFloat));
  pda::AttnParams p{};
  p.q = bp(q); p.k = bp(k); p.v = bp(v); p.o = bpm(o); p.lse = lse.data_ptr<float>();
  p.q_sb = q.stride(0); p.q_st = q.stride(1); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_st = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_st = v.stride(1); p.v_sh = v.stride(2);
  p.o_sb = o.stride(0); p.o_st = o.stride(1); p.o_sh = o.stride(2);
  p.B = B; p.T = T; p.Hq = Hq; p.Hkv = Hkv; p.D = D; p.causal = causal ? 1 : 0; p.scale = (float)scale;
  p.dout = bp(dout); p.do_sb = dout.stride(0); p.do_st = dout.stride(1); p.do_sh = dout.stride(2);
  p.delta = delta.data_ptr<float>();
  p.dq = bpm(dq); p.dq_sb = dq.stride(0); p.dq_st = dq.stride(1); p.dq_sh = dq.stride(2);
  p.dk = bpm(dk); p.dk_sb = dk.stride(0); p.dk_st = dk.stride(1); p.dk_sh = dk.stride(2);
  p.dv = bpm(dv); p.dv_sb = dv.stride(0); p.dv_st = dv.stride(1); p.dv_sh = dv.stride(2);
  rope_tables(p, rope_cos, rope_sin, T, D);
  const int64_t wsn = pda::attention_bwd_ws_floats(B, T, Hq, Hkv, D, rope_cos.has_value());
  const int64_t dqn = pda::attention_bwd_fused(D, rope_cos.has_value()) ? (int64_t)B * Hq * T * D : 0;
  Tensor ws;
  if (wsn + dqn > 0) {
    ws = at::empty({wsn + dqn}, q.options().dtype(at::kFloat));
    if (wsn > 0) p.dkv_part = ws.data_ptr<float>();
    if (dqn > 0) p.dq_acc = ws.data_ptr<float>() + wsn;
  }
  CHECK_HIP_OK(pda::attention_bwd(p, stream_of(q)));
}

// ------------------------------------------------------------------ decode attention (serving)
// q [B, 1, Hq, D] (any B/H strides), k/v caches [B, Tmax, Hkv, D] (any strides, contiguous D); attends the
// first L cache rows; returns o [B, 1, Hq, D]
Tensor decode_attn(Tensor q, Tensor k, Tensor v, int64_t L, double scale, int64_t splits,
                   c10::optional<Tensor> pos_dev) {
  attn_check(q, "q");
  attn_check(k, "k cache");
  attn_check(v, "v cache");
  const int B = q.size(0), Hq = q.size(2), D = q.size(3), Hkv = k.size(2);
  TORCH_CHECK(q.size(1) == 1, "decode_attn: one query token per sequence");
  TORCH_CHECK(D == 64 || D == 128, "head dim must be 64 or 128");
  TORCH_CHECK(k.size(0) == B && k.size(3) == D && v.sizes() == k.sizes(), "decode_attn: cache shape mismatch");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0 && (Hq / Hkv == 1 || Hq / Hkv == 2 || Hq / Hkv == 4 || Hq / Hkv == 8),
              "decode_attn: query heads per kv head must be 1, 2, 4 or 8");
  TORCH_CHECK(L >= 1 && L <= k.size(1), "decode_attn: L must be in [1, cache length]");
  if (pos_dev.has_value()) {
    check_gpu(*pos_dev, "pos");
    TORCH_CHECK(pos_dev->scalar_type() == at::kInt && pos_dev->numel() == 1, "decode_attn: pos must be one int32");
  }
  c10::DeviceGuard g(q.device());
  Tensor o = at::empty({B, 1, Hq, D}, q.options());
  pda::DecodeAttnParams p{};
  p.q = bp(q); p.k = bp(k); p.v = bp(v); p.o = bpm(o);
  p.q_sb = q.stride(0); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_st = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_st = v.stride(1); p.v_sh = v.stride(2);
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.D = D; p.L = (int)L;
  p.splits = splits > 0 ? (int)splits : pda::decode_attn_splits(B, Hkv, (int)L, D);
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  // device position (graph replay): L is the cache capacity here; the kernel reads pos + 1 at run time
  p.L_dev = pos_dev.has_value() ? pos_dev->data_ptr<int>() : nullptr;
  Tensor ws;
  if (p.splits > 1) {
    ws = at::empty({(int64_t)B * Hq * p.splits * (D + 2)}, q.options().dtype(at::kFloat));
    p.ws_acc = ws.data_ptr<float>();
    p.ws_ml = p.ws_acc + (int64_t)B * Hq * p.splits * D;
  }
  CHECK_HIP_OK(pda::decode_attention(p, stream_of(q)));
  return o;
}

// new decode token: q rotated -> returned [B, 1, Hq, D]; k rotated into k_cache[:, pos]; v into v_cache[:, pos];
// pos is a device int32 (graph-replayable); rope tables optional (GPT-2 has none)
Tensor kv_append(Tensor qkv, Tensor k_cache, Tensor v_cache, Tensor pos, int64_t n_heads, int64_t n_kv_heads,
                 c10::optional<Tensor> cs, c10::optional<Tensor> sn) {
  attn_check(qkv, "qkv");
  attn_check(k_cache, "k cache");
  attn_check(v_cache, "v cache");
  check_gpu(pos, "pos");
  TORCH_CHECK(pos.scalar_type() == at::kInt && pos.numel() == 1, "kv_append: pos must be one int32");
  const int B = qkv.size(0), D = qkv.size(3);
  TORCH_CHECK(qkv.size(1) == 1 && qkv.size(2) == n_heads + 2 * n_kv_heads, "kv_append: qkv must be [B, 1, Hq+2Hkv, D]");
  TORCH_CHECK(k_cache.size(0) == B && k_cache.size(2) == n_kv_heads && k_cache.size(3) == D &&
              v_cache.sizes() == k_cache.sizes(), "kv_append: cache shape mismatch");
  TORCH_CHECK(D % 2 == 0 && D <= 128, "kv_append: head dim must be even and <= 128");
  c10::DeviceGuard g(qkv.device());
  Tensor q = at::empty({B, 1, n_heads, D}, qkv.options());
  pda::KvAppendParams p{};
  p.qkv = bp(qkv); p.q_out = bpm(q); p.k_cache = bpm(k_cache); p.v_cache = bpm(v_cache);
  p.cos = p.sin = nullptr;
  if (cs.has_value()) {
    check_f32(*cs, "cos");
    check_f32(*sn, "sin");
    TORCH_CHECK(cs->numel() >= k_cache.size(1) * D / 2, "kv_append: rope tables must cover the cache length");
    p.cos = cs->data_ptr<float>();
    p.sin = sn->data_ptr<float>();
  }
  p.pos = pos.data_ptr<int>();
  p.x_sb = qkv.stride(0); p.x_sh = qkv.stride(2);
  p.k_sb = k_cache.stride(0); p.k_st = k_cache.stride(1); p.k_sh = k_cache.stride(2);
  p.v_sb = v_cache.stride(0); p.v_st = v_cache.stride(1); p.v_sh = v_cache.stride(2);
  p.B = B; p.Hq = (int)n_heads; p.Hkv = (int)n_kv_heads; p.D = D;
  CHECK_HIP_OK(pda::kv_append_rope(p, stream_of(qkv)));
  return q;
}

// weight-only int8 GEMM (decode): x [M, K] bf16 (M <= 64, rows contiguous), w [N, K] int8, scale [N] fp32;
// ws [>= 8 * 64 * N] fp32 (partial slabs) and tickets [>= N / 64] int32 (zero-initialised, left zeroed) are
// caller-owned
Tensor w8_gemm(Tensor x, Tensor w, Tensor scale, Tensor ws, Tensor tickets, int64_t splits) {
  check_bf16(x, "x");
  check_gpu(w, "w");
  check_f32(scale, "scale");
  TORCH_CHECK(w.scalar_type() == at::kChar && w.dim() == 2 && w.is_contiguous(), "w8_gemm: w must be int8 [N, K]");
  const int64_t K = w.size(1), N = w.size(0);
  TORCH_CHECK(x.size(-1) == K && x.stride(-1) == 1, "w8_gemm: x must be [..., K] with contiguous rows");
  Tensor x2 = x.reshape({-1, K});
  const int64_t M = x2.size(0);
  TORCH_CHECK(M >= 1 && M <= 64, "w8_gemm: at most 64 rows (decode steps)");
  TORCH_CHECK(N % pda::w8_gemm_rows() == 0 && K % 256 == 0 && scale.numel() == N, "w8_gemm: N % 16 == 0, K % 256 == 0");
  TORCH_CHECK(x2.stride(0) % 8 == 0, "w8_gemm: x row stride must be a multiple of 8");
  check_aligned16(x2, "x");
  const int S = splits > 0 ? (int)splits : pda::w8_gemm_splits((int)N, (int)K);
  TORCH_CHECK(S <= 8 && K % (256 * S) == 0, "w8_gemm: K must split into 4*S slices of 64 (S <= 8)");
  if (S > 1) {
    check_f32(ws, "ws");
    TORCH_CHECK(ws.numel() >= (int64_t)S * M * N && tickets.scalar_type() == at::kInt &&
                tickets.numel() >= N / pda::w8_gemm_rows(), "w8_gemm: workspace too small");
  }
  c10::DeviceGuard g(x.device());
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  Tensor y = at::empty(sizes, x.options());
  pda::W8GemmParams p{};
  p.x = bp(x2); p.w = reinterpret_cast<const int8_t*>(w.data_ptr()); p.scale = scale.data_ptr<float>(); p.y = bpm(y);
  p.ws = S > 1 ? ws.data_ptr<float>() : nullptr;
  p.tickets = S > 1 ? tickets.data_ptr<int>() : nullptr;
  p.ldx = x2.stride(0); p.ldy = N;
  p.M = (int)M; p.N = (int)N; p.K = (int)K; p.S = S;
  CHECK_HIP_OK(pda::w8_gemm(p, stream_of(x)));
  return y;
}

// ------------------------------------------------------------------ embedding / rope
Tensor embedding_fwd(Tensor idx, Tensor table) {
  check_gpu(idx, "idx");
  check_bf16(table, "table");
  TORCH_CHECK(idx.scalar_type() == at::kLong && table.dim() == 2 && table.size(1) % 8 == 0);
  c10::DeviceGuard g(table.device());
  auto sizes = idx.sizes().vec();
  sizes.push_back(table.size(1));
  Tensor out = at::empty(sizes, table.options());
  CHECK_HIP_OK(pda::embedding_fwd(idx.data_ptr<int64_t>(), bp(table), bpm(out), idx.numel(), table.size(1),
                                  stream_of(table)));
  return out;
}

// returns the table gradient in `out_dtype` (fp32 accumulate); writes into `out` when given
Tensor embedding_bwd(Tensor idx, Tensor dy, int64_t V, c10::optional<Tensor> out) {
  check_gpu(idx, "idx");
  check_bf16(dy, "dy");
  const int64_t D = dy.size(-1);
  c10::DeviceGuard g(dy.device());
  Tensor acc = at::zeros({V, D}, dy.options().dtype(at::kFloat));
  const char* det = getenv("PDA_DETERMINISTIC");
  if (det != nullptr && det[0] == '1') {  // fixed-order sums: stable sort by token id, one lane per run
    auto sorted = at::sort(idx.reshape({-1}), /*stable=*/true, /*dim=*/0, /*descending=*/false);
    Tensor sidx = std::get<0>(sorted).contiguous(), order = std::get<1>(sorted).contiguous();
    CHECK_HIP_OK(pda::embedding_bwd_sorted(sidx.data_ptr<int64_t>(), order.data_ptr<int64_t>(), bp(dy),
                                           acc.data_ptr<float>(), idx.numel(), D, stream_of(dy)));
  } else {
    CHECK_HIP_OK(pda::embedding_bwd(idx.data_ptr<int64_t>(), bp(dy), acc.data_ptr<float>(), idx.numel(), D,
                                    stream_of(dy)));
  }
  Tensor res = out.has_value() ? *out : at::empty({V, D}, dy.options());
  TORCH_CHECK(res.numel() == V * D);
  CHECK_HIP_OK(pda::cast_scale(acc.data_ptr(), false, res.data_ptr(), is_bf16(res), V * D, 1.f, nullptr,
                               stream_of(dy)));
  return res;
}

// rotate-half RoPE of x [B, T, H, D] (any B/T/H strides, contiguous D); writes a new contiguous tensor
// or `out` (same shape, its own strides, e.g. a head slice of a fused QKV gradient)
Tensor rope(Tensor x, Tensor cs, Tensor sn, bool inverse, c10::optional<Tensor> out) {
  attn_check(x, "x");
  check_f32(cs, "cos");
  check_f32(sn, "sin");
  const int B = x.size(0), T = x.size(1), H = x.size(2), D = x.size(3);
  TORCH_CHECK(D % 16 == 0 && cs.numel() >= (int64_t)T * D / 2);
  c10::DeviceGuard g(x.device());
  Tensor y = out.has_value() ? *out : at::empty({B, T, H, D}, x.options());
  attn_check(y, "out");
  TORCH_CHECK(y.sizes() == x.sizes(), "rope: out shape mismatch");
  CHECK_HIP_OK(pda::rope_apply(bp(x), bpm(y), cs.data_ptr<float>(), sn.data_ptr<float>(), B, T, H, D, x.stride(0),
                               x.stride(1), x.stride(2), y.stride(0), y.stride(1), y.stride(2), inverse,
                               stream_of(x)));
  return y;
}


// ------------------------------------------------------------------ xGMI one-shot all-reduce
class XgmiComm {
 public:
  struct Reg {  // a zero-copy registration: every rank's tensor, mapped into this process
    void* base[pda::kXgmiMaxRanks] = {};
    int64_t bytes = 0;
  };
  XgmiComm(int rank, int world, int64_t capacity_bytes, int device, double timeout_s)
      : rank_(rank), world_(world), cap_(capacity_bytes), dev_(device) {
    TORCH_CHECK(world >= 1 && world <= pda::kXgmiMaxRanks && rank >= 0 && rank < world, "xgmi: bad rank/world");
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device));
    CHECK_HIP_OK(pda::xgmi_alloc(&data_, (size_t)cap_));
    CHECK_HIP_OK(pda::xgmi_alloc(&flags_, flag_bytes()));
    CHECK_HIP_OK(pda::xgmi_alloc_error_word(&err_host_, &err_));
    int rate_khz = 0;
    CHECK_HIP_OK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device));
    timeout_ticks_ = (long long)(timeout_s * (double)rate_khz * 1000.0);
    for (int r = 0; r < pda::kXgmiMaxRanks; ++r) {
      peer_data_[r] = nullptr;
      peer_flags_[r] = nullptr;
    }
    peer_data_[rank] = data_;
    peer_flags_[rank] = reinterpret_cast<uint32_t*>(flags_);
  }
  ~XgmiComm() {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, dev_));
    for (auto& kv : mapped_) (void)pda::xgmi_close_handle(kv.second);
    for (int r = 0; r < world_; ++r)
      if (r != rank_) {
        if (peer_data_[r]) (void)pda::xgmi_close_handle(peer_data_[r]);
        if (peer_flags_[r]) (void)pda::xgmi_close_handle(peer_flags_[r]);
      }
    (void)pda::xgmi_free(data_);
    (void)pda::xgmi_free(flags_);
    (void)pda::xgmi_free_error_word(err_host_);
  }
  static size_t flag_bytes() { return (size_t)pda::kXgmiPhases * pda::kXgmiMaxBlocks * pda::kXgmiMaxRanks * sizeof(uint32_t); }
  py::bytes handles() {
    std::string h(2 * HIP_IPC_HANDLE_SIZE, '\0');
    CHECK_HIP_OK(pda::xgmi_get_handle(data_, &h[0]));
    CHECK_HIP_OK(pda::xgmi_get_handle(flags_, &h[HIP_IPC_HANDLE_SIZE]));
    return py::bytes(h);
  }
  void open(const std::vector<std::string>& all) {
    TORCH_CHECK((int)all.size() == world_, "xgmi: need one handle blob per rank");
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, dev_));
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(all[r].size() == 2 * HIP_IPC_HANDLE_SIZE, "xgmi: bad handle blob");
      void* d = nullptr;
      void* f = nullptr;
      CHECK_HIP_OK(pda::xgmi_open_handle(all[r].data(), &d));
      CHECK_HIP_OK(pda::xgmi_open_handle(all[r].data() + HIP_IPC_HANDLE_SIZE, &f));
      peer_data_[r] = d;
      peer_flags_[r] = reinterpret_cast<uint32_t*>(f);
    }
    opened_ = true;
  }
  // in-place all-reduce of a contiguous fp32 / bf16 tensor on this communicator's device
  void allreduce(Tensor t, bool average, int algo) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi: open() the peer handles first");
    TORCH_CHECK(algo == pda::kXgmiOneShot || algo == pda::kXgmiTwoShot || algo == pda::kXgmiRing,
                "xgmi: algo 0 (one-shot), 1 (two-shot) or 2 (ring)");
    check_gpu(t, "t");
    TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "xgmi: fp32 / bf16 only");
    const int64_t n = t.numel(), bytes = n * t.element_size();
    TORCH_CHECK(n % 8 == 0 && bytes <= cap_, "xgmi: numel must be a multiple of 8 and fit the exchange buffer");
    c10::DeviceGuard g(t.device());
    auto st = stream_of(t);
    CHECK_HIP_OK(hipMemcpyAsync(data_, t.data_ptr(), (size_t)bytes, hipMemcpyDeviceToDevice, st));
    launch(t.data_ptr(), n, average ? 1.f / (float)world_ : 1.f, algo, t.scalar_type() == at::kBFloat16, st);
  }
  void launch_on(const Reg& reg, int64_t byte_off, void* out, int64_t n, float scale, int algo, bool bf16,
                 hipStream_t st) {
    pda::XgmiArgs a{};
    for (int r = 0; r < pda::kXgmiMaxRanks; ++r) {
      a.data[r] = reg.base[r] ? (char*)reg.base[r] + byte_off : nullptr;
      a.flags[r] = peer_flags_[r];
    }
    a.out = out;
    a.n = n;
    a.rank = rank_;
    a.world = world_;
    a.scale = scale;
    a.epoch = ++epoch_;
    a.timeout_ticks = timeout_ticks_;
    a.err = err_;
    a.algo = algo;
    CHECK_HIP_OK(pda::xgmi_allreduce(a, bf16, st));
  }
  void launch(void* out, int64_t n, float scale, int algo, bool bf16, hipStream_t st) {
    pda::XgmiArgs a{};
    for (int r = 0; r < pda::kXgmiMaxRanks; ++r) {
      a.data[r] = peer_data_[r];
      a.flags[r] = peer_flags_[r];
    }
    a.out = out;
    a.n = n;
    a.rank = rank_;
    a.world = world_;
    a.scale = scale;
    a.epoch = ++epoch_;
    a.timeout_ticks = timeout_ticks_;
    a.err = err_;
    a.algo = algo;
    CHECK_HIP_OK(pda::xgmi_allreduce(a, bf16, st));
  }
  // out[world * n] = every rank's `in` [n] in rank order (all-gather over the IPC mesh)
  void allgather(Tensor in, Tensor out) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi: open() the peer handles first");
    check_gpu(in, "in");
    check_gpu(out, "out");
    TORCH_CHECK(in.scalar_type() == out.scalar_type() &&
                    (in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16),
                "xgmi: fp32 / bf16, same dtype");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "xgmi: contiguous tensors");
    const int64_t n = in.numel(), bytes = n * in.element_size();
    TORCH_CHECK(n % 8 == 0 && bytes <= cap_ && out.numel() == n * world_,
                "xgmi all-gather: shard numel % 8 == 0, shard fits the exchange buffer, out = world x shard");
    c10::DeviceGuard g(in.device());
    auto st = stream_of(in);
    CHECK_HIP_OK(hipMemcpyAsync(data_, in.data_ptr(), (size_t)bytes, hipMemcpyDeviceToDevice, st));
    launch(out.data_ptr(), n, 1.f, pda::kXgmiAllGather, in.scalar_type() == at::kBFloat16, st);
  }
  // out[n / world] = scale * sum over ranks of chunk `rank` of `in` [n]
  void reduce_scatter(Tensor in, Tensor out, bool average) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi: open() the peer handles first");
    check_gpu(in, "in");
    check_gpu(out, "out");
    TORCH_CHECK(in.scalar_type() == out.scalar_type() &&
                    (in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16),
                "xgmi: fp32 / bf16, same dtype");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "xgmi: contiguous tensors");
    const int64_t n = in.numel(), bytes = n * in.element_size();
    TORCH_CHECK(n % (8 * world_) == 0 && bytes <= cap_ && out.numel() * world_ == n,
                "xgmi reduce-scatter: numel % (8 world) == 0, input fits the exchange buffer, out = shard");
    c10::DeviceGuard g(in.device());
    auto st = stream_of(in);
    CHECK_HIP_OK(hipMemcpyAsync(data_, in.data_ptr(), (size_t)bytes, hipMemcpyDeviceToDevice, st));
    launch(out.data_ptr(), n, average ? 1.f / (float)world_ : 1.f, pda::kXgmiReduceScatter,
           in.scalar_type() == at::kBFloat16, st);
  }
  // ---- zero-copy (registered) buffers: the collective reads the peers' tensors in place
  // instead of a copy into the exchange buffer.  reg_handle(t): this rank's IPC handle of t's allocation
  // (hipMemGetAddressRange gives the base of the caching allocator's segment) + t's byte offset in it;
  // reg_open(blobs): maps every peer's allocation once (mappings cached per handle, shared by later
  // registrations in the same segment) and returns a registration id.  A registered tensor must stay
  // allocated, unmoved, for as long as collectives use it (DDP's flat gradient buffers, FSDP shards).
  py::bytes reg_handle(Tensor t) {
    check_gpu(t, "t");
    TORCH_CHECK(t.is_contiguous(), "xgmi: registered tensors are contiguous");
    c10::DeviceGuard g(t.device());
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    CHECK_HIP_OK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)t.data_ptr()));
    std::string h(HIP_IPC_HANDLE_SIZE + 16, '\0');
    CHECK_HIP_OK(pda::xgmi_get_handle(base, &h[0]));
    const int64_t off = (int64_t)((char*)t.data_ptr() - (char*)base);
    const int64_t bytes = t.numel() * t.element_size();
    std::memcpy(&h[HIP_IPC_HANDLE_SIZE], &off, 8);
    std::memcpy(&h[HIP_IPC_HANDLE_SIZE + 8], &bytes, 8);
    return py::bytes(h);
  }
  int reg_open(Tensor own, const std::vector<std::string>& all) {
    TORCH_CHECK((int)all.size() == world_, "xgmi: need one registration blob per rank");
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, dev_));
    Reg reg;
    reg.bytes = own.numel() * own.element_size();
    for (int r = 0; r < world_; ++r) {
      TORCH_CHECK(all[r].size() == HIP_IPC_HANDLE_SIZE + 16, "xgmi: bad registration blob");
      int64_t off = 0, bytes = 0;
      std::memcpy(&off, all[r].data() + HIP_IPC_HANDLE_SIZE, 8);
      std::memcpy(&bytes, all[r].data() + HIP_IPC_HANDLE_SIZE + 8, 8);
      TORCH_CHECK(bytes == reg.bytes, "xgmi: registered tensors differ in size across ranks");
      if (r == rank_) {
        reg.base[r] = own.data_ptr();
        continue;
      }
      const std::string key = std::to_string(r) + ":" + all[r].substr(0, HIP_IPC_HANDLE_SIZE);
      auto it = mapped_.find(key);
      void* b = nullptr;
      if (it != mapped_.end()) {
        b = it->second;
      } else {
        CHECK_HIP_OK(pda::xgmi_open_handle(all[r].data(), &b));
        mapped_[key] = b;
      }
      reg.base[r] = (char*)b + off;
    }
    regs_.push_back(reg);
    return (int)regs_.size() - 1;
  }
  // in-place all-reduce of t = registration `id`'s tensor [elem_off, elem_off + numel) (two-shot / ring:
  // both are in-place safe; one-shot reads every peer's whole input while writing its own, so it runs as
  // two-shot here)
  void allreduce_reg(int id, Tensor t, int64_t elem_off, bool average, int algo) {
    TORCH_CHECK(id >= 0 && id < (int)regs_.size(), "xgmi: unknown registration");
    TORCH_CHECK(algo == pda::kXgmiOneShot || algo == pda::kXgmiTwoShot || algo == pda::kXgmiRing, "xgmi: bad algo");
    check_gpu(t, "t");
    TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "xgmi: fp32 / bf16 only");
    const Reg& reg = regs_[id];
    const int64_t es = t.element_size(), n = t.numel();
    TORCH_CHECK(n % 8 == 0 && elem_off >= 0 && (elem_off + n) * es <= reg.bytes, "xgmi: slice outside the registration");
    TORCH_CHECK((char*)reg.base[rank_] + elem_off * es == (char*)t.data_ptr(), "xgmi: t is not that slice");
    c10::DeviceGuard g(t.device());
    launch_on(reg, elem_off * es, t.data_ptr(), n, average ? 1.f / (float)world_ : 1.f,
              algo == pda::kXgmiRing ? pda::kXgmiRing : pda::kXgmiTwoShot, t.scalar_type() == at::kBFloat16,
              stream_of(t));
  }
  // out[world * n] = every rank's registered shard (registration `id`), pulled in place
  void allgather_reg(int id, Tensor in, Tensor out) {
    TORCH_CHECK(id >= 0 && id < (int)regs_.size(), "xgmi: unknown registration");
    check_gpu(in, "in");
    check_gpu(out, "out");
    const Reg& reg = regs_[id];
    TORCH_CHECK(in.data_ptr() == reg.base[rank_] && in.numel() * in.element_size() == reg.bytes,
                "xgmi: all-gather input must be the registered tensor");
    TORCH_CHECK(in.scalar_type() == out.scalar_type() && out.is_contiguous() && out.numel() == in.numel() * world_ &&
                    in.numel() % 8 == 0 && (in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16),
                "xgmi all-gather: out = world x shard, same fp32 / bf16 dtype");
    c10::DeviceGuard g(in.device());
    launch_on(reg, 0, out.data_ptr(), in.numel(), 1.f, pda::kXgmiAllGather, in.scalar_type() == at::kBFloat16,
              stream_of(in));
  }
  // out[n / world] = scale * sum over ranks of chunk `rank` of every rank's registered input (in place)
  void reduce_scatter_reg(int id, Tensor in, Tensor out, bool average) {
    TORCH_CHECK(id >= 0 && id < (int)regs_.size(), "xgmi: unknown registration");
    check_gpu(in, "in");
    check_gpu(out, "out");
    const Reg& reg = regs_[id];
    TORCH_CHECK(in.data_ptr() == reg.base[rank_] && in.numel() * in.element_size() == reg.bytes,
                "xgmi: reduce-scatter input must be the registered tensor");
    const int64_t n = in.numel();
    TORCH_CHECK(in.scalar_type() == out.scalar_type() && out.is_contiguous() && n % (8 * world_) == 0 &&
                    out.numel() * world_ == n && (in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16),
                "xgmi reduce-scatter: numel % (8 world) == 0, out = shard, same fp32 / bf16 dtype");
    c10::DeviceGuard g(in.device());
    launch_on(reg, 0, out.data_ptr(), n, average ? 1.f / (float)world_ : 1.f, pda::kXgmiReduceScatter,
              in.scalar_type() == at::kBFloat16, stream_of(in));
  }
  int num_registrations() const { return (int)regs_.size(); }

  // non-blocking: the kernels store the error word into pinned host memory; 0 = no timeout so far
  int error() const { return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE); }
  void reset_error() { __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE); }
  int64_t capacity() const { return cap_; }

 private:
  int rank_, world_;
  int64_t cap_;
  int dev_;
  void* data_ = nullptr;
  void* flags_ = nullptr;
  int* err_ = nullptr;       // device alias of err_host_
  int* err_host_ = nullptr;  // pinned host-coherent error word
  void* peer_data_[pda::kXgmiMaxRanks];
  uint32_t* peer_flags_[pda::kXgmiMaxRanks];
  uint32_t epoch_ = 0;
  long long timeout_ticks_ = 0;
  bool opened_ = false;
  std::vector<Reg> regs_;
  std::map<std::string, void*> mapped_;  // "rank:handle" -> mapped peer allocation base (opened once)
};
// HIP stream at an explicit queue priority (PyTorch's stream pools only reach normal and high; the
// weight-gradient side stream wants LOW, so the dispatcher hands a freed CU to the critical-path
// queue first).  Returns the raw handle for torch.cuda.ExternalStream; lives for the process.
int64_t stream_create(int64_t device, int64_t priority) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  int least = 0, greatest = 0;
  CHECK_HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  int p = (int)priority;
  // HIP: numerically lower = higher priority; clamp into [greatest, least]
  if (p > least) p = least;
  if (p < greatest) p = greatest;
  hipStream_t s = nullptr;
  CHECK_HIP_OK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p));
  return reinterpret_cast<int64_t>(s);
}

// a stream whose hardware queue dispatches only to `ncu` CUs spread over the XCDs (invert: all the others)
int64_t stream_create_cumask(int64_t device, int64_t ncu, bool invert) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  int total = 0;
  CHECK_HIP_OK(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, (int)device));
  std::vector<uint32_t> mask = pda_rt::cu_mask_spread((int)ncu, total, invert);
  hipStream_t s = nullptr;
  CHECK_HIP_OK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  return reinterpret_cast<int64_t>(s);
}

std::vector<int64_t> stream_priority_range(int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  int least = 0, greatest = 0;
  CHECK_HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  return {least, greatest};
}
}  // namespace

// ------------------------------------------------------------------ fp32 path (fp32x3.hip)
// hi / lo bf16 split of an fp32 tensor, laid out along a GEMM's K:
//   stack=false: [rows, C] -> [rows, nseg * C] (segments side by side in each row; rows = numel / C_last)
//   stack=true:  [d0, ...] -> [nseg * d0, ...] (segments stacked along the leading dim)
// bit s of lo_mask selects the lo part for segment s
Tensor split_bf16(Tensor x, int64_t nseg, int64_t lo_mask, bool stack) {
  check_f32(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.dim() >= 1, "split_bf16: contiguous input");
  TORCH_CHECK(nseg >= 1 && nseg <= 4, "split_bf16: 1..4 segments");
  c10::DeviceGuard g(x.device());
  auto sizes = x.sizes().vec();
  Tensor out;
  if (stack) {
    sizes[0] *= nseg;
    out = at::empty(sizes, x.options().dtype(at::kBFloat16));
    TORCH_CHECK(x.numel() % 4 == 0, "split_bf16: numel % 4");
    CHECK_HIP_OK(pda::split_bf16(x.data_ptr<float>(), bpm(out), 1, x.numel(), (int)nseg, (int)lo_mask, x.numel(),
                                 x.numel() * nseg, stream_of(x)));
  } else {
    const int64_t C = sizes.back();
    TORCH_CHECK(C % 4 == 0, "split_bf16: last dim % 4");
    sizes.back() = C * nseg;
    out = at::empty(sizes, x.options().dtype(at::kBFloat16));
    CHECK_HIP_OK(pda::split_bf16(x.data_ptr<float>(), bpm(out), x.numel() / C, C, (int)nseg, (int)lo_mask, C,
                                 C * nseg, stream_of(x)));
  }
  return out;
}

const float* fptr(const c10::optional<Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value()) return nullptr;
  check_f32(*t, name);
  TORCH_CHECK(t->numel() == n && t->is_contiguous(), name, ": wrong size");
  return t->data_ptr<float>();
}

// BatchNorm training forward over the last dim of fp32 x: returns {y, save_mean, save_invstd}
std::vector<Tensor> bn_f32_fwd_train(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> gamma,
                                     c10::optional<Tensor> beta, c10::optional<Tensor> running_mean,
                                     c10::optional<Tensor> running_var, double momentum, double eps, bool relu,
                                     c10::optional<Tensor> num_batches) {
  check_f32(x, "x");
  TORCH_CHECK(x.is_contiguous());
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 4 == 0, "bn fp32: C % 4");
  if (res) {
    check_f32(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous());
  }
  c10::DeviceGuard g(x.device());
  auto fo = x.options();
  Tensor y = at::empty_like(x), mean = at::empty({C}, fo), invstd = at::empty({C}, fo), ss = at::empty({2 * C}, fo);
  Tensor part = at::empty({(int64_t)pda::bn_f32_partials(M, (int)C) * 2 * C}, fo);
  // shift = running mean (a close guess of the batch mean: shifted sums keep the variance accurate)
  const float* rm = fptr(running_mean, C, "running_mean");
  Tensor shift = rm ? running_mean->clone() : at::zeros({C}, fo);
  int64_t* nb = nullptr;
  if (num_batches) {
    check_gpu(*num_batches, "num_batches");
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1);
    nb = num_batches->data_ptr<int64_t>();
  }
  CHECK_HIP_OK(pda::bn_f32_fwd_train(x.data_ptr<float>(), res ? res->data_ptr<float>() : nullptr,
                                     fptr(gamma, C, "gamma"), fptr(beta, C, "beta"), (float*)rm,
                                     (float*)fptr(running_var, C, "running_var"), shift.data_ptr<float>(),
                                     (float)momentum, (float)eps, relu ? 1 : 0, y.data_ptr<float>(),
                                     mean.data_ptr<float>(), invstd.data_ptr<float>(), ss.data_ptr<float>(),
                                     part.data_ptr<float>(), nb, M, (int)C, stream_of(x)));
  return {y, mean, invstd};
}

// y = x * ss[:C] + ss[C:] (+ res) (relu)  (eval-mode BN with host-folded coefficients)
Tensor bn_f32_apply(Tensor x, c10::optional<Tensor> res, Tensor ss, bool relu) {
  check_f32(x, "x");
  TORCH_CHECK(x.is_contiguous());
  const int64_t C = x.size(-1), M = x.numel() / C;
  check_f32(ss, "ss");
  TORCH_CHECK(ss.numel() == 2 * C && C % 4 == 0);
  if (res) {
    check_f32(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous());
  }
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  CHECK_HIP_OK(pda::bn_f32_apply(x.data_ptr<float>(), res ? res->data_ptr<float>() : nullptr, ss.data_ptr<float>(),
                                 y.data_ptr<float>(), M, (int)C, relu ? 1 : 0, stream_of(x)));
  return y;
}

// BN backward: y (optional) = the forward output for the ReLU mask; returns {dx, g (masked dy, or
// undefined), dgamma, dbeta}
std::vector<Tensor> bn_f32_bwd(Tensor dy, Tensor x, c10::optional<Tensor> y, Tensor mean, Tensor invstd,
                               c10::optional<Tensor> gamma, bool want_g) {
  check_f32(dy, "dy");
  check_f32(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.is_contiguous() && x.is_contiguous());
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C % 4 == 0);
  if (y) {
    check_f32(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes() && y->is_contiguous());
  }
  c10::DeviceGuard g(x.device());
  auto fo = x.options();
  Tensor dx = at::empty_like(x), gout = want_g ? at::empty_like(x) : Tensor();
  Tensor dgamma = at::empty({C}, fo), dbeta = at::empty({C}, fo), co = at::empty({3 * C}, fo);
  Tensor part = at::empty({(int64_t)pda::bn_f32_partials(M, (int)C) * 2 * C}, fo);
  CHECK_HIP_OK(pda::bn_f32_bwd(dy.data_ptr<float>(), x.data_ptr<float>(), y ? y->data_ptr<float>() : nullptr,
                               fptr(mean, C, "mean"), fptr(invstd, C, "invstd"), fptr(gamma, C, "gamma"),
                               dx.data_ptr<float>(), want_g ? gout.data_ptr<float>() : nullptr,
                               dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), part.data_ptr<float>(),
                               co.data_ptr<float>(), M, (int)C, stream_of(x)));
  return {dx, gout, dgamma, dbeta};
}

std::vector<Tensor> maxpool_f32_fwd(Tensor x, int64_t k, int64_t s, int64_t pad) {
  check_f32(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "x must be [N,H,W,C]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 4 == 0 && k * k <= 255);
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, P, Q, C}, x.options());
  Tensor idx = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  CHECK_HIP_OK(pda::maxpool2d_f32_fwd(x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(), N, H, W, C, P,
                                      Q, k, s, pad, stream_of(x)));
  return {y, idx};
}

Tensor maxpool_f32_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad) {
  check_f32(dy, "dy");
  check_gpu(idx, "idx");
  TORCH_CHECK(idx.sizes() == dy.sizes() && dy.is_contiguous() && idx.scalar_type() == at::kByte);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  c10::DeviceGuard g(dy.device());
  Tensor dx = at::empty({N, H, W, C}, dy.options());
  CHECK_HIP_OK(pda::maxpool2d_f32_bwd(dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), dx.data_ptr<float>(), N, H, W, C,
                                      P, Q, k, s, pad, stream_of(dy)));
  return dx;
}

Tensor avgpool_f32_fwd(Tensor x) {
  check_f32(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous());
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  c10::DeviceGuard g(x.device());
  Tensor y = at::empty({N, C}, x.options());
  CHECK_HIP_OK(pda::avgpool_f32_fwd(x.data_ptr<float>(), y.data_ptr<float>(), N, HW, C, stream_of(x)));
  return y;
}

Tensor avgpool_f32_bwd(Tensor dy, int64_t H, int64_t W) {
  check_f32(dy, "dy");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous());
  const int N = dy.size(0), C = dy.size(1);
  c10::DeviceGuard g(dy.device());
  Tensor dx = at::empty({N, H, W, C}, dy.options());
  CHECK_HIP_OK(pda::avgpool_f32_bwd(dy.data_ptr<float>(), dx.data_ptr<float>(), N, H * W, C, stream_of(dy)));
  return dx;
}

PYBIND11_MODULE(_C, m) {
  m.def("stream_create", &stream_create, py::arg("device"), py::arg("priority"));
  m.def("stream_priority_range", &stream_priority_range, py::arg("device"));
  m.def("stream_create_cumask", &stream_create_cumask, py::arg("device"), py::arg("ncu"), py::arg("invert") = false);
  m.doc() = "pytorchdistributed_amd native layer: CDNA4 HIP kernels + C++ runtime";
  m.def("sgd_step", &sgd_step);
  m.def("adam_step", &adam_step);
  m.def("grad_norm", &grad_norm);
  m.def("cast_scale", &cast_scale);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("bn_fwd_train", &bn_fwd_train);
  m.def("bn_fwd_eval", &bn_fwd_eval);
  m.def("bn_bwd", &bn_bwd);
  m.def("bn_bwd_table", &bn_bwd_table);
  m.def("set_bn_bwd_fused_max_c", &set_bn_bwd_fused_max_c);
  m.def("set_dgrad_stream", [](int64_t m) { pda::set_dgrad_stream((int)m); });
  m.def("set_fwd_stream", [](int64_t m) { pda::set_fwd_stream((int)m); });
  m.def("set_attn_bwd_fused", [](int64_t m) { pda::attention_bwd_fused_mode() = (int)m; });
  m.def("attn_bwd_fused_mode", []() { return (int64_t)pda::attention_bwd_fused_mode(); });
  m.def("bn_bwd_fused_max_c", []() { return bn_bwd_fused_max_c(); });
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd);
  m.def("stem_pool_bn_bwd", &stem_pool_bn_bwd);
  m.def("stem_pool_bn_bwd_ok", &stem_pool_bn_bwd_ok);
  m.def("stem_s2d", &stem_s2d);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("fill_random", &fill_random);
  m.def("fill_randint", &fill_randint);
  m.def("gemm", &gemm);
  m.def("gemm_act", &gemm_act);
  m.def("gemm_wgrad_db", &gemm_wgrad_db);
  m.def("gemm_pp_lab", &gemm_pp_lab);
  m.def("set_gemm_paths", &pda::set_gemm_paths,
        "force a GEMM kernel path: wide=-1 env default, 0 off, 1 auto, 2 force", pybind11::arg("wide"));
  m.def("set_gemm_pp", &pda::set_gemm_pp,
        "pipelined 256x256 kernel for plain wide GEMMs: -1 env default (PDA_GEMM_PP), 0 off, 1 on",
        pybind11::arg("on"));
  m.def("set_splitk_fixup", &pda::set_splitk_fixup,
        "split-K weight gradients reduced by the GEMM's last split per tile: -1 env default (PDA_SPLITK_FIXUP, "
        "off), 0 separate reduce launch, 1 on",
        pybind11::arg("on"));
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"), py::arg("dil"),
        py::arg("bias") = py::none(), py::arg("relu") = false, py::arg("out_f32") = false);
  m.def("split_bf16", &split_bf16, py::arg("x"), py::arg("nseg"), py::arg("lo_mask"), py::arg("stack"));
  m.def("bn_f32_fwd_train", &bn_f32_fwd_train);
  m.def("bn_f32_apply", &bn_f32_apply);
  m.def("bn_f32_bwd", &bn_f32_bwd);
  m.def("maxpool_f32_fwd", &maxpool_f32_fwd);
  m.def("maxpool_f32_bwd", &maxpool_f32_bwd);
  m.def("avgpool_f32_fwd", &avgpool_f32_fwd);
  m.def("avgpool_f32_bwd", &avgpool_f32_bwd);
  m.def("conv_fwd_stats", &conv_fwd_stats);
  m.def("bn_fwd_train_sums", &bn_fwd_train_sums);
  m.def("bn_fwd_train_sums_dual", &bn_fwd_train_sums_dual);
  m.def("bn_dual_ok", &bn_dual_ok);
  m.def("bn_bwd_dual", &bn_bwd_dual, py::arg("dy"), py::arg("bits"), py::arg("x"), py::arg("mean"), py::arg("invstd"),
        py::arg("gamma"), py::arg("x2"), py::arg("mean2"), py::arg("invstd2"), py::arg("gamma2"),
        py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(), py::arg("dgamma2_out") = py::none(),
        py::arg("dbeta2_out") = py::none(), py::arg("table") = py::none(), py::arg("table2") = py::none());
  m.def("bn_bwd_dual_ok", &bn_bwd_dual_ok);
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("H"), py::arg("W"), py::arg("stride"),
        py::arg("pad"), py::arg("dil"), py::arg("addend") = py::none(), py::arg("addend_bits") = py::none(),
        py::arg("out_f32") = false, py::arg("bst_z") = py::none(), py::arg("bst_ss") = py::none(),
        py::arg("bst_bits") = py::none(), py::arg("bst_mean") = py::none(), py::arg("bst_table") = py::none(),
        py::arg("bst_z2") = py::none(), py::arg("bst_mean2") = py::none(), py::arg("bst_table2") = py::none());
  m.def("conv_wgrad", &conv_wgrad);
  m.def("act_fwd", &act_fwd);
  m.def("act_bwd", &act_bwd);
  m.def("relu_bwd", &relu_bwd);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("colsum", &colsum, py::arg("x"), py::arg("out") = py::none(), py::arg("out_bf16") = false);
  m.def("simt_gemm", &simt_gemm);
  m.def("rownorm_fwd", &rownorm_fwd);
  m.def("add_rownorm_fwd", &add_rownorm_fwd);
  m.def("rownorm_bwd", &rownorm_bwd, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("rms"), py::arg("addend") = py::none(), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none());
  m.def("add_rownorm_fwd_train", &add_rownorm_fwd_train);
  m.def("attn_fwd", &attn_fwd);
  m.def("decode_attn", &decode_attn, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("L"), py::arg("scale"),
        py::arg("splits") = 0, py::arg("pos_dev") = py::none());
  m.def("kv_append", &kv_append);
  m.def("w8_gemm", &w8_gemm, py::arg("x"), py::arg("w"), py::arg("scale"), py::arg("ws"), py::arg("tickets"),
        py::arg("splits") = 0);
  m.def("attn_bwd", &attn_bwd);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("rope", &rope);
  py::class_<XgmiComm>(m, "XgmiComm")
      .def(py::init<int, int, int64_t, int, double>(), py::arg("rank"), py::arg("world"), py::arg("capacity_bytes"),
           py::arg("device"), py::arg("timeout") = 10.0)
      .def("handles", &XgmiComm::handles)
      .def("open", &XgmiComm::open)
      .def("allreduce", &XgmiComm::allreduce, py::arg("t"), py::arg("average") = false, py::arg("algo") = 0)
      .def("allgather", &XgmiComm::allgather, py::arg("inp"), py::arg("out"))
      .def("reduce_scatter", &XgmiComm::reduce_scatter, py::arg("inp"), py::arg("out"), py::arg("average") = false)
      .def("error", &XgmiComm::error)
      .def("reg_handle", &XgmiComm::reg_handle)
      .def("reg_open", &XgmiComm::reg_open)
      .def("allreduce_reg", &XgmiComm::allreduce_reg, py::arg("id"), py::arg("t"), py::arg("elem_off"),
           py::arg("average") = false, py::arg("algo") = 1)
      .def("allgather_reg", &XgmiComm::allgather_reg)
      .def("reduce_scatter_reg", &XgmiComm::reduce_scatter_reg, py::arg("id"), py::arg("inp"), py::arg("out"),
           py::arg("average") = false)
      .def_property_readonly("num_registrations", &XgmiComm::num_registrations)
      .def("reset_error", &XgmiComm::reset_error)
      .def_property_readonly("capacity", &XgmiComm::capacity);
  pda_rt::bind_runtime(m);
  pda_comm::bind_comm(m);
}
