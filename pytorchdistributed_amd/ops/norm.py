"""Normalisation ops.

* :func:`batch_norm` — training/eval BatchNorm over channels-last activations with fused residual add
  and ReLU (reference ResNet-50 BN ×53, `03_model_parallel.ipynb` raw line 314).
* :func:`layer_norm`, :func:`rms_norm` — row norms for GPT-2 / Llama-3 (K19, K20).
* :func:`add_norm_train` — the residual add fused into the following norm, with autograd (training
  counterpart of the serving :func:`add_norm`): one forward pass writes ``h = x + r`` and ``norm(h)``,
  and the backward writes ``dh_total = norm_bwd(dn) + dh`` once (no separate add kernels in either
  direction for the residual stream).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._native import C
from ..parallel.flat import grad_target
from .grad_join import BnBwdStats, MaskedGrad


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, training, momentum, eps, relu, join,
                table=None, shift=None, num_batches=None, bwd_table=None):
        x = x.contiguous()
        if residual is not None:
            residual = residual.contiguous()
        ss = bits = None
        # BN+residual+ReLU: the forward also writes the ReLU mask as bits (1/16 of y), read by both
        # backward passes instead of the 16-bit output
        want_bits = relu and residual is not None
        if training and table is not None:  # statistics accumulated by the producing conv's epilogue
            y, mean, invstd, ss, bits = C().bn_fwd_train_sums(x, table, shift, residual, gamma, beta, running_mean,
                                                              running_var, momentum, eps, relu, want_bits, num_batches)
        elif training:
            y, mean, invstd, ss, bits = C().bn_fwd_train(x, residual, gamma, beta, running_mean, running_var,
                                                         momentum, eps, relu, want_bits, num_batches)
        else:
            y = C().bn_fwd_eval(x, residual, gamma, beta, running_mean, running_var, eps, relu)
            mean = running_mean
            invstd = torch.rsqrt(running_var + eps)
        # BN+ReLU without a residual: the backward recomputes the ReLU mask from x and the saved
        # per-channel scale/shift, so y is neither kept alive nor re-read (one fewer HBM pass)
        ctx.save_for_backward(x, bits if want_bits else None, ss if (relu and not want_bits) else None, mean, invstd,
                              gamma)
        ctx.cfg = (relu, residual is not None, training)
        ctx.beta = beta
        ctx.join = join
        # backward reduction handed to the consuming conv's dgrad epilogue (ops/grad_join.py:BnBwdStats):
        # ReLU outputs only (the mask source: scale/shift or the residual path's bit mask)
        ctx.bnb = None
        if bwd_table is not None and training and relu and (bits is not None or ss is not None):
            table_, token = bwd_table
            ctx.bnb = BnBwdStats(x, ss if bits is None else None, bits, mean, table_, residual is not None, token)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bits, ss, mean, invstd, gamma = ctx.saved_tensors
        relu, has_res, training = ctx.cfg
        if not training:
            raise NotImplementedError("backward through eval-mode BatchNorm is not supported")
        tg = grad_target(gamma) if gamma is not None and ctx.needs_input_grad[1] else None
        tb = grad_target(ctx.beta) if ctx.beta is not None and ctx.needs_input_grad[2] else None
        if (tg is None) != (tb is None):
            tg = tb = None
        dy = dy.contiguous()
        # residual gradient of a bottleneck whose shortcut gradient joins conv1's dgrad (not the last
        # contributor): dres = dy * relu_mask is handed over as (dy, bits) and applied in that conv's
        # epilogue, so the backward apply kernel never stores it
        masked = has_res and ctx.join is not None and bits is not None and not ctx.join.is_last()
        bnb = ctx.bnb
        if bnb is not None and bnb.take_if_matches(dy):
            # the sums were accumulated by the dgrad that produced dy: finalize + apply only
            dx, dres, dgamma, dbeta = C().bn_bwd_table(dy, x, bits, ss if bits is None else None, mean, invstd, gamma,
                                                       relu, has_res and not masked, bnb.table, tg, tb)
        else:
            dx, dres, dgamma, dbeta = C().bn_bwd(dy, x, bits, ss, mean, invstd, gamma, relu, has_res and not masked,
                                                 tg, tb)
        ctx.bnb = None
        dg = dgamma if gamma is not None and ctx.needs_input_grad[1] else None
        db = dbeta if ctx.needs_input_grad[2] else None
        if masked:
            ctx.join.stash(MaskedGrad(dy, bits))
            dres = None
        elif has_res and ctx.join is not None:
            dres = ctx.join.contribute(dres)  # usually stashed for the consumer conv's dgrad epilogue
        return dx, dg, db, (dres if has_res else None), None, None, None, None, None, None, None, None, None, None, None


def _param_targets(ctx, gamma, beta, ig, ib):
    tg = grad_target(gamma) if gamma is not None and ctx.needs_input_grad[ig] else None
    tb = grad_target(beta) if beta is not None and ctx.needs_input_grad[ib] else None
    return (None, None) if (tg is None) != (tb is None) else (tg, tb)


_DUAL_BWD = os.environ.get("PDA_DUAL_BN_BWD", "1") == "1"


class _DualBatchNormFn(torch.autograd.Function):
    """``y = relu(bn(x) + bn2(x2))`` — a bottleneck's output with its downsample shortcut, both BNs
    finalized from their producing convs' statistics tables.  The forward writes y and the 1-bit ReLU
    mask in one pass (the shortcut's normalised tensor is never stored); the backward runs the two BN
    backwards on (dy, mask) directly, so the shortcut's gradient dy * mask is never stored either."""

    @staticmethod
    def forward(ctx, x, gamma, beta, x2, gamma2, beta2, rm, rv, rm2, rv2, table, shift, table2, shift2, nbt, nbt2,
                momentum, eps, bwd_tables=None):
        x, x2 = x.contiguous(), x2.contiguous()
        y, bits, mean, invstd, mean2, invstd2 = C().bn_fwd_train_sums_dual(
            x, table, shift, gamma, beta, rm, rv, nbt, x2, table2, shift2, gamma2, beta2, rm2, rv2, nbt2, momentum,
            eps)
        ctx.save_for_backward(x, x2, bits, mean, invstd, mean2, invstd2, gamma, gamma2)
        ctx.betas = (beta, beta2)
        # both BNs' backward sums from the next block's conv1 dgrad epilogue (the gradient join's last
        # contributor): (bt1, token), (bt2, token2) = bwd_tables
        ctx.bnb = None
        if bwd_tables is not None:
            (bt1, tok), (bt2, tok2) = bwd_tables
            ctx.bnb = BnBwdStats(x, None, bits, mean, bt1, True, (tok, tok2), second=(x2, mean2, bt2))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, x2, bits, mean, invstd, mean2, invstd2, gamma, gamma2 = ctx.saved_tensors
        beta, beta2 = ctx.betas
        dy = dy.contiguous()
        tg, tb = _param_targets(ctx, gamma, beta, 1, 2)
        tg2, tb2 = _param_targets(ctx, gamma2, beta2, 4, 5)
        bnb, ctx.bnb = ctx.bnb, None
        if bnb is not None and bnb.take_if_matches(dy):
            # both reductions were accumulated by the dgrad that produced dy: finalizes + the apply pass(es)
            if C().bn_bwd_dual_ok(x.shape[-1]):
                dx, dx2, dg, db, dg2, db2 = C().bn_bwd_dual(dy, bits, x, mean, invstd, gamma, x2, mean2, invstd2,
                                                            gamma2, tg, tb, tg2, tb2, bnb.table, bnb.table2)
            else:
                dx, _, dg, db = C().bn_bwd_table(dy, x, bits, None, mean, invstd, gamma, True, False, bnb.table, tg,
                                                 tb)
                dx2, _, dg2, db2 = C().bn_bwd_table(dy, x2, bits, None, mean2, invstd2, gamma2, True, False,
                                                    bnb.table2, tg2, tb2)
        elif _DUAL_BWD and C().bn_bwd_dual_ok(x.shape[-1]):
            # one reduce pass over (dy, bits, x, x2) and one apply pass writing dx and dx2
            dx, dx2, dg, db, dg2, db2 = C().bn_bwd_dual(dy, bits, x, mean, invstd, gamma, x2, mean2, invstd2, gamma2,
                                                        tg, tb, tg2, tb2)
        else:
            dx, _, dg, db = C().bn_bwd(dy, x, bits, None, mean, invstd, gamma, True, False, tg, tb)
            dx2, _, dg2, db2 = C().bn_bwd(dy, x2, bits, None, mean2, invstd2, gamma2, True, False, tg2, tb2)
        ng = ctx.needs_input_grad
        return (dx, dg if gamma is not None and ng[1] else None, db if beta is not None and ng[2] else None,
                dx2, dg2 if gamma2 is not None and ng[4] else None, db2 if beta2 is not None and ng[5] else None) \
            + (None,) * 13


def dual_bn_ok(x: torch.Tensor, training: bool) -> bool:
    """True when :func:`batch_norm_dual` runs as one native kernel for ``x``."""
    return training and x.is_cuda and x.dtype == torch.bfloat16 and C().bn_dual_ok(x.shape[-1])


def batch_norm_dual(x, bn, x2, bn2, stats, stats2, fuse_bwd_stats: bool = False):
    """``relu(bn(x) + bn2(x2))`` for two training-mode ``BatchNorm2d`` modules whose batch statistics
    were accumulated by the producing convs (``stats = (table, shift)`` from ``Conv2d(..., bn=...)``).
    ``fuse_bwd_stats``: the output feeds the next block's gradient join, whose last contributing conv
    reduces both BNs' backward sums in its dgrad epilogue (``PDA_BN_BWD_EPILOGUE=0``: the reduce pass)."""
    (t1, s1), (t2, s2) = stats, stats2
    bt = None
    if fuse_bwd_stats and _BWD_EPILOGUE and torch.is_grad_enabled():
        m = x.numel() // x.shape[-1]
        bt = (bn.bwd_table(x.device, m), bn2.bwd_table(x.device, m))
    y = _DualBatchNormFn.apply(x, bn.weight, bn.bias, x2, bn2.weight, bn2.bias, bn.running_mean, bn.running_var,
                               bn2.running_mean, bn2.running_var, t1, s1, t2, s2, bn.num_batches_tracked,
                               bn2.num_batches_tracked, bn.momentum, bn.eps, bt)
    if bt is not None and y.grad_fn is not None and getattr(y.grad_fn, "bnb", None) is not None:
        y._pda_bnb = y.grad_fn.bnb
    return y


def _ref_batch_norm(x, gamma, beta, residual, running_mean, running_var, training, momentum, eps, relu):
    C_ = x.shape[-1]
    xf = x.reshape(-1, C_)
    g = gamma.float() if gamma is not None else None
    b = beta.float() if beta is not None else None
    y = F.batch_norm(xf.float(), running_mean, running_var, g, b, training, momentum, eps)
    y = y.reshape(x.shape)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


_BWD_EPILOGUE = os.environ.get("PDA_BN_BWD_EPILOGUE", "1") == "1"


def batch_norm(x, gamma, beta, running_mean=None, running_var=None, training=True, momentum=0.1, eps=1e-5,
               residual=None, relu=False, residual_join=None, stats=None, num_batches_tracked=None, bwd_table=None):
    """BatchNorm over the last (channel) dim of ``x`` (any leading dims), then ``+residual``, then ReLU.
    ``residual_join``: the residual's gradient is handed to the join instead of autograd's add.
    ``stats``: ``(table, shift)`` — the statistics table filled by :func:`~.conv.conv2d_bn_stats`
    (``BatchNorm2d.stat_table``; re-zeroed by the finalize) — skips the statistics pass.
    ``num_batches_tracked``: int64 counter incremented in training mode (inside the finalize kernel on
    the native path, so it costs no launch of its own).
    ``bwd_table``: (zeroed [R, 2, C] fp32 table, token) (``BatchNorm2d.bwd_table``) — the caller guarantees that the
    output's only consumer is a conv (or, with a residual, the gradient join of the next block), whose
    dgrad epilogue then reduces this BN's backward sums (``PDA_BN_BWD_EPILOGUE=0``: the reduce pass)."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        table, shift = stats if stats is not None else (None, None)
        bt = bwd_table if (_BWD_EPILOGUE and training and torch.is_grad_enabled()) else None
        y = _BatchNormFn.apply(x, gamma, beta, residual, running_mean, running_var, training, momentum, eps,
                               relu, residual_join, table, shift, num_batches_tracked if training else None, bt)
        if bt is not None and y.grad_fn is not None:
            bnb = getattr(y.grad_fn, "bnb", None)
            if bnb is not None:
                y._pda_bnb = bnb
        return y
    if x.is_cuda and x.dtype == torch.float32 and x.shape[-1] % 4 == 0 and residual_join is None:
        from . import fp32

        return fp32.batch_norm(x, gamma, beta, running_mean, running_var, training, momentum, eps, residual, relu,
                               num_batches_tracked)
    if training and num_batches_tracked is not None:
        num_batches_tracked.add_(1)
    return _ref_batch_norm(x, gamma, beta, residual, running_mean, running_var, training, momentum, eps, relu)


def _param_grad_slots(ctx, gi: int):
    """Flat-buffer gradient slots of (gamma, beta) when both have one (the norm backward's finalize
    writes dgamma / dbeta there in the parameter dtype: no cast kernel, no copy into the DDP bucket)."""
    gamma, beta = ctx.params
    ng = ctx.needs_input_grad
    tg = grad_target(gamma) if ng[gi] else None
    tb = grad_target(beta) if (beta is not None and ng[gi + 1]) else None
    if beta is not None and (tg is None) != (tb is None):  # one slot only: let both allocate
        for p, t in ((gamma, tg), (beta, tb)):
            if t is not None:
                p._pda_claimed = False
        tg = tb = None
    return tg, tb


class _RowNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, rms):
        x = x.contiguous()
        y, mean, rstd = C().rownorm_fwd(x, gamma.contiguous(), beta, eps, rms)
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.rms = rms
        ctx.has_beta = beta is not None
        ctx.params = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, mean, rstd = ctx.saved_tensors
        tg, tb = _param_grad_slots(ctx, 1)
        dx, dg, db = C().rownorm_bwd(dy.contiguous(), x, gamma, mean, rstd, ctx.rms, None, tg, tb)
        return dx, dg, (db if ctx.has_beta else None), None, None


def layer_norm(x, weight, bias, eps=1e-5):
    if x.is_cuda and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192:
        return _RowNormFn.apply(x, weight, bias, eps, False)
    return F.layer_norm(x.float(), (x.shape[-1],), weight.float(), bias.float() if bias is not None else None,
                        eps).to(x.dtype)


def rms_norm(x, weight, eps=1e-6):
    if x.is_cuda and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192:
        return _RowNormFn.apply(x, weight, None, eps, True)
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return y.to(x.dtype)


class _AddRowNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, gamma, beta, eps, rms):
        h, y, mean, rstd = C().add_rownorm_fwd_train(x.contiguous(), r.contiguous(), gamma, beta, eps, rms)
        ctx.save_for_backward(h, gamma, mean, rstd)
        ctx.rms = rms
        ctx.has_beta = beta is not None
        ctx.params = (gamma, beta)
        return h, y

    @staticmethod
    def backward(ctx, dh, dy):
        h, gamma, mean, rstd = ctx.saved_tensors
        if dy is None:  # the normed output is unused: the residual gradient passes straight through
            return dh, dh, None, None, None, None
        addend = dh.contiguous() if dh is not None else None
        tg, tb = _param_grad_slots(ctx, 2)
        dx, dg, db = C().rownorm_bwd(dy.contiguous(), h, gamma, mean, rstd, ctx.rms, addend, tg, tb)
        return dx, dx, dg, (db if ctx.has_beta else None), None, None


def add_norm_train(x, r, weight, bias=None, eps=1e-5, rms=True):
    """``h = x + r`` and ``norm(h)`` with autograd; ``r=None`` is the plain norm (h = x).  Returns
    ``(h, normed)``.  GPU bf16: `rownorm.hip:add_rownorm_fwd_kernel` forward, `rownorm_bwd_dx_kernel`
    with the residual gradient as addend backward."""
    if r is None:
        return x, (rms_norm(x, weight, eps) if rms else layer_norm(x, weight, bias, eps))
    if (x.is_cuda and x.dtype == torch.bfloat16 and r.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and (bias is None or bias.dtype == torch.bfloat16) and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192
            and x.shape == r.shape):
        return _AddRowNormFn.apply(x, r, weight, None if rms else bias, eps, rms)
    h = x + r
    return h, (rms_norm(h, weight, eps) if rms else layer_norm(h, weight, bias, eps))


@torch.no_grad()
def add_norm(x, r, weight, bias=None, eps=1e-5, rms=True):
    """Inference: ``h = x + r`` and ``norm(h)`` in one pass (serving path; no autograd).
    Returns ``(h, normed)``.  GPU bf16: `rownorm.hip:add_rownorm_fwd_kernel`."""
    if (x.is_cuda and x.dtype == torch.bfloat16 and r.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192):
        h, y = C().add_rownorm_fwd(x.contiguous(), r.contiguous(), weight, bias, eps, rms)
        return h, y
    h = x + r
    return h, (rms_norm(h, weight, eps) if rms else layer_norm(h, weight, bias, eps))
