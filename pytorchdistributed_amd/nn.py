"""``nn.Module`` layers over :mod:`pytorchdistributed_amd.ops`.

Image layers are channels-last: activations ``[N, H, W, C]``, conv weights ``[C_out, R, S, C_in]``.
Parameter initialisation follows torch's defaults (kaiming-uniform(a=sqrt(5)) for conv / linear,
ones / zeros for norms) so parameter counts and init statistics match the reference's torch models.
"""
from __future__ import annotations

import math

import os

import torch
import torch.nn as tnn

from . import ops

_EPILOGUE_STATS = os.environ.get("PDA_BN_EPILOGUE_STATS", "1") == "1"
# rows of the epilogue statistics table (atomic contention vs finalize read; 32..128 measured equal)
_STAT_ROWS = int(os.environ.get("PDA_BN_STAT_ROWS", "64"))


def deterministic() -> bool:
    """``PDA_DETERMINISTIC=1``: bit-reproducible training steps.  The only order-dependent reductions of
    the ResNet path are the BatchNorm sums the conv epilogues add atomically into a statistics table
    (forward) and the dgrad epilogues into the backward table: tile t adds into row t % R.  With R at
    least the number of output-row tiles (64-row tiles are the smallest), every row receives exactly one
    add per column (0 + v is exact) and the finalize sums the rows in a fixed order.  Split-K weight
    gradients already reduce fp32 slabs in a fixed order; everything else is elementwise or slab-based.
    The transformer path's two atomic reductions switch too (read per call by the native layer): the
    fused attention backward (dQ by fp32 atomics) gives way to the dQ + dK/dV kernel pair, and the
    embedding backward sums each token id's rows in sorted order (`embed.hip:embedding_bwd_sorted_kernel`)."""
    return os.environ.get("PDA_DETERMINISTIC", "0") == "1"


def stat_rows(m_rows: int) -> int:
    """Rows of a BN sums table for a conv output of ``m_rows`` pixels (see :func:`deterministic`)."""
    if deterministic():
        return max(_STAT_ROWS, (int(m_rows) + 63) // 64)
    return _STAT_ROWS


def _kaiming_uniform_(w: torch.Tensor, fan_in: int):
    bound = 1.0 / math.sqrt(fan_in) * math.sqrt(3.0) * math.sqrt(2.0 / (1 + 5))
    with torch.no_grad():
        w.uniform_(-bound, bound)
    return w


class Linear(tnn.Module):
    def __init__(self, in_features, out_features, bias=True, relu=False, device=None, dtype=None):
        super().__init__()
        self.in_features, self.out_features, self.relu = in_features, out_features, relu
        self.weight = tnn.Parameter(torch.empty(out_features, in_features, device=device, dtype=dtype))
        self.bias = tnn.Parameter(torch.empty(out_features, device=device, dtype=dtype)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        _kaiming_uniform_(self.weight, self.in_features)
        if self.bias is not None:
            b = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            with torch.no_grad():
                self.bias.uniform_(-b, b)

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, self.relu)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"


class Conv2d(tnn.Module):
    """Channels-last conv; ``weight`` is OHWI."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, bias=False,
                 device=None, dtype=None):
        super().__init__()
        k = kernel_size
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, k
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.weight = tnn.Parameter(torch.empty(out_channels, k, k, in_channels, device=device, dtype=dtype))
        self.bias = tnn.Parameter(torch.zeros(out_channels, device=device, dtype=dtype)) if bias else None
        _kaiming_uniform_(self.weight, in_channels * k * k)

    def forward(self, x, relu=False, grad_join=None, bn=None):
        """``bn``: the BatchNorm2d this conv feeds; ``(y, stats)`` is returned (pass it to the BN).  In
        training on the GPU (``PDA_BN_EPILOGUE_STATS=1``, default) the conv epilogue reduces that BN's
        batch statistics (each output tile atomically adds its column sums into the BN's statistics
        table), so the BN skips its statistics pass over y (one fewer HBM read of every BN input)."""
        if bn is not None:
            if (_EPILOGUE_STATS and x.is_cuda and bn.training and self.bias is None and not relu
                    and x.dtype == torch.bfloat16):
                k, st_, pd = self.kernel_size, self.stride, self.padding
                P = (x.shape[1] + 2 * pd - self.dilation * (k - 1) - 1) // st_ + 1
                Q = (x.shape[2] + 2 * pd - self.dilation * (k - 1) - 1) // st_ + 1
                table = bn.stat_table(x.device, x.shape[0] * P * Q)
                y = ops.conv2d_bn_stats(x, self.weight, self.stride, self.padding, self.dilation,
                                        bn.running_mean, table, grad_join)
                return y, (table, bn.running_mean)
            return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, relu,
                              grad_join), None
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, relu, grad_join)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, stride={self.stride}, "
                f"padding={self.padding}")


class BatchNorm2d(tnn.Module):
    """BatchNorm over the channel (last) dim; running statistics stay fp32 whatever the param dtype."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, device=None, dtype=None):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        if affine:
            self.weight = tnn.Parameter(torch.ones(num_features, device=device, dtype=dtype))
            self.bias = tnn.Parameter(torch.zeros(num_features, device=device, dtype=dtype))
        else:
            self.weight = self.bias = None
        self.register_buffer("running_mean", torch.zeros(num_features, device=device))
        self.register_buffer("running_var", torch.ones(num_features, device=device))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long, device=device))

    def stat_table(self, device, m_rows: int = 0) -> torch.Tensor:
        """Zeroed [R, 2, C] fp32 table that the producing conv's epilogue accumulates this BN's batch
        sums into (output tile t adds into row t % R, spreading the atomics over R rows) and that the
        BN finalize reads and re-zeroes — so it is zero between uses and needs no per-step memset.
        Not a registered buffer: never saved, broadcast or all-reduced."""
        t = getattr(self, "_stat_table", None)
        rows = stat_rows(m_rows)
        if t is None or t.device != torch.device(device) or t.shape[0] != rows:
            t = torch.zeros(rows, 2, self.num_features, device=device)
            self._stat_table = t
        return t

    def bwd_table(self, device, m_rows: int = 0):
        """(table, token) for the backward reduction fused into the consuming conv's dgrad epilogue
        (ops/grad_join.py:BnBwdStats): a zeroed [R, 2, C] fp32 table the epilogue accumulates into and the BN
        backward finalize re-zeroes, and the [filled] flag; a table some dgrad filled without a BN backward
        consuming it (aborted backward) is re-zeroed here before it is handed out again."""
        t = getattr(self, "_bwd_table", None)
        rows = stat_rows(m_rows)
        if t is None or t.device != torch.device(device) or t.shape[0] != rows:
            t = torch.zeros(rows, 2, self.num_features, device=device)
            self._bwd_table, self._bwd_token = t, [False]
        elif self._bwd_token[0]:
            t.zero_()
            self._bwd_token[0] = False
        return t, self._bwd_token

    def _apply(self, fn, recurse=True):
        # keep running stats in fp32 when the module is cast to bf16
        rm, rv = self.running_mean, self.running_var
        super()._apply(fn, recurse)
        if self.running_mean.dtype != torch.float32:
            self.running_mean = fn(rm).float()
            self.running_var = fn(rv).float()
        return self

    def forward(self, x, residual=None, relu=False, residual_join=None, stats=None, fuse_bwd_stats=False):
        """``fuse_bwd_stats``: the output's consumers are known to be one conv (or, with a residual, the next
        block's gradient join): that conv's dgrad epilogue then reduces this BN's backward sums."""
        if isinstance(x, tuple):  # (y, stats) from Conv2d(..., bn=self)
            x, stats = x
        bt = None
        if fuse_bwd_stats and self.training and x.is_cuda and x.dtype == torch.bfloat16 and relu:
            bt = self.bwd_table(x.device, x.numel() // x.shape[-1])
        return ops.batch_norm(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                              self.momentum, self.eps, residual=residual, relu=relu, residual_join=residual_join,
                              stats=stats, num_batches_tracked=self.num_batches_tracked, bwd_table=bt)


class ReLU(tnn.Module):
    def forward(self, x):
        return ops.relu(x)


class MaxPool2d(tnn.Module):
    def __init__(self, kernel_size=3, stride=2, padding=1):
        super().__init__()
        self.k, self.s, self.p = kernel_size, stride, padding

    def forward(self, x):
        return ops.max_pool2d(x, self.k, self.s, self.p)


class GlobalAvgPool2d(tnn.Module):
    def forward(self, x):
        return ops.global_avg_pool2d(x)


class LayerNorm(tnn.Module):
    def __init__(self, dim, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = tnn.Parameter(torch.ones(dim, device=device, dtype=dtype))
        self.bias = tnn.Parameter(torch.zeros(dim, device=device, dtype=dtype))

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, self.eps)


class RMSNorm(tnn.Module):
    def __init__(self, dim, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = tnn.Parameter(torch.ones(dim, device=device, dtype=dtype))

    def forward(self, x):
        return ops.rms_norm(x, self.weight, self.eps)
