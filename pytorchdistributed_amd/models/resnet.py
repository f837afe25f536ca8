"""ResNet-50 v1.5, channels-last, built on the framework's native layers.

Reference: torchvision ``ResNet(Bottleneck, [3, 4, 6, 3], 1000)`` used in
`03 模型并行/03_model_parallel.ipynb` (raw lines 107-110, 314: 25,557,032 parameters; the model/pipeline
parallel variants at raw lines 325-349 and 538-561).  torchvision is not available on the target, so
the architecture is re-built here: same layer names (``conv1``, ``bn1``, ``layer1..4``, ``fc``, blocks
``conv1..3`` / ``bn1..3`` / ``downsample``), same parameter count, stride on the 3x3 conv (v1.5).

Differences by design (MI355X-first):
* activations are ``[N, H, W, C]`` and conv weights OHWI; the 7x7/2 stem runs as a 4x4/1 conv over a
  2x2 space-to-depth image with 16 channels (:func:`space_to_depth_stem`; implicit-GEMM gathers want
  16-byte channel vectors);
* BN+ReLU and BN+residual-add+ReLU are single fused kernels (``bn(x, residual=..., relu=True)``).
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.nn as tnn
import torch.nn.functional as F

from .. import nn as pnn
from .. import ops
from ..ops.grad_join import GradJoin


class Bottleneck(tnn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=False, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        width = planes
        self.conv1 = pnn.Conv2d(inplanes, width, 1, **kw)
        self.bn1 = pnn.BatchNorm2d(width, **kw)
        self.conv2 = pnn.Conv2d(width, width, 3, stride=stride, padding=1, **kw)
        self.bn2 = pnn.BatchNorm2d(width, **kw)
        self.conv3 = pnn.Conv2d(width, planes * 4, 1, **kw)
        self.bn3 = pnn.BatchNorm2d(planes * 4, **kw)
        if downsample:
            self.downsample = tnn.Sequential(pnn.Conv2d(inplanes, planes * 4, 1, stride=stride, **kw),
                                             pnn.BatchNorm2d(planes * 4, **kw))
        else:
            self.downsample = None

    def forward(self, x):
        # x feeds conv1 and the shortcut: its two gradients are summed inside conv1's (or the
        # downsample conv's) dgrad store instead of by a separate autograd add (ops/grad_join.py)
        # Every conv also reduces the batch statistics of the BN it feeds in its epilogue (bn=...).
        join = (GradJoin(2) if (x.is_cuda and x.dtype == torch.bfloat16 and x.requires_grad and torch.is_grad_enabled())
                else None)
        # bn1 / bn2 outputs feed exactly one conv each: their backward reductions run in conv2's / conv3's
        # dgrad epilogues (fuse_bwd_stats); bn3's output feeds the next block's gradient join
        out = self.bn1(self.conv1(x, grad_join=join, bn=self.bn1), relu=True, fuse_bwd_stats=True)
        out = self.bn2(self.conv2(out, bn=self.bn2), relu=True, fuse_bwd_stats=True)
        if self.downsample is not None:
            conv_ds, bn_ds = self.downsample
            zd = conv_ds(x, grad_join=join, bn=bn_ds)
            z3 = self.conv3(out, bn=self.bn3)
            if (_DUAL_BN and zd[1] is not None and z3[1] is not None and ops.dual_bn_ok(z3[0], self.bn3.training)
                    and (bn_ds.eps, bn_ds.momentum) == (self.bn3.eps, self.bn3.momentum)):
                # relu(bn3(z3) + bn_ds(zd)) in one kernel: the shortcut's BN output and its gradient
                # are never stored (PDA_DUAL_BN=0: the separate shortcut BN apply)
                return ops.batch_norm_dual(z3[0], self.bn3, zd[0], bn_ds, z3[1], zd[1], fuse_bwd_stats=_BN3_BWD_JOIN)
            return self.bn3(z3, residual=bn_ds(zd), relu=True)
        return self.bn3(self.conv3(out, bn=self.bn3), residual=x, relu=True, residual_join=join,
                        fuse_bwd_stats=_BN3_BWD_JOIN)


_STEM_S2D = os.environ.get("PDA_STEM_S2D", "1") == "1"
_DUAL_BN = os.environ.get("PDA_DUAL_BN", "1") == "1"
_STEM_BN_POOL = os.environ.get("PDA_STEM_BN_POOL", "1") == "1"
# an identity block's output BN: its backward sums from the next block's conv1 dgrad (the gradient join's
# last contributor, whose epilogue adds the shortcut gradient) — PDA_BN3_BWD_JOIN=0: the reduce pass
_BN3_BWD_JOIN = os.environ.get("PDA_BN3_BWD_JOIN", "1") == "1"


def space_to_depth_stem(x: torch.Tensor, w: torch.Tensor):
    """Rewrite the 7x7 / stride-2 / pad-3 stem conv as a 4x4 / stride-1 conv over a 2x2
    space-to-depth image (the MLPerf ResNet stem trick):

        y[p, q] = sum_{a,b<4} w2[a, b, (i, j, c)] * X2[p + a, q + b, (i, j, c)]
        X2[u, v, (i, j, c)] = pad3(x)[2u + i, 2v + j, c],   w2[a, b, (i, j, c)] = w[2a + i, 2b + j, c]

    (w2 is zero where 2a + i = 7 or 2b + j = 7).  Channels (i, j, c) = 12 are padded to 16, so the
    implicit GEMM has K = 4*4*16 = 256 instead of 7*7*8 = 392: 35 % fewer forward MACs, and the weight
    gradient's N = 256 fills two 128-wide tiles exactly instead of 392 spilling into a fourth.  The
    weight transform is differentiable torch ops on a 9.4k-element tensor, so autograd maps the
    gradient back onto the [64, 7, 7, 3] parameter."""
    Cc = w.shape[-1]
    cpad = (-4 * Cc) % 16
    x2 = None
    if x is not None:  # (x = None: weight only; the GPU path builds x2 with the stem_s2d kernel)
        N, H, W, _ = x.shape
        xp = F.pad(x, (0, 0, 3, 3 + H % 2, 3, 3 + W % 2))  # H, W -> even sizes >= H + 6
        Hp, Wp = xp.shape[1], xp.shape[2]
        x2 = xp.view(N, Hp // 2, 2, Wp // 2, 2, Cc).permute(0, 1, 3, 2, 4, 5).reshape(N, Hp // 2, Wp // 2, 4 * Cc)
        x2 = F.pad(x2, (0, cpad)) if cpad else x2.contiguous()
    O = w.shape[0]
    w8 = F.pad(w[..., :Cc], (0, 0, 0, 1, 0, 1))  # [O, 8, 8, C]
    w2 = w8.view(O, 4, 2, 4, 2, Cc).permute(0, 1, 3, 2, 4, 5).reshape(O, 4, 4, 4 * Cc)
    w2 = F.pad(w2, (0, cpad)) if cpad else w2
    return x2, w2


class Stem(tnn.Module):
    def __init__(self, device=None, dtype=None):
        super().__init__()
        self.conv1 = pnn.Conv2d(3, 64, 7, stride=2, padding=3, device=device, dtype=dtype)
        self.bn1 = pnn.BatchNorm2d(64, device=device, dtype=dtype)
        self.maxpool = pnn.MaxPool2d(3, 2, 1)

    def forward(self, x):
        if x.dim() == 4 and x.shape[1] == 3 and x.shape[-1] != 3:  # NCHW input -> NHWC
            x = x.permute(0, 2, 3, 1)
        if x.is_cuda and _STEM_S2D and self.conv1.weight.shape[-1] == 3:
            # (input channels beyond the weight's 3 are device-side padding: dropped by the rewrite)
            if x.dtype == torch.bfloat16 and not x.requires_grad:
                from .._native import C as _C

                x2 = _C().stem_s2d(x.contiguous(), 3, 3)  # one pass, HIP kernel
                w2 = space_to_depth_stem(None, self.conv1.weight)[1]
            else:
                x2, w2 = space_to_depth_stem(x[..., :3], self.conv1.weight)
            # (the space-to-depth image is sized so the 4x4 valid conv yields exactly ceil(H/2) x ceil(W/2))
            bn = self.bn1
            if pnn._EPILOGUE_STATS and bn.training and x2.dtype == torch.bfloat16:
                table = bn.stat_table(x2.device, x2.shape[0] * (x2.shape[1] - 3) * (x2.shape[2] - 3))
                y = ops.conv2d_bn_stats(x2, w2, 1, 0, 1, bn.running_mean, table)
                mp = self.maxpool
                if _STEM_BN_POOL:  # BN + ReLU applied inside the pool's loads: the BN output is never stored
                    return ops.bn_relu_max_pool2d(y, bn, (table, bn.running_mean), mp.k, mp.s, mp.p)
                return mp(bn((y, (table, bn.running_mean)), relu=True))
            return self.maxpool(bn(ops.conv2d(x2, w2, None, 1, 0), relu=True))
        if x.is_cuda and x.shape[-1] % 8 != 0:
            x = F.pad(x, (0, 8 - x.shape[-1] % 8))
        x = x.contiguous()
        return self.maxpool(self.bn1(self.conv1(x, bn=self.bn1), relu=True))


class ResNet(tnn.Module):
    nhwc = True  # activations are channels-last end to end (utils.summary reports NCHW shapes)

    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.stem = Stem(**kw)
        inplanes = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            blocks = []
            for j in range(n):
                blocks.append(Bottleneck(inplanes, planes, stride if j == 0 else 1, downsample=(j == 0), **kw))
                inplanes = planes * 4
            setattr(self, f"layer{i + 1}", tnn.Sequential(*blocks))
        self.fc = pnn.Linear(512 * 4, num_classes, **kw)

    # torchvision-compatible aliases for the stem layers
    @property
    def conv1(self):
        return self.stem.conv1

    @property
    def bn1(self):
        return self.stem.bn1

    def features(self, x):
        x = self.stem(x)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        return self.layer4(x)

    def forward(self, x):
        x = self.features(x)
        x = ops.global_avg_pool2d(x)
        return self.fc(x)

    # checkpoint layout of the reference (torchvision ResNet: `conv1`/`bn1` at top level, OIHW conv
    # weights) — utils/checkpoint.py saves MODEL_STATE in it, so a stock torchvision ResNet-50 loads it
    def reference_state_dict(self) -> dict:
        return to_torchvision_state_dict(self)

    def load_reference_state_dict(self, sd: dict):
        return from_torchvision_state_dict(self, sd)

    def stage_modules(self) -> List[tnn.Module]:
        """Ordered top-level stages (used by model/pipeline parallel splits, `NB03:325-349`)."""
        return [self.stem, self.layer1, self.layer2, self.layer3, self.layer4, _Head(self.fc)]


class _Head(tnn.Module):
    def __init__(self, fc):
        super().__init__()
        self.fc = fc

    def forward(self, x):
        return self.fc(ops.global_avg_pool2d(x))


def resnet50(num_classes=1000, device=None, dtype=None) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes, device=device, dtype=dtype)


def num_parameters(model: tnn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def to_torchvision_state_dict(model: ResNet) -> dict:
    """Convert to torchvision key/layout conventions (OIHW conv weights, ``conv1``/``bn1`` at top level)."""
    out = {}
    for k, v in model.state_dict().items():
        if k.startswith("stem."):
            k = k[len("stem."):]
        if v.dim() == 4:
            v = v.permute(0, 3, 1, 2).contiguous()
        out[k] = v
    return out


def from_torchvision_state_dict(model: ResNet, sd: dict):
    mine = {}
    for k, v in sd.items():
        key = ("stem." + k) if (k.startswith("conv1") or k.startswith("bn1")) else k
        if v.dim() == 4:
            v = v.permute(0, 2, 3, 1).contiguous()
        mine[key] = v
    return model.load_state_dict(mine)
