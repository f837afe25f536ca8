"""Implementation of the fused optimizers (see package docstring)."""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from .._native import C
from ..parallel.flat import FlatGroup, flat_group_of


class _FusedBase(torch.optim.Optimizer):
    """Common machinery: per-group flat-path detection, fp32 masters, gradient scale / clip input."""

    _state_names: tuple = ()

    def __init__(self, params, defaults, master_weights: Optional[bool] = None):
        super().__init__(params, defaults)
        self.master_weights = master_weights
        self._flat: Dict[int, dict] = {}  # group index -> flat state
        self.grad_scale: Optional[torch.Tensor] = None  # device scalar multiplied into every gradient
        # step counters mirrored on the device, so the update kernels read the step (Adam bias
        # correction) from memory and a captured step can be replayed from a HIP graph
        self._dstep: Dict[torch.device, list] = {}  # device -> [host value, device tensor]

    def _device_step(self, device: torch.device, host_step: int) -> Optional[torch.Tensor]:
        """Device counter equal to ``host_step`` after this step's increment (None if they diverge:
        a parameter that skipped steps keeps the exact host value instead)."""
        ent = self._dstep.get(device)
        if ent is None:
            ent = self._dstep[device] = [host_step - 1, torch.full((1,), float(host_step - 1),
                                                                  dtype=torch.float32, device=device), -1]
        if ent[2] != self._step_calls:  # first use of this device in this step() call: advance once
            ent[2] = self._step_calls
            ent[0] += 1
            ent[1].add_(1.0)
        return ent[1] if ent[0] == host_step else None

    def advance_steps(self, n: int):
        """Account for ``n`` updates that ran without Python (HIP graph replays): bump host counters."""
        for st in self._flat.values():
            st["step"] += n
        for s in self.state.values():
            if "step" in s:
                s["step"] += n
        for ent in self._dstep.values():
            ent[0] += n

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dstep.clear()
        # loaded per-parameter tensors replace the flat-buffer views in self.state: copy them back into
        # the flat buffers the update kernels read (and re-bind the views)
        for st in self._flat.values():
            self._link(st, load=True)

    def state_dict(self):
        # the flat path keeps the step count per group: mirror it into every parameter's state (torch's
        # layout: state[p]["step"]) so a resumed Adam continues its bias correction
        for st in self._flat.values():
            for p in st["fg"].params:
                self.state[p]["step"] = torch.tensor(float(st["step"]))
        return super().state_dict()

    # --------------------------------------------------------------- flat path
    def _link(self, st: dict, load: bool = False, old: Optional[dict] = None):
        """Expose per-parameter views of the flat state as regular optimizer state (checkpoint layout =
        torch's).  ``load``: tensors already in ``self.state`` (a loaded checkpoint) are copied into the
        flat buffers first.  ``old``: the state of the FlatGroup this one replaced (DDP re-bucketing):
        every parameter's slice is carried over to its new offset."""
        fg = st["fg"]
        names = list(self._state_names) + (["master_param"] if st["master"] is not fg.param_buffer else [])
        bufs = {n: st[n] for n in self._state_names}
        bufs["master_param"] = st["master"]
        ofg = old["fg"] if old is not None else None
        for p, off in zip(fg.params, fg.offsets):
            s = self.state[p]
            n = p.numel()
            for name in names:
                view = bufs[name][off: off + n].view_as(p)
                if old is not None and name in old and name != "master_param":
                    o = ofg.offsets[ofg.index[id(p)]]
                    view.copy_(old[name][o: o + n].view_as(p))
                elif old is not None and name == "master_param" and old["master"] is not ofg.param_buffer:
                    o = ofg.offsets[ofg.index[id(p)]]
                    view.copy_(old["master"][o: o + n].view_as(p))
                elif load and name in s and s[name].data_ptr() != view.data_ptr():
                    view.copy_(s[name].reshape(p.shape).to(view.dtype))
                s[name] = view
            if load and "step" in s:
                st["step"] = int(float(s["step"]))
        if old is not None:
            st["step"] = old["step"]

    def _flat_for(self, gi: int, group) -> Optional[dict]:
        params = [p for p in group["params"]]
        if not params or not params[0].is_cuda:
            return None
        fg = flat_group_of(params[0])
        if fg is None or not fg.covers(params):
            return None
        st = self._flat.get(gi)
        if st is None or st["fg"] is not fg:
            old = st if st is not None and getattr(st["fg"], "_pda_replaced_by", None) is fg else None
            # low-precision parameters always get an fp32 master; fp32 ones only on request
            need_master = fg.dtype != torch.float32 or bool(self.master_weights)
            master = fg.param_buffer.float().clone() if need_master else fg.param_buffer
            st = {"fg": fg, "master": master, "bf16": fg.param_buffer if fg.dtype == torch.bfloat16 and need_master
                  else None, "step": 0}
            for name in self._state_names:
                st[name] = torch.zeros(fg.numel, dtype=torch.float32, device=fg.device)
            self._flat[gi] = st
            # a checkpoint loaded before the first step left per-parameter tensors in self.state
            loaded = old is None and any(name in self.state.get(p, {}) for p in fg.params
                                         for name in self._state_names)
            self._link(st, load=loaded, old=old)
        return st

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._step_calls = getattr(self, "_step_calls", 0) + 1
        for gi, group in enumerate(self.param_groups):
            st = self._flat_for(gi, group)
            if st is not None:
                fg: FlatGroup = st["fg"]
                if fg.pending_comm:
                    raise RuntimeError(
                        f"optimizer step on a flat gradient buffer with {fg.pending_comm} bucket all-reduce(s) "
                        "the compute stream has not waited on (DDP backward did not finish its final callback)")
                if any(p.grad is None for p in fg.params):
                    fg.attach_grads()  # grads were set to None without a backward: the flat buffer holds them
                st["step"] += 1
                self._flat_update(st, group, fg.grad_buffer)
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                self._param_update(p, group)
        return loss

    # subclasses implement these
    def _flat_update(self, st, group, grad):
        raise NotImplementedError

    def _param_update(self, p, group):
        raise NotImplementedError

    def _gscale_args(self):
        return (1.0, self.grad_scale)


class SGD(_FusedBase):
    _state_names = ("momentum_buffer",)

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 master_weights: Optional[bool] = None):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults, master_weights)

    def _flat_update(self, st, group, grad):
        gs, gs_t = self._gscale_args()
        C().sgd_step(st["master"], st["bf16"], grad, st["momentum_buffer"], group["lr"], group["momentum"],
                     group["dampening"], group["weight_decay"], group["nesterov"], st["step"] == 1, gs, gs_t, None)

    def _param_update(self, p, group):
        s = self.state[p]
        lr, mom, damp, wd, nest = (group[k] for k in ("lr", "momentum", "dampening", "weight_decay", "nesterov"))
        if p.is_cuda and p.dtype in (torch.float32, torch.bfloat16) and p.is_contiguous():
            first = "step" not in s
            s["step"] = s.get("step", 0) + 1
            if p.dtype == torch.float32:
                master, pb = p, None
            else:
                if "master_param" not in s:
                    s["master_param"] = p.detach().float().clone()
                master, pb = s["master_param"], p
            if "momentum_buffer" not in s:
                s["momentum_buffer"] = torch.zeros_like(master)
            gs, gs_t = self._gscale_args()
            C().sgd_step(master, pb, p.grad.contiguous(), s["momentum_buffer"], lr, mom, damp, wd, nest, first, gs,
                         gs_t, None)
            return
        # reference math (torch.optim.SGD semantics)
        g = p.grad.float()
        if self.grad_scale is not None:
            g = g * self.grad_scale.to(g.device)
        if wd != 0:
            g = g + wd * p.float()
        if mom != 0:
            buf = s.get("momentum_buffer")
            if buf is None:
                buf = g.clone()
            else:
                buf.mul_(mom).add_(g, alpha=1 - damp)
            s["momentum_buffer"] = buf
            g = g + mom * buf if nest else buf
        p.add_((-lr * g).to(p.dtype))


class Adam(_FusedBase):
    _state_names = ("exp_avg", "exp_avg_sq")
    _decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 master_weights: Optional[bool] = None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults, master_weights)

    def _flat_update(self, st, group, grad):
        b1, b2 = group["betas"]
        gs, gs_t = self._gscale_args()
        C().adam_step(st["master"], st["bf16"], grad, st["exp_avg"], st["exp_avg_sq"], group["lr"], b1, b2,
                      group["eps"], group["weight_decay"], self._decoupled, st["step"], gs, gs_t, None,
                      self._device_step(grad.device, st["step"]))

    def _param_update(self, p, group):
        s = self.state[p]
        b1, b2 = group["betas"]
        lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
        s["step"] = s.get("step", 0) + 1
        t = s["step"]
        if p.is_cuda and p.dtype in (torch.float32, torch.bfloat16) and p.is_contiguous():
            if p.dtype == torch.float32:
                master, pb = p, None
            else:
                if "master_param" not in s:
                    s["master_param"] = p.detach().float().clone()
                master, pb = s["master_param"], p
            for n in self._state_names:
                if n not in s:
                    s[n] = torch.zeros_like(master)
            gs, gs_t = self._gscale_args()
            C().adam_step(master, pb, p.grad.contiguous(), s["exp_avg"], s["exp_avg_sq"], lr, b1, b2, eps, wd,
                          self._decoupled, t, gs, gs_t, None, self._device_step(p.device, t))
            return
        g = p.grad.float()
        if self.grad_scale is not None:
            g = g * self.grad_scale.to(g.device)
        pf = p.float()
        if self._decoupled:
            pf = pf * (1 - lr * wd)
        elif wd != 0:
            g = g + wd * pf
        for n in self._state_names:
            if n not in s:
                s[n] = torch.zeros_like(pf)
        m, v = s["exp_avg"], s["exp_avg_sq"]
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / math.sqrt(1 - b2 ** t)).add_(eps)
        pf = pf - (lr / (1 - b1 ** t)) * m / denom
        p.copy_(pf.to(p.dtype))


class AdamW(Adam):
    _decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 master_weights: Optional[bool] = None):
        super().__init__(params, lr, betas, eps, weight_decay, master_weights)


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm: float, optimizer: Optional[_FusedBase] = None) -> torch.Tensor:
    """Total-norm gradient clipping without a host sync.

    With a fused optimizer the clip coefficient is handed over as its device-side ``grad_scale`` (the
    gradients are not rewritten); otherwise gradients are scaled in place.  Returns the norm (device).
    """
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.zeros(())
    fg = flat_group_of(params[0])
    if params[0].is_cuda and fg is not None and fg.covers(params):
        out = C().grad_norm(fg.grad_buffer, 1.0, float(max_norm))
    elif params[0].is_cuda:
        sq = torch.stack([C().grad_norm(p.grad.contiguous(), 1.0, 0.0)[0] ** 2 for p in params]).sum()
        norm = sq.sqrt()
        out = torch.stack([norm, torch.clamp(max_norm / (norm + 1e-6), max=1.0)])
    else:
        norm = torch.norm(torch.stack([p.grad.float().norm() for p in params]))
        out = torch.stack([norm, torch.clamp(max_norm / (norm + 1e-6), max=1.0)])
    if optimizer is not None and isinstance(optimizer, _FusedBase):
        optimizer.grad_scale = out[1:2].float()
    else:
        for p in params:
            p.grad.mul_(out[1].to(p.grad.dtype))
    return out[0]
