"""Flat-buffer parameters and the fused clip_grad_norm_ + Adam/RMSprop step.

The policy's parameters are re-pointed into ONE contiguous fp32 HBM buffer (and
their .grad into a second), so the optimizer step is two HIP launches over a flat
array (rai_clip_optim_step) instead of per-tensor foreach kernels plus the
reference's `.item()` sync inside clip_grad_norm_ (rl_algo_impls/ppo/ppo.py:441-447).

Checkpoint drop-in: state_dict()/load_state_dict() speak torch.optim.Adam /
RMSprop's format (per-parameter 'step', 'exp_avg', 'exp_avg_sq' / 'square_avg'
in policy.parameters() order), which is what rl_algo_impls/shared/algorithm.py:48-60
saves as optimizer.pt.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib


def struct_to_device(struct, device, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    raw = torch.frombuffer(bytearray(bytes(struct)), dtype=torch.uint8)
    if out is None:
        out = torch.empty(raw.shape, dtype=torch.uint8, device=device)
    out.copy_(raw, non_blocking=False)
    return out


class FlatParams:
    """Views every parameter of `module` into one flat fp32 buffer (+ flat grads).

    channels_last: parameters (4-D convolution weights) whose segment is laid out (K, kh, kw, C),
    the parameter being a channels_last-strided view of it.  The NHWC MIOpen convolutions then take
    the weight as stored (no per-call NCHW -> NHWC copy of the weight, forward and backward) and
    the weight gradient they return accumulates with matching strides.  The logical tensors (and so
    state_dict(), model.pth and optimizer.pt) are unchanged; vector() gives parameters() order."""

    def __init__(self, module: torch.nn.Module, device: torch.device, channels_last=()):
        self.params: List[torch.nn.Parameter] = list(module.parameters())
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("flat optimizer expects fp32 parameters")
        cl = {id(p) for p in channels_last}
        self.cl = [id(p) in cl and p.dim() == 4 for p in self.params]
        self.shapes = [tuple(p.shape) for p in self.params]
        sizes = [p.numel() for p in self.params]
        self.P = int(sum(sizes))
        self.flat = torch.empty(self.P, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.P, dtype=torch.float32, device=device)
        off = 0
        self.offsets = []
        for p, n in zip(self.params, sizes):
            self.offsets.append(off)
            off += n
        with torch.no_grad():
            for i, p in enumerate(self.params):
                self.as_param(self.flat, i).copy_(p.detach())
                p.data = self.as_param(self.flat, i)
                p.grad = self.as_param(self.grad, i)

    def as_param(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        """Parameter i's segment of a flat buffer (params, grads, optimizer moments) as a tensor of
        the parameter's shape and layout."""
        off, shp = self.offsets[i], self.shapes[i]
        seg = buf[off:off + int(np.prod(shp))]
        if self.cl[i]:
            K, C, kh, kw = shp
            return seg.view(K, kh, kw, C).permute(0, 3, 1, 2)
        return seg.view(shp)

    def vector(self, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        """A flat buffer in parameters() order with each parameter flattened row-major (what
        torch.nn.utils.parameters_to_vector gives), whatever the segments' layout."""
        buf = self.flat if buf is None else buf
        if not any(self.cl):
            return buf
        return torch.cat([self.as_param(buf, i).reshape(-1) for i in range(len(self.params))])

    def check_views(self) -> None:
        for p, off in zip(self.params, self.offsets):
            assert p.data.data_ptr() == self.flat.data_ptr() + 4 * off, "parameter storage was replaced"
            assert p.grad is not None and p.grad.data_ptr() == self.grad.data_ptr() + 4 * off, (
                "gradient storage was replaced (zero_grad(set_to_none=True)?)")
            assert p.data.stride() == p.grad.stride(), "parameter / gradient layouts differ"


class FlatOptimizer:
    """Adam(eps) / RMSprop(alpha, eps) with clip_grad_norm_ fused, torch-format state."""

    ADAM, RMSPROP = 0, 1

    def __init__(self, flat: FlatParams, kind: int, lr: float, eps: float, betas=(0.9, 0.999),
                 alpha: float = 0.99, max_grad_norm: float = 0.5):
        self.flat = flat
        self.kind = kind
        dev = flat.flat.device
        self.device = dev
        self.state1 = torch.zeros_like(flat.flat)
        self.state2 = torch.zeros_like(flat.flat) if kind == self.ADAM else None
        self.betas = tuple(betas)
        self.eps = eps
        self.alpha = alpha
        self.max_grad_norm = max_grad_norm
        self.param_groups = [dict(lr=lr)]
        self.step_count = 0
        self.hp_dev = torch.empty(C.sizeof(_lib.OptimHparams), dtype=torch.uint8, device=dev)
        # the per-block partial sums of squares between the two launches
        self.workspace = torch.zeros(int(_lib.lib().rai_optim_workspace_bytes(flat.P)), dtype=torch.uint8,
                                     device=dev)
        self.sync_hparams()

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def sync_hparams(self) -> None:
        hp = _lib.OptimHparams(lr=float(self.lr), beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                               alpha=self.alpha, max_grad_norm=float(self.max_grad_norm or 0.0), kind=self.kind,
                               beta1_d=float(self.betas[0] if self.kind == self.ADAM else self.alpha),
                               beta2_d=float(self.betas[1]))
        struct_to_device(hp, self.device, self.hp_dev)

    def step(self, state_dev: torch.Tensor, norms: Optional[torch.Tensor], count: bool = True) -> None:
        """Enqueue clip + update (+ zero grads); no host sync.  count=False for launches recorded
        into a graph (the caller accounts for the replays in step_count)."""
        f = self.flat
        rc = _lib.lib().rai_clip_optim_step(
            f.flat.data_ptr(), f.grad.data_ptr(), self.state1.data_ptr(),
            None if self.state2 is None else self.state2.data_ptr(), f.P, self.hp_dev.data_ptr(),
            state_dev.data_ptr(), None if norms is None else norms.data_ptr(),
            0 if norms is None else int(norms.numel()), self.workspace.data_ptr(), self.workspace.numel(),
            _lib.stream_handle(self.device))
        _lib.check(rc, "rai_clip_optim_step")
        if count:
            self.step_count += 1

    # -- torch-format checkpoint ------------------------------------------------------
    def state_dict(self) -> Dict:
        state = {}
        for i, (p, off) in enumerate(zip(self.flat.params, self.flat.offsets)):
            n = p.numel()
            if self.step_count == 0:
                continue
            s = {"step": torch.tensor(float(self.step_count))}
            as_p = lambda buf: self.flat.as_param(buf, i).contiguous().clone()  # torch's layout
            if self.kind == self.ADAM:
                s["exp_avg"] = as_p(self.state1)
                s["exp_avg_sq"] = as_p(self.state2)
            else:
                s["square_avg"] = as_p(self.state1)
            state[i] = s
        if self.kind == self.ADAM:
            group = dict(lr=self.lr, betas=self.betas, eps=self.eps, weight_decay=0, amsgrad=False,
                         maximize=False, foreach=None, capturable=False, differentiable=False, fused=None)
        else:
            group = dict(lr=self.lr, alpha=self.alpha, eps=self.eps, weight_decay=0, momentum=0,
                         centered=False, capturable=False, foreach=None, maximize=False, differentiable=False)
        group["params"] = list(range(len(self.flat.params)))
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd: Dict) -> None:
        steps = set()
        for i, s in sd["state"].items():
            i = int(i)
            p = self.flat.params[i]
            as_p = lambda buf: self.flat.as_param(buf, i)
            if self.kind == self.ADAM:
                as_p(self.state1).copy_(s["exp_avg"].reshape(p.shape))
                as_p(self.state2).copy_(s["exp_avg_sq"].reshape(p.shape))
            else:
                as_p(self.state1).copy_(s["square_avg"].reshape(p.shape))
            steps.add(int(float(s["step"])))
        if len(steps) > 1:
            raise NotImplementedError("per-parameter step counts differ; flat optimizer needs one")
        self.step_count = steps.pop() if steps else 0
        self.param_groups[0]["lr"] = sd["param_groups"][0]["lr"]
        self.sync_hparams()
