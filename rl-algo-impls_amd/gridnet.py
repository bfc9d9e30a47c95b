"""GridNet (MicroRTS) masked-categorical action head with a fused HIP log-prob/entropy operator.

Mirrors rl_algo_impls/shared/actor/gridnet.py: ValueDependentMask (:21-35) and
GridnetDistribution (:38-224) for per-position actions.  The reference builds H*W*7 torch
MaskedCategoricals per minibatch and stacks ~30 eager kernels per sub-action for log_prob and
entropy (plus their autograd backward); here log_prob + entropy of every cell and sub-action is
ONE launch (rai_gridnet_logp_entropy) and the backward ONE launch (rai_gridnet_backward), through
`GridnetLogpEntropy` (a torch.autograd.Function, so the network upstream still backpropagates
through PyTorch-ROCm).  The rollout samples every cell and plane and takes the sample's log-prob in
ONE launch (rai_gridnet_sample, `sample_with_logp`); sample()/mode keep the per-group torch form for
eval/enjoy.  The Lux
"pick_position" variant is outside the hot path and rejected loudly.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, NamedTuple, Optional, Tuple

import numpy as np
import torch

from . import _lib

F32_MIN = torch.finfo(torch.float32).min


class ValueDependentMask(NamedTuple):  # gridnet.py:21-35
    reference_index: int
    value: int

    @classmethod
    def from_reference_index_to_index_to_value(cls, ref_idx_to_idx_to_value: Dict[int, Dict[int, int]]):
        return {idx: cls(ref, v) for ref, m in ref_idx_to_idx_to_value.items() for idx, v in m.items()}


class _Spec:
    """Host arrays of the launch (nvec, gate reference and value per group)."""

    def __init__(self, action_vec, subaction_mask: Optional[Dict[int, ValueDependentMask]]):
        self.nvec = np.ascontiguousarray(np.asarray(action_vec, dtype=np.int32))
        G = len(self.nvec)
        if G > _lib.RAI_GRID_MAX_G or int(self.nvec.sum()) > _lib.RAI_GRID_MAX_A:
            raise NotImplementedError(f"GridNet head with {G} groups / {int(self.nvec.sum())} logits per cell")
        self.sub_ref = np.full(G, -1, dtype=np.int32)
        self.sub_val = np.zeros(G, dtype=np.int32)
        for idx, (ref, val) in (subaction_mask or {}).items():
            self.sub_ref[idx], self.sub_val[idx] = ref, val
        self.G, self.A = G, int(self.nvec.sum())

    def ptrs(self):
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        return p(self.nvec), p(self.sub_ref), p(self.sub_val)


_CAT_SPECS: Dict[int, "_Spec"] = {}


def categorical_spec(n: int) -> "_Spec":
    """A flat Categorical(n) as a GridNet head with one cell and one plane."""
    sp = _CAT_SPECS.get(n)
    if sp is None:
        sp = _CAT_SPECS[n] = _Spec([n], None)
    return sp


def _u8(m: torch.Tensor) -> torch.Tensor:
    m = m.contiguous()
    return m.view(torch.uint8) if m.dtype == torch.bool else m.to(torch.uint8)


def gridnet_num_actions(actions: torch.Tensor, action_masks: torch.Tensor, action_vec,
                        subaction_mask: Optional[Dict[int, ValueDependentMask]]) -> torch.Tensor:
    """Batch.num_actions of a GridNet rollout, rl_algo_impls/rollout/rollout.py:158-180
    (per_position_num_actions): actions (..., C, G) int64, action_masks (..., C, A) bool -> (...,)
    counts, one launch (rai_gridnet_num_actions).  Without a subaction mask: cells with any valid
    action, int64 (np.sum of a bool array; actions may be None); with one: valid groups per cell, each gated by its
    ValueDependentMask, int32 (the reference's np.zeros(..., dtype=np.int32) accumulator)."""
    _lib.require_device(actions, action_masks)
    per_group = bool(subaction_mask)
    spec = _Spec(action_vec if per_group else [int(action_masks.shape[-1])], subaction_mask)
    lead = tuple(action_masks.shape[:-2])
    Cc, A = int(action_masks.shape[-2]), int(action_masks.shape[-1])
    if A != spec.A or (per_group and (tuple(actions.shape[:-1]) != lead + (Cc,) or int(actions.shape[-1]) != spec.G)):
        raise AssertionError(f"num_actions: actions {None if actions is None else tuple(actions.shape)} / masks "
                             f"{tuple(action_masks.shape)} do not match nvec {np.asarray(action_vec).tolist()}")
    out = torch.empty(lead, dtype=torch.int32 if per_group else torch.int64, device=action_masks.device)
    m = _u8(action_masks)
    act = actions.contiguous() if per_group else None  # the plain count never reads the actions
    nv, sr, sv = spec.ptrs()
    rc = _lib.lib().rai_gridnet_num_actions(m.data_ptr(), _lib.ptr(act), int(out.numel()), Cc, spec.G, nv, sr, sv,
                                            int(per_group), out.element_size(), out.data_ptr(),
                                            _lib.stream_handle(m.device))
    _lib.check(rc, "rai_gridnet_num_actions")
    return out


class GridnetLogpEntropy(torch.autograd.Function):
    """(logits (B, C, A), masks (B, C, A), actions (B, C, G) | None) -> (logp (B,), entropy (B,))."""

    @staticmethod
    def forward(ctx, logits, masks, actions, spec: _Spec):
        _lib.require_device(logits, masks, actions)
        B, Cc = int(logits.shape[0]), int(logits.shape[1])
        z = logits.contiguous()
        m = _u8(masks)
        act = actions.contiguous() if actions is not None else None
        logp = torch.empty(B, dtype=torch.float32, device=z.device)
        ent = torch.empty(B, dtype=torch.float32, device=z.device)
        nv, sr, sv = spec.ptrs()
        rc = _lib.lib().rai_gridnet_logp_entropy(z.data_ptr(), m.data_ptr(), _lib.ptr(act), B, Cc, spec.G, nv, sr, sv,
                                                 logp.data_ptr() if act is not None else None, ent.data_ptr(),
                                                 _lib.stream_handle(z.device))
        _lib.check(rc, "rai_gridnet_logp_entropy")
        if act is None:
            logp = torch.zeros_like(ent)
        ctx.save_for_backward(z, m, act if act is not None else torch.empty(0, dtype=torch.int64, device=z.device))
        ctx.spec, ctx.has_act = spec, act is not None
        return logp, ent

    @staticmethod
    def backward(ctx, d_logp, d_ent):
        z, m, act = ctx.saved_tensors
        spec = ctx.spec
        B, Cc = int(z.shape[0]), int(z.shape[1])
        if not ctx.has_act:  # entropy only: gate and one-hot terms vanish with a zero upstream logp grad
            act = torch.zeros((B, Cc, spec.G), dtype=torch.int64, device=z.device)
            d_logp = None
        gl = d_logp.contiguous().float() if d_logp is not None else torch.zeros(B, device=z.device)
        ge = d_ent.contiguous().float() if d_ent is not None else torch.zeros(B, device=z.device)
        dz = torch.empty_like(z)
        nv, sr, sv = spec.ptrs()
        rc = _lib.lib().rai_gridnet_backward(z.data_ptr(), m.data_ptr(), act.data_ptr(), B, Cc, spec.G, nv, sr, sv,
                                             gl.data_ptr(), ge.data_ptr(), dz.data_ptr(), _lib.stream_handle(z.device))
        _lib.check(rc, "rai_gridnet_backward")
        return dz, None, None, None


class GridnetDistribution:  # gridnet.py:38-224 (per-position actions)
    def __init__(self, map_size: int, action_vec, logits: torch.Tensor, masks, validate_args=None,
                 subaction_mask: Optional[Dict[int, ValueDependentMask]] = None) -> None:
        if isinstance(masks, dict):
            if "pick_position" in masks:
                raise NotImplementedError("pick_position (Lux) GridNet actions are outside the hot path")
            masks = masks["per_position"]
        self.map_size = map_size
        self.action_vec = np.asarray(action_vec)
        self.subaction_mask = subaction_mask
        self._spec = _Spec(self.action_vec, subaction_mask)
        A = self._spec.A
        self.logits = logits.reshape(-1, map_size, logits.shape[-1])[..., :A]
        if logits.shape[-1] != A:
            raise NotImplementedError("logits wider than sum(action_vec) (pick_position) are not supported")
        self.masks = masks.reshape(-1, map_size, A)
        self._cache: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None
        self._entropy: Optional[torch.Tensor] = None

    def _fused(self, action: Optional[torch.Tensor]):
        act = None if action is None else action.reshape(-1, self.map_size, self._spec.G)
        return GridnetLogpEntropy.apply(self.logits, self.masks, act, self._spec)

    def log_prob(self, action) -> torch.Tensor:
        if isinstance(action, dict):
            if "pick_position" in action:
                raise NotImplementedError("pick_position (Lux) GridNet actions are outside the hot path")
            action = action["per_position"]
        logp, ent = self._fused(action)
        self._entropy = ent  # the same launch produced it: entropy() reuses it (one backward)
        return logp

    def entropy(self) -> torch.Tensor:
        if self._entropy is None:
            _, self._entropy = self._fused(None)
        return self._entropy

    def _groups(self):
        offs = np.concatenate([[0], np.cumsum(self.action_vec)])
        for g in range(len(self.action_vec)):
            lg = self.logits[..., offs[g]:offs[g + 1]]
            mk = self.masks[..., offs[g]:offs[g + 1]].bool()
            yield torch.where(mk, lg, torch.tensor(F32_MIN, dtype=lg.dtype, device=lg.device))

    def sample_with_logp(self, seed: int, offset: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Rollout path: sample() + log_prob(sample) in ONE launch (rai_gridnet_sample; Philox keyed
        (seed, offset), so a rollout step is reproducible without the torch generator)."""
        z = self.logits.contiguous()
        _lib.require_device(z)
        m = _u8(self.masks)
        B = int(z.shape[0])
        act = torch.empty((B, self.map_size, self._spec.G), dtype=torch.int64, device=z.device)
        logp = torch.empty(B, dtype=torch.float32, device=z.device)
        nv, sr, sv = self._spec.ptrs()
        rc = _lib.lib().rai_gridnet_sample(z.data_ptr(), m.data_ptr(), B, self.map_size, self._spec.G, nv, sr, sv,
                                           int(seed), int(offset), act.data_ptr(), logp.data_ptr(),
                                           _lib.stream_handle(z.device))
        _lib.check(rc, "rai_gridnet_sample")
        return act, logp

    def sample(self, sample_shape=torch.Size()) -> torch.Tensor:
        outs = [torch.distributions.Categorical(logits=zm).sample(sample_shape) for zm in self._groups()]
        return torch.stack(outs, dim=-1).view(-1, self.map_size, len(self.action_vec))

    @property
    def mode(self) -> torch.Tensor:
        return torch.stack([zm.argmax(-1) for zm in self._groups()], dim=-1).view(-1, self.map_size,
                                                                                 len(self.action_vec))
