"""Shared machinery for the PPO / A2C updates: device-resident hyperparameter and
train-state blocks, the fused loss launch, and the one-per-update stats read-back.

The reference performs ~6 host syncs per minibatch (`.item()`, `.cpu()` in
rl_algo_impls/ppo/ppo.py:353,380-409,442-444).  Here every per-minibatch scalar
(loss terms, approx_kl, clip fractions, grad norm) is written by the kernels into
HBM tables and read back ONCE per update.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from . import _lib
from .optim import struct_to_device

OPTIMIZER_FILENAME = "optimizer.pt"
VF_LOSS_FNS = {"mse_loss": 0, "huber_loss": 1, "smooth_l1_loss": 2}


def num_or_array(x):  # rl_algo_impls/shared/tensor_utils.py:38-41
    if isinstance(x, list):
        return np.array(x)
    return x


def log_scalars(tb_writer, main_tag: str, d: Dict, global_step: int = 0) -> None:  # shared/stats.py:213-224
    if tb_writer is None:
        return
    for tag, value in d.items():
        if isinstance(value, np.ndarray):
            for i, v in enumerate(value.flatten()):
                tb_writer.add_scalar(f"{main_tag}/{tag}_{i}", v)
        else:
            tb_writer.add_scalar(f"{main_tag}/{tag}", value)


@dataclass
class TrainStats:  # rl_algo_impls/ppo/ppo.py:36-99
    loss: float
    pi_loss: float
    v_loss: Union[float, np.ndarray]
    entropy_loss: float
    approx_kl: float
    clipped_frac: float
    val_clipped_frac: Union[float, np.ndarray]
    additional_losses: Dict[str, float]
    explained_var: float
    grad_norm: float

    def write_to_tensorboard(self, tb_writer) -> None:
        if tb_writer is None:
            return
        for name, value in asdict(self).items():
            if isinstance(value, np.ndarray):
                for idx, v in enumerate(value.flatten()):
                    tb_writer.add_scalar(f"losses/{name}_{idx}", v)
            elif isinstance(value, dict):
                for k, v in value.items():
                    tb_writer.add_scalar(f"losses/{k}", v)
            else:
                tb_writer.add_scalar(f"losses/{name}", value)


class DeviceBlocks:
    """HBM copies of rai_ppo_hparams and rai_train_state + the stats/norm tables."""

    def __init__(self, device: torch.device):
        self.device = device
        self.hp = torch.empty(C.sizeof(_lib.PPOHparams), dtype=torch.uint8, device=device)
        self.state = torch.empty(C.sizeof(_lib.TrainState), dtype=torch.uint8, device=device)
        self.stats = torch.zeros((1, _lib.RAI_STAT_STRIDE), dtype=torch.float32, device=device)
        self.norms = torch.zeros((1,), dtype=torch.float32, device=device)
        self._grads: Dict = {}

    def ensure_tables(self, n_stats: int, n_norms: int) -> None:
        if self.stats.shape[0] < n_stats:
            self.stats = torch.zeros((n_stats, _lib.RAI_STAT_STRIDE), dtype=torch.float32, device=self.device)
        if self.norms.shape[0] < n_norms:
            self.norms = torch.zeros((n_norms,), dtype=torch.float32, device=self.device)

    def upload(self, hp: _lib.PPOHparams, opt_step: int) -> None:
        struct_to_device(hp, self.device, self.hp)
        struct_to_device(_lib.TrainState(opt_step=opt_step, stat_index=0, pi_coef_zero=0, norm_index=0),
                         self.device, self.state)

    def grad_buffers(self, logp: torch.Tensor, ent: torch.Tensor, v: torch.Tensor):
        key = (tuple(logp.shape), tuple(ent.shape), tuple(v.shape))
        bufs = self._grads.get(key)
        if bufs is None:
            bufs = (torch.empty_like(logp), torch.empty_like(ent), torch.empty_like(v))
            self._grads[key] = bufs
        return bufs


def make_hparams(*, loss_kind: int, K: int, clip_range=0.2, clip_range_vf=None, ent_coef=0.0, vf_coef=0.5,
                 vf_weights=None, multi_reward_weights=None, normalize_advantage=True,
                 standardize_advantage=False, normalize_after_scaling=False, ppo2_vf_coef_halving=False,
                 kl_cutoff=None, vf_loss_fn="mse_loss", grad_scale=1.0) -> _lib.PPOHparams:
    if K > _lib.RAI_MAX_K:
        raise NotImplementedError(f"K={K} exceeds RAI_MAX_K")
    if vf_loss_fn not in VF_LOSS_FNS:
        raise NotImplementedError(f"vf_loss_fn={vf_loss_fn}")
    hp = _lib.PPOHparams()
    hp.clip_range = float(clip_range)
    hp.has_clip_range_vf = int(clip_range_vf is not None)
    hp.clip_range_vf = float(clip_range_vf) if clip_range_vf is not None else 0.0
    hp.ent_coef = float(ent_coef)
    hp.has_kl_cutoff = int(kl_cutoff is not None)
    hp.kl_cutoff = float(kl_cutoff) if kl_cutoff is not None else 0.0
    hp.grad_scale = float(grad_scale)
    hp.K = K
    hp.normalize_advantage = int(bool(normalize_advantage))
    hp.standardize_advantage = int(bool(standardize_advantage))
    hp.normalize_after_scaling = int(bool(normalize_after_scaling))
    hp.ppo2_vf_coef_halving = int(bool(ppo2_vf_coef_halving))
    hp.vf_loss_fn = VF_LOSS_FNS[vf_loss_fn]
    hp.loss_kind = loss_kind
    vf = np.asarray(vf_coef, dtype=np.float64)
    if vf_weights is not None:
        w = np.asarray(vf_weights, np.float32).reshape(-1)
        assert w.shape[0] == K, f"vf_weights {w.shape} must match K={K}"
        eff = np.float32(vf.sum()) * w  # (vf_coef * (l @ w).mean()).sum()  (ppo.py:344-360)
        hp.has_vf_weights = 1
        for k in range(K):
            hp.vf_weights[k] = float(w[k])
    else:
        eff = np.broadcast_to(vf.astype(np.float32), (K,))
    for k in range(K):
        hp.vf_coef[k] = float(eff[k])
    if multi_reward_weights is not None:
        mrw = np.asarray(multi_reward_weights, np.float32).reshape(-1)
        assert mrw.shape[0] == K, f"multi_reward_weights {mrw.shape} must match K={K}"
        hp.has_multi_reward_weights = 1
        for k in range(K):
            hp.multi_reward_weights[k] = float(mrw[k])
    elif K > 1:
        raise ValueError("K>1 value columns need multi_reward_weights (ppo.py:317-329 broadcasting)")
    return hp


def launch_loss(blocks: DeviceBlocks, logp, ent, v, old_logp, old_values, adv, ret, K: int):
    d_logp, d_ent, d_v = blocks.grad_buffers(logp, ent, v)
    B = int(logp.shape[0])
    logp_c, ent_c, v_c = logp.detach().contiguous(), ent.detach().contiguous(), v.detach().contiguous()
    rc = _lib.lib().rai_ppo_loss(
        logp_c.data_ptr(), ent_c.data_ptr(), ent_c.numel(), v_c.data_ptr(),
        None if old_logp is None else old_logp.contiguous().data_ptr(),
        None if old_values is None else old_values.contiguous().data_ptr(),
        adv.contiguous().data_ptr(), ret.contiguous().data_ptr(), B, K, blocks.hp.data_ptr(),
        blocks.state.data_ptr(), d_logp.data_ptr(), d_ent.data_ptr(), d_v.data_ptr(), blocks.stats.data_ptr(),
        int(blocks.stats.shape[0]), None, 0, _lib.stream_handle(logp.device))
    _lib.check(rc, "rai_ppo_loss")
    return d_logp, d_ent, d_v


def scale_logp_by_num_actions(logp: torch.Tensor, num_actions: Optional[torch.Tensor]) -> torch.Tensor:
    """scale_loss_by_num_actions (rl_algo_impls/a2c/a2c.py:144-147, rl_algo_impls/acbc/acbc.py:114-117): the
    policy term uses logp / num_actions where num_actions > 0, else 0 -- the reference's expression, on the
    device, differentiated by autograd (the loss kernel then sees the scaled log-probabilities).  The
    rollout's Batch.num_actions exists for action-masked (GridNet) rollouts only."""
    if num_actions is None:
        raise ValueError("scale_loss_by_num_actions needs Batch.num_actions (an action-masked GridNet rollout)")
    return torch.where(num_actions > 0, logp / num_actions, 0)


def value_columns(v: torch.Tensor) -> int:
    return 1 if v.dim() == 1 else int(v.shape[1])


def unsupported(**kw) -> None:
    bad = [k for k, v in kw.items() if v]
    if bad:
        raise NotImplementedError(f"options outside the PPO/A2C hot-path scope: {bad}")


def save_optimizer(optimizer, path: str) -> None:
    torch.save(optimizer.state_dict(), os.path.join(path, OPTIMIZER_FILENAME))


def load_optimizer(optimizer, path: str, device) -> None:
    p = os.path.join(path, OPTIMIZER_FILENAME)
    if os.path.exists(p):
        optimizer.load_state_dict(torch.load(p, map_location=device, weights_only=True))
