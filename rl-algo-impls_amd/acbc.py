"""ACBC on MI355X — drop-in for rl_algo_impls/acbc/acbc.py:29-165 (Actor-Critic Behavior Cloning
with critic bootstrapping).

The third algorithm over the same hot path: the device rollout with its GAE returns
(rai_gae; the critic regresses onto the bootstrapped returns = advantages + values,
rl_algo_impls/rollout/vec_rollout.py:78-88), minibatches of the HBM rollout, one fused loss
launch and the fused clip_grad_norm_ + Adam.  Per minibatch (acbc.py:94-128):

    pi_loss = -mean(logp(a))                         (or of logp / num_actions, scale_loss_by_num_actions)
    v_loss  = mean((v - R)^2) per value column
    loss    = pi_loss + sum(vf_coef * v_loss)        (/ num_minibatches under gradient accumulation)

which is rai_ppo_loss in its A2C mode (loss_kind 1: pi_loss = -mean(A * logp)) with a unit
advantage and no entropy term.  Adam keeps torch's default eps = 1e-8 (acbc.py:51).
"""
from __future__ import annotations

import logging
from time import perf_counter
from typing import Dict, List, Optional

import numpy as np
import torch

from .optim import FlatOptimizer, FlatParams
from .pg_common import (DeviceBlocks, launch_loss, load_optimizer, log_scalars, make_hparams, num_or_array,
                        save_optimizer, scale_logp_by_num_actions, unsupported, value_columns)


class ACBCTrainStats:
    """rl_algo_impls/acbc/train_stats.py: means of the last epoch's per-step stats + explained_var."""

    def __init__(self, step_stats: Dict[str, object], explained_var: float):
        self.step_stats = step_stats
        self.explained_var = explained_var

    def write_to_tensorboard(self, tb_writer) -> None:
        if tb_writer is None:
            return
        stats = {**self.step_stats, "explained_var": self.explained_var}
        for name, value in stats.items():
            if isinstance(value, np.ndarray):
                for idx, v in enumerate(value.flatten()):
                    tb_writer.add_scalar(f"losses/{name}_{idx}", v)
            else:
                tb_writer.add_scalar(f"losses/{name}", value)


class ACBC:
    def __init__(self, policy, device: torch.device, tb_writer, learning_rate: float = 3e-4, batch_size: int = 64,
                 n_epochs: int = 10, gamma=0.99, gae_lambda=0.95, vf_coef=0.25, max_grad_norm: float = 0.5,
                 gradient_accumulation: bool = False, scale_loss_by_num_actions: bool = False):
        self.scale_loss_by_num_actions = scale_loss_by_num_actions
        self.policy = policy
        self.device = torch.device(device)
        self.tb_writer = tb_writer
        self.learning_rate = learning_rate
        cl = policy.channels_last_params() if self.device.type == "cuda" and hasattr(policy, "channels_last_params") else ()
        self.flat = FlatParams(policy, self.device, channels_last=cl)
        self.optimizer = FlatOptimizer(self.flat, FlatOptimizer.ADAM, lr=learning_rate, eps=1e-8,
                                       max_grad_norm=max_grad_norm)
        self.batch_size = batch_size
        self.n_epochs = n_epochs
        self.gamma = num_or_array(gamma)
        self.gae_lambda = num_or_array(gae_lambda)
        self.vf_coef = num_or_array(vf_coef)
        self.max_grad_norm = max_grad_norm
        self.gradient_accumulation = gradient_accumulation
        self.blocks = DeviceBlocks(self.device)
        self._unit_adv: Dict[tuple, torch.Tensor] = {}

    def _unit_advantage(self, B: int, K: int) -> torch.Tensor:
        """(B, K) with column 0 = 1: the A2C-mode loss's advantage sum over columns is then 1."""
        t = self._unit_adv.get((B, K))
        if t is None:
            t = torch.zeros((B, K) if K > 1 else (B,), dtype=torch.float32, device=self.device)
            (t[:, 0] if K > 1 else t).fill_(1.0)
            self._unit_adv[(B, K)] = t
        return t

    def learn(self, train_timesteps: int, rollout_generator, callbacks=None, total_timesteps: Optional[int] = None,
              start_timesteps: int = 0) -> "ACBC":
        if total_timesteps is None:
            total_timesteps = train_timesteps
        assert start_timesteps + train_timesteps <= total_timesteps
        timesteps_elapsed = start_timesteps
        while timesteps_elapsed < start_timesteps + train_timesteps:
            start_time = perf_counter()
            self.optimizer.param_groups[0]["lr"] = self.learning_rate  # update_learning_rate
            self.optimizer.max_grad_norm = self.max_grad_norm
            self.optimizer.sync_hparams()
            log_scalars(self.tb_writer, "charts", {"learning_rate": self.learning_rate, "vf_coef": self.vf_coef},
                        timesteps_elapsed)
            r = rollout_generator.rollout(self.gamma, self.gae_lambda)
            timesteps_elapsed += r.total_steps
            train_stats = self._update(r)
            train_stats.write_to_tensorboard(self.tb_writer)
            self.last_train_stats = train_stats
            end_time = perf_counter()
            if self.tb_writer is not None:
                self.tb_writer.add_scalar("train/steps_per_second", r.total_steps / (end_time - start_time))
                if hasattr(self.tb_writer, "on_steps"):
                    self.tb_writer.on_steps(r.total_steps)
            if callbacks and not all(c.on_step(timesteps_elapsed=r.total_steps) for c in callbacks):
                logging.info(f"Callback terminated training at {timesteps_elapsed} timesteps")
                break
        return self

    def _update(self, r) -> ACBCTrainStats:
        """Every epoch x minibatch of one rollout, enqueued without host syncs (acbc.py:91-132)."""
        nmb = r.num_minibatches(self.batch_size)
        n_steps = self.n_epochs * nmb
        blocks = self.blocks
        blocks.ensure_tables(n_steps, self.n_epochs if self.gradient_accumulation else n_steps)
        K = None
        for _ in range(self.n_epochs):
            for mb in r.minibatches(self.batch_size, shuffle=not self.gradient_accumulation):
                logp, ent, v = self.policy(mb.obs, mb.actions, action_masks=mb.action_masks)
                if self.scale_loss_by_num_actions:  # acbc.py:114-117
                    logp = scale_logp_by_num_actions(logp, mb.num_actions)
                if K is None:
                    K = value_columns(v)
                    hp = make_hparams(loss_kind=1, K=K, ent_coef=0.0, vf_coef=self.vf_coef,
                                      normalize_advantage=False,
                                      grad_scale=(1.0 / nmb) if self.gradient_accumulation else 1.0)
                    blocks.upload(hp, self.optimizer.step_count)
                B = int(logp.shape[0])
                d = launch_loss(blocks, logp, ent, v, None, None, self._unit_advantage(B, K), mb.returns, K)
                torch.autograd.backward([logp, ent, v], list(d))
                if not self.gradient_accumulation:
                    self.optimizer.step(blocks.state, blocks.norms)
            if self.gradient_accumulation:
                self.optimizer.step(blocks.state, blocks.norms)
        K = K or 1
        rows = blocks.stats[:n_steps].cpu().numpy().astype(np.float64)[-nmb:]  # last epoch (step_stats.clear())
        vl = rows[:, 5:5 + K]
        stats = {"loss": float(rows[:, 0].mean()), "pi_loss": float(rows[:, 1].mean()),
                 "v_loss": float(vl[:, 0].mean()) if K == 1 else vl.mean(0)}
        return ACBCTrainStats(stats, r.explained_variance())

    def save(self, path: str) -> None:
        save_optimizer(self.optimizer, path)

    def load(self, path: str) -> None:
        load_optimizer(self.optimizer, path, self.device)
