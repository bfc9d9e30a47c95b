"""A2C on MI355X — drop-in for rl_algo_impls/a2c/a2c.py:24-205.

Same rollout path as PPO; the fused loss kernel runs in A2C mode
(pi_loss = -mean(A * logp), value MSE, entropy; a2c.py:132-158) and the fused
optimizer step runs RMSprop(alpha=0.99, eps=rms_prop_eps) or Adam.
"""
from __future__ import annotations

import logging
from time import perf_counter
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from .optim import FlatOptimizer, FlatParams
from .pg_common import (DeviceBlocks, launch_loss, load_optimizer, log_scalars, make_hparams, num_or_array,
                        save_optimizer, scale_logp_by_num_actions, unsupported, value_columns)


class A2CTrainStats:  # rl_algo_impls/a2c/train_stats.py
    def __init__(self, data):
        self.data = data

    def write_to_tensorboard(self, tb_writer) -> None:
        if tb_writer is None:
            return
        for name, value in self.data.items():
            if isinstance(value, np.ndarray):
                for i, v in enumerate(value.flatten()):
                    tb_writer.add_scalar(f"losses/{name}_{i}", v)
            else:
                tb_writer.add_scalar(f"losses/{name}", value)


class A2C:
    def __init__(self, policy, device: torch.device, tb_writer, learning_rate: float = 7e-4, gamma=0.99,
                 gae_lambda=1.0, ent_coef: float = 0.0, vf_coef=0.5, max_grad_norm: float = 0.5,
                 rms_prop_eps: float = 1e-5, use_rms_prop: bool = True, normalize_advantage: bool = False,
                 multi_reward_weights: Optional[List[float]] = None, scale_loss_by_num_actions: bool = False,
                 gradient_accumulation: bool = False, autocast_loss: bool = False,
                 num_minibatches: Optional[int] = None):
        unsupported(autocast_loss=autocast_loss)
        self.scale_loss_by_num_actions = scale_loss_by_num_actions
        self.policy = policy
        self.device = torch.device(device)
        self.tb_writer = tb_writer
        self.learning_rate = learning_rate
        cl = policy.channels_last_params() if self.device.type == "cuda" and hasattr(policy, "channels_last_params") else ()
        self.flat = FlatParams(policy, self.device, channels_last=cl)
        if use_rms_prop:
            self.optimizer = FlatOptimizer(self.flat, FlatOptimizer.RMSPROP, lr=learning_rate, eps=rms_prop_eps,
                                           max_grad_norm=max_grad_norm)
        else:
            self.optimizer = FlatOptimizer(self.flat, FlatOptimizer.ADAM, lr=learning_rate, eps=1e-8,
                                           max_grad_norm=max_grad_norm)
        self.gamma = num_or_array(gamma)
        self.gae_lambda = num_or_array(gae_lambda)
        self.vf_coef = num_or_array(vf_coef)
        self.ent_coef = ent_coef
        self.max_grad_norm = max_grad_norm
        self.normalize_advantage = normalize_advantage
        self.multi_reward_weights = np.array(multi_reward_weights) if multi_reward_weights else None
        self.gradient_accumulation = gradient_accumulation
        self.num_minibatches = num_minibatches or 1
        assert self.num_minibatches == 1 or self.gradient_accumulation, (
            "A2C only supports single step batches. Therefore, non-1 minibatches must be gradient accumulated")
        self.blocks = DeviceBlocks(self.device)

    def learn(self, train_timesteps: int, rollout_generator, callbacks=None, total_timesteps=None,
              start_timesteps: int = 0) -> "A2C":
        if total_timesteps is None:
            total_timesteps = train_timesteps
        assert start_timesteps + train_timesteps <= total_timesteps
        timesteps_elapsed = start_timesteps
        while timesteps_elapsed < start_timesteps + train_timesteps:
            start_time = perf_counter()
            self.optimizer.param_groups[0]["lr"] = self.learning_rate
            self.optimizer.max_grad_norm = self.max_grad_norm
            self.optimizer.sync_hparams()
            chart = {"ent_coef": self.ent_coef, "learning_rate": self.learning_rate, "gamma": self.gamma,
                     "gae_lambda": self.gae_lambda, "vf_coef": self.vf_coef}
            if self.multi_reward_weights is not None:
                chart["reward_weights"] = self.multi_reward_weights
            log_scalars(self.tb_writer, "charts", chart, timesteps_elapsed)
            r = rollout_generator.rollout(gamma=self.gamma, gae_lambda=self.gae_lambda)
            timesteps_elapsed += r.total_steps
            nmb = self.num_minibatches
            blocks = self.blocks
            blocks.ensure_tables(nmb, nmb)
            K = None
            for mb in r.minibatches(r.total_steps // nmb, shuffle=not self.gradient_accumulation):
                logp, ent, v = self.policy(mb.obs, mb.actions, action_masks=mb.action_masks)
                if self.scale_loss_by_num_actions:  # a2c.py:144-147
                    logp = scale_logp_by_num_actions(logp, mb.num_actions)
                if K is None:
                    K = value_columns(v)
                    hp = make_hparams(loss_kind=1, K=K, ent_coef=self.ent_coef, vf_coef=self.vf_coef,
                                      multi_reward_weights=self.multi_reward_weights,
                                      normalize_advantage=self.normalize_advantage,
                                      grad_scale=(1.0 / nmb) if self.gradient_accumulation else 1.0)
                    blocks.upload(hp, self.optimizer.step_count)
                d = launch_loss(blocks, logp, ent, v, None, None, mb.advantages, mb.returns, K)
                torch.autograd.backward([logp, ent, v], list(d))
                if not self.gradient_accumulation:
                    self.optimizer.step(blocks.state, blocks.norms)
            if self.gradient_accumulation:
                self.optimizer.step(blocks.state, blocks.norms)
            rows = blocks.stats[:nmb].cpu().numpy().astype(np.float64)
            explained_var = r.explained_variance()
            end_time = perf_counter()
            if self.tb_writer is not None:
                self.tb_writer.add_scalar("train/steps_per_second", r.total_steps / (end_time - start_time))
            K = K or 1
            vl = rows[:, 5:5 + K].mean(0)
            stats = A2CTrainStats({"explained_var": explained_var, "loss": float(rows[:, 0].mean()),
                                   "pi_loss": float(rows[:, 1].mean()),
                                   "v_loss": float(vl[0]) if K == 1 else vl,
                                   "entropy_loss": float(rows[:, 2].mean())})
            stats.write_to_tensorboard(self.tb_writer)
            self.last_train_stats = stats
            if self.tb_writer is not None and hasattr(self.tb_writer, "on_steps"):
                self.tb_writer.on_steps(r.total_steps)
            if callbacks and not all(c.on_step(timesteps_elapsed=r.total_steps) for c in callbacks):
                logging.info(f"Callback terminated training at {timesteps_elapsed} timesteps")
                break
        return self

    def save(self, path: str) -> None:
        save_optimizer(self.optimizer, path)

    def load(self, path: str) -> None:
        load_optimizer(self.optimizer, path, self.device)
