"""ORACLE — test/benchmark infrastructure only.

CPU restatement ("port") of the reference trainer's hot path, used as bench.py's
`cpu_baseline` leg.  It follows rl_algo_impls op for op on the CPU, eagerly, like
the reference does when run with device=cpu:
  rollout   rollout/sync_step_rollout.py:181-216 (numpy (T,N,...) buffers, one
            policy.step per env step: torch forward, Categorical sample, .numpy())
  GAE       shared/gae.py:97-124 (numpy reverse loop; oracle.compute_advantages)
  batch     rollout/vec_rollout.py:113-175 (flatten, torch.randperm, fancy-index gather)
  update    ppo/ppo.py:286-411 (normalise advantages, forward, clipped loss,
            backward, clip_grad_norm_(...).item(), Adam(eps=1e-7).step, zero_grad,
            the per-minibatch .item() stats)
  metric    ppo/ppo.py:221,422-427 (rollout steps / wall time of learn_epoch)
The policy is a self-contained torch MLP with the reference's CartPole shape
(4 -> 64 -> 64 -> {2, 1}, tanh, separate actor/critic MLPs).
"""
from __future__ import annotations

import time
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

import oracle


class MLPActorCritic(nn.Module):
    def __init__(self, obs_dim=4, n_act=2, hidden=(64, 64)):
        super().__init__()

        def mlp(sizes, gain):
            layers = []
            for i in range(len(sizes) - 1):
                lin = nn.Linear(sizes[i], sizes[i + 1])
                nn.init.orthogonal_(lin.weight, np.sqrt(2) if i < len(sizes) - 2 else gain)
                nn.init.constant_(lin.bias, 0.0)
                layers.append(lin)
                if i < len(sizes) - 2:
                    layers.append(nn.Tanh())
            return nn.Sequential(*layers)

        self.pi = mlp((obs_dim,) + hidden + (n_act,), 0.01)
        self.v = mlp((obs_dim,) + hidden + (1,), 1.0)

    def forward(self, obs, actions):
        d = torch.distributions.Categorical(logits=self.pi(obs))
        return d.log_prob(actions), d.entropy(), self.v(obs).squeeze(-1)


class CpuPPO:
    def __init__(self, num_envs=4096, n_steps=128, batch_size=256, n_epochs=20, lr=1e-3, gamma=0.98,
                 gae_lambda=0.8, clip_range=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, seed=1):
        torch.manual_seed(seed)
        self.rng = np.random.default_rng(seed)
        self.N, self.T = num_envs, n_steps
        self.bs, self.n_epochs = batch_size, n_epochs
        self.gamma, self.gae_lambda = gamma, gae_lambda
        self.clip, self.ent_coef, self.vf_coef, self.max_grad_norm = clip_range, ent_coef, vf_coef, max_grad_norm
        self.policy = MLPActorCritic()
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=lr, eps=1e-7)
        self.next_obs = self.rng.standard_normal((self.N, 4), dtype=np.float32)
        self.next_starts = np.ones(self.N, dtype=np.bool_)

    def _env_step(self, actions):  # SyntheticVecEnv("cartpole") dynamics
        obs = self.rng.standard_normal((self.N, 4), dtype=np.float32)
        term = self.rng.random(self.N) < 1 / 200
        return obs, np.ones(self.N, np.float32), term, np.zeros(self.N, np.bool_)

    def rollout(self):
        T, N = self.T, self.N
        obs = np.zeros((T, N, 4), np.float32)
        rewards = np.zeros((T, N), np.float32)
        starts = np.zeros((T, N), np.bool_)
        values = np.zeros((T, N), np.float32)
        logprobs = np.zeros((T, N), np.float32)
        actions = np.zeros((T, N), np.int64)
        for s in range(T):
            obs[s] = self.next_obs
            starts[s] = self.next_starts
            with torch.no_grad():
                o = torch.as_tensor(self.next_obs)
                d = torch.distributions.Categorical(logits=self.policy.pi(o))
                a = d.sample()
                lp = d.log_prob(a)
                v = self.policy.v(o).squeeze(-1)
            values[s], logprobs[s], actions[s] = v.numpy(), lp.numpy(), a.numpy()
            self.next_obs, rewards[s], term, trunc = self._env_step(actions[s])
            self.next_starts = term | trunc
        with torch.no_grad():
            next_values = self.policy.v(torch.as_tensor(self.next_obs)).squeeze(-1).numpy()
        return dict(obs=obs, rewards=rewards, starts=starts, values=values, logprobs=logprobs, actions=actions,
                    next_values=next_values, next_starts=self.next_starts.copy())

    def minibatch_step(self, b_obs, b_lp, b_act, b_val, b_adv, b_ret, idx) -> float:
        mb_obs, mb_lp, mb_act = b_obs[idx], b_lp[idx], b_act[idx]
        mb_val, mb_adv, mb_ret = b_val[idx], b_adv[idx], b_ret[idx]
        mb_adv = (mb_adv - mb_adv.mean(0)) / (mb_adv.std(0) + 1e-8)
        new_lp, ent, new_v = self.policy(mb_obs, mb_act)
        logratio = new_lp - mb_lp
        ratio = torch.exp(logratio)
        clipped = torch.clamp(ratio, 1 - self.clip, 1 + self.clip)
        pi_loss = -torch.min(ratio * mb_adv, clipped * mb_adv).mean()
        v_loss = nn.functional.mse_loss(new_v, mb_ret, reduction="none").mean(0)
        entropy_loss = -ent.mean()
        with torch.no_grad():
            approx_kl = ((ratio - 1) - logratio).mean().cpu().numpy().item()
        loss = pi_loss + self.ent_coef * entropy_loss + self.vf_coef * v_loss
        loss.backward()
        grad_norm = nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm).item()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        with torch.no_grad():
            clipped_frac = ((ratio - 1).abs() > self.clip).float().mean().cpu().numpy().item()
        _ = (loss.item(), pi_loss.item(), v_loss.detach().float().cpu().numpy(), entropy_loss.item(), approx_kl,
             clipped_frac, grad_norm)
        return grad_norm


def time_sampled_update(budget_seconds: float = 15.0, **kw) -> Dict:
    """Time one full rollout + GAE + batch prep, then as many minibatch steps as fit in
    `budget_seconds`; extrapolate the update time to all n_epochs*num_minibatches steps."""
    t = CpuPPO(**kw)
    t0 = time.perf_counter()
    r = t.rollout()
    t1 = time.perf_counter()
    adv = oracle.compute_advantages(r["rewards"], r["values"], r["starts"], r["next_starts"], r["next_values"],
                                    t.gamma, t.gae_lambda)
    ret = adv + r["values"]
    t2 = time.perf_counter()
    fl = lambda a: torch.as_tensor(a.reshape((-1,) + a.shape[2:]))
    b_obs, b_lp, b_act, b_val, b_adv, b_ret = (fl(r["obs"]), fl(r["logprobs"]), fl(r["actions"]), fl(r["values"]),
                                               fl(adv), fl(ret))
    total = t.N * t.T
    n_mb = total // t.bs + (1 if total % t.bs else 0)
    n_steps_total = n_mb * t.n_epochs
    done = 0
    t3 = time.perf_counter()
    perm = torch.randperm(total)
    while done < n_steps_total:
        i = done % n_mb
        if i == 0 and done:
            perm = torch.randperm(total)
        t.minibatch_step(b_obs, b_lp, b_act, b_val, b_adv, b_ret, perm[i * t.bs:(i + 1) * t.bs])
        done += 1
        if time.perf_counter() - t3 > budget_seconds:
            break
    t4 = time.perf_counter()
    per_step = (t4 - t3) / done
    update_s = (t1 - t0) + (t2 - t1) + per_step * n_steps_total
    return dict(env_steps_per_s=total / update_s, rollout_s=t1 - t0, gae_s=t2 - t1, minibatch_s=per_step,
                minibatches_timed=done, minibatches_total=n_steps_total, update_s_extrapolated=update_s,
                threads=torch.get_num_threads())
