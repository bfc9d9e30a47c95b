"""ORACLE — test/benchmark infrastructure only.

CPU restatement ("port") of the reference trainer's hot path, used as bench.py's
`cpu_baseline` leg and pinned to the reference's own outputs by
tests/test_cpu_trainer.py (learn_epoch_cartpole.npz: a whole learn_epoch;
pong_steps.npz: NatureCNN minibatch steps).  It follows rl_algo_impls op for op on
the CPU, eagerly, like the reference does when run with device=cpu:
  rollout   rollout/sync_step_rollout.py:181-216 (numpy (T,N,...) buffers, one
            policy.step per env step: torch forward, Categorical sample, .numpy())
  GAE       shared/gae.py:97-124 (numpy reverse loop; oracle.compute_advantages)
  batch     rollout/vec_rollout.py:113-175 (flatten, torch.randperm, fancy-index gather)
  update    ppo/ppo.py:286-411 (normalise advantages, forward, clipped loss,
            backward, clip_grad_norm_(...).item(), Adam(eps=1e-7).step, zero_grad,
            the per-minibatch .item() stats), TrainStats means over the last epoch
            (ppo.py:36-99, 413-420)
  metric    ppo/ppo.py:221,422-427 (rollout steps / wall time of learn_epoch)
Policies: the reference's CartPole MLP (4 -> 64 -> 64 -> {2, 1}, tanh, separate actor
and critic) and its Atari NatureCNN actor-critic (shared/encoder/nature_cnn.py:10-53,
cnn.py:24-72, Categorical(6) head, critic), in the reference's parameters() order.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

import oracle


def _orthogonal(lin, gain):
    nn.init.orthogonal_(lin.weight, gain)
    nn.init.constant_(lin.bias, 0.0)
    return lin


class MLPActorCritic(nn.Module):
    def __init__(self, obs_dim=4, n_act=2, hidden=(64, 64)):
        super().__init__()

        def mlp(sizes, gain):
            layers = []
            for i in range(len(sizes) - 1):
                layers.append(_orthogonal(nn.Linear(sizes[i], sizes[i + 1]),
                                          np.sqrt(2) if i < len(sizes) - 2 else gain))
                if i < len(sizes) - 2:
                    layers.append(nn.Tanh())
            return nn.Sequential(*layers)

        self.pi = mlp((obs_dim,) + hidden + (n_act,), 0.01)
        self.v = mlp((obs_dim,) + hidden + (1,), 1.0)

    def logits_value(self, obs):
        return self.pi(obs), self.v(obs).squeeze(-1)

    def forward(self, obs, actions):
        logits, v = self.logits_value(obs)
        d = torch.distributions.Categorical(logits=logits)
        return d.log_prob(actions), d.entropy(), v


class NatureCnnActorCritic(nn.Module):
    """ConnectedTrio with a NatureCnn encoder (relu), actor Linear(512, n_act), critic
    Linear(512, 1): parameters() in the reference's order (cnn.{0,2,4}, fc.1, _pi, _v)."""

    def __init__(self, in_ch=4, n_act=6):
        super().__init__()
        self.range_size = 255.0  # np.max(high) - np.min(low) of Box(0, 255, uint8) (cnn.py:24)
        self.cnn = nn.Sequential(_orthogonal(nn.Conv2d(in_ch, 32, 8, stride=4), np.sqrt(2)), nn.ReLU(),
                                 _orthogonal(nn.Conv2d(32, 64, 4, stride=2), np.sqrt(2)), nn.ReLU(),
                                 _orthogonal(nn.Conv2d(64, 64, 3, stride=1), np.sqrt(2)), nn.ReLU())
        self.fc = nn.Sequential(nn.Flatten(), _orthogonal(nn.Linear(3136, 512), np.sqrt(2)), nn.ReLU())
        self.pi = _orthogonal(nn.Linear(512, n_act), 0.01)
        self.v = _orthogonal(nn.Linear(512, 1), 1.0)

    def logits_value(self, obs):
        h = self.fc(self.cnn(obs.float() / self.range_size))
        return self.pi(h), self.v(h).squeeze(-1)

    def forward(self, obs, actions):
        logits, v = self.logits_value(obs)
        d = torch.distributions.Categorical(logits=logits)
        return d.log_prob(actions), d.entropy(), v


def load_flat(module: nn.Module, flat: np.ndarray) -> None:
    off = 0
    with torch.no_grad():
        for p in module.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(np.asarray(flat[off:off + n])).reshape(p.shape))
            off += n
    assert off == len(flat), (off, len(flat))


def flat_params(module: nn.Module) -> np.ndarray:
    return torch.cat([p.detach().reshape(-1) for p in module.parameters()]).numpy().copy()


class CpuPPO:
    """The reference's PPO update on the CPU (ppo.py:286-420), for a policy whose forward
    returns (logp, entropy, v)."""

    def __init__(self, policy: nn.Module, lr=1e-3, batch_size=256, n_epochs=20, clip_range=0.2, ent_coef=0.0,
                 vf_coef=0.5, max_grad_norm=0.5):
        self.policy = policy
        self.bs, self.n_epochs = batch_size, n_epochs
        self.clip, self.ent_coef, self.vf_coef, self.max_grad_norm = clip_range, ent_coef, vf_coef, max_grad_norm
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=lr, eps=1e-7)

    def minibatch_step(self, mb_obs, mb_lp, mb_act, mb_val, mb_adv, mb_ret) -> tuple:
        mb_adv = (mb_adv - mb_adv.mean(0)) / (mb_adv.std(0) + 1e-8)
        new_lp, ent, new_v = self.policy(mb_obs, mb_act)
        logratio = new_lp - mb_lp
        ratio = torch.exp(logratio)
        clipped = torch.clamp(ratio, min=1 - self.clip, max=1 + self.clip)
        pi_loss = -torch.min(ratio * mb_adv, clipped * mb_adv).mean()
        v_loss = nn.functional.mse_loss(new_v, mb_ret, reduction="none").mean(0)
        entropy_loss = -ent.mean()
        with torch.no_grad():
            approx_kl = ((ratio - 1) - logratio).mean().cpu().numpy().item()
        loss = pi_loss + self.ent_coef * entropy_loss + (self.vf_coef * v_loss).sum()
        loss.backward()
        grad_norm = nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm).item()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        with torch.no_grad():
            clipped_frac = ((ratio - 1).abs() > self.clip).float().mean().cpu().numpy().item()
        return (loss.item(), pi_loss.item(), float(v_loss.detach().float().cpu().numpy()), entropy_loss.item(),
                approx_kl, clipped_frac, grad_norm)

    def update(self, b: Dict[str, torch.Tensor], perms: Optional[Sequence] = None, deadline: Optional[float] = None):
        """n_epochs over the flat batch b (obs, logprobs, actions, values, advantages, returns);
        perms[e] is epoch e's permutation (torch.randperm when None), minibatches are its slices
        of batch_size (the last one partial, vec_rollout.py:108-111,166-175).  Returns the per-step
        stat rows and the TrainStats means over the last epoch; stops early (means None) once
        time.perf_counter() passes `deadline`."""
        n = int(b["obs"].shape[0])
        rows: List[tuple] = []
        for e in range(self.n_epochs):
            perm = torch.as_tensor(perms[e]) if perms is not None else torch.randperm(n)
            for i in range(0, n, self.bs):
                idx = perm[i:i + self.bs]
                rows.append(self.minibatch_step(b["obs"][idx], b["logprobs"][idx], b["actions"][idx],
                                                b["values"][idx], b["advantages"][idx], b["returns"][idx]))
                if deadline is not None and time.perf_counter() > deadline:
                    return np.array(rows), None
        nmb = (n + self.bs - 1) // self.bs
        last = np.array(rows[-nmb:], np.float64)
        means = dict(zip(("loss", "pi_loss", "v_loss", "entropy_loss", "approx_kl", "clipped_frac", "grad_norm"),
                         last.mean(0)))
        return np.array(rows), means


def explained_variance(returns: np.ndarray, values: np.ndarray) -> float:
    """ppo.py:415-418 on the flattened rollout."""
    y, p = returns.reshape(-1), values.reshape(-1)
    var_y = np.var(y).item()
    return float("nan") if var_y == 0 else 1 - np.var(y - p).item() / var_y


class CpuCartPoleRun:
    """The C2 workload on the CPU: SyntheticVecEnv("cartpole")-shaped rollout with the
    reference's policy.step per env step, numpy GAE, then the update."""

    def __init__(self, num_envs=4096, n_steps=128, batch_size=256, n_epochs=20, lr=1e-3, gamma=0.98,
                 gae_lambda=0.8, clip_range=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, seed=1):
        torch.manual_seed(seed)
        self.rng = np.random.default_rng(seed)
        self.N, self.T = num_envs, n_steps
        self.gamma, self.gae_lambda = gamma, gae_lambda
        self.policy = MLPActorCritic()
        self.ppo = CpuPPO(self.policy, lr=lr, batch_size=batch_size, n_epochs=n_epochs, clip_range=clip_range,
                          ent_coef=ent_coef, vf_coef=vf_coef, max_grad_norm=max_grad_norm)
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
                logits, v = self.policy.logits_value(torch.as_tensor(self.next_obs))
                d = torch.distributions.Categorical(logits=logits)
                a = d.sample()
                lp = d.log_prob(a)
            values[s], logprobs[s], actions[s] = v.numpy(), lp.numpy(), a.numpy()
            self.next_obs, rewards[s], term, trunc = self._env_step(actions[s])
            self.next_starts = term | trunc
        with torch.no_grad():
            next_values = self.policy.logits_value(torch.as_tensor(self.next_obs))[1].numpy()
        return dict(obs=obs, rewards=rewards, starts=starts, values=values, logprobs=logprobs, actions=actions,
                    next_values=next_values, next_starts=self.next_starts.copy())

    def batch(self, r):
        adv = oracle.compute_advantages(r["rewards"], r["values"], r["starts"], r["next_starts"], r["next_values"],
                                        self.gamma, self.gae_lambda)
        ret = adv + r["values"]
        fl = lambda a: torch.as_tensor(a.reshape((-1,) + a.shape[2:]))
        return dict(obs=fl(r["obs"]), logprobs=fl(r["logprobs"]), actions=fl(r["actions"]), values=fl(r["values"]),
                    advantages=fl(adv), returns=fl(ret))


def time_update(budget_seconds: Optional[float] = 15.0, **kw) -> Dict:
    """One learn_epoch of the C2 workload on the CPU: the full rollout, GAE and batch prep,
    then the update's minibatch steps — all of them when budget_seconds is None, else as many
    as fit in budget_seconds with the update time extrapolated to all n_epochs x minibatches."""
    t = CpuCartPoleRun(**kw)
    t0 = time.perf_counter()
    r = t.rollout()
    t1 = time.perf_counter()
    b = t.batch(r)
    t2 = time.perf_counter()
    n = t.N * t.T
    steps_total = ((n + t.ppo.bs - 1) // t.ppo.bs) * t.ppo.n_epochs
    if budget_seconds is None:
        t.ppo.update(b)
        done = steps_total
    else:
        t3 = time.perf_counter()
        rows, _ = t.ppo.update(b, deadline=t3 + budget_seconds)  # bounded sample of the same steps
        done = len(rows)
        per_step = (time.perf_counter() - t3) / done
        update_s = (t1 - t0) + (t2 - t1) + per_step * steps_total
        return dict(env_steps_per_s=n / update_s, rollout_s=t1 - t0, gae_s=t2 - t1, minibatch_s=per_step,
                    minibatches_timed=done, minibatches_total=steps_total, update_s=update_s, extrapolated=True,
                    threads=torch.get_num_threads())
    t4 = time.perf_counter()
    return dict(env_steps_per_s=n / (t4 - t0), rollout_s=t1 - t0, gae_s=t2 - t1, minibatch_s=(t4 - t2) / done,
                minibatches_timed=done, minibatches_total=steps_total, update_s=t4 - t0, extrapolated=False,
                threads=torch.get_num_threads())


def time_sampled_update(budget_seconds: float = 15.0, **kw) -> Dict:
    """Backward-compatible name for the bounded-sample timing."""
    return time_update(budget_seconds, **kw)
