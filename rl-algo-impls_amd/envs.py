"""Host-side environments behind the reference's gymnasium VectorEnv API
(rl_algo_impls/wrappers/vector_wrapper.py:16-20; rollout/sync_step_rollout.py:80-92,
202-209): reset() -> (obs, info); step(a) -> (obs, rew, term, trunc, info);
num_envs, single_observation_space, single_action_space.

Env stepping stays on the host CPU (north star).  Provided here:
  * minimal Box / Discrete spaces (gymnasium is not installed; real gymnasium
    spaces work too — the trainer duck-types on .n / .low / .shape),
  * SyntheticVecEnv: the seeded synthetic environments the benchmark and the
    golden fixtures use (SURVEY.md §8d "Synthetic inputs"),
  * CartPoleVecEnv: a vectorised CartPole-v1 restated from gymnasium's public
    dynamics, with same-step autoreset and RecordEpisodeStatistics-style
    episode returns, for return-parity runs.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()

    def sample(self, rng: Optional[np.random.Generator] = None):
        rng = rng or np.random.default_rng()
        if np.issubdtype(self.dtype, np.integer):
            return rng.integers(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(lo, hi, size=self.shape).astype(self.dtype)


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def sample(self, rng: Optional[np.random.Generator] = None):
        rng = rng or np.random.default_rng()
        return np.int64(rng.integers(self.n))


class MultiDiscrete:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(np.int64)

    def sample(self, rng: Optional[np.random.Generator] = None):
        rng = rng or np.random.default_rng()
        return rng.integers(0, self.nvec)


MICRORTS_NVEC = (6, 4, 4, 4, 4, 7, 49)  # MicroRTS per-cell action planes (78 logits)


def is_multidiscrete(space) -> bool:
    return hasattr(space, "nvec")


def is_discrete(space) -> bool:
    return hasattr(space, "n") and not hasattr(space, "nvec")


def is_box(space) -> bool:
    return hasattr(space, "low") and hasattr(space, "high")


class SyntheticVecEnv:
    """Seeded synthetic vector env with the shapes of the BASELINE configs.

    kind = "cartpole": obs ~ N(0,1) f32 (N,4), 2 actions, reward 1.0,
                       termination ~ Bernoulli(term_prob) (default 1/200)
    kind = "pong":     obs ~ U{0..255} u8 (N,4,84,84), 6 actions, reward ~ N(0,1),
                       termination ~ Bernoulli(1/1000)
    kind = "halfcheetah": obs ~ N(0,1) f32 (N,17), Box(6) actions in [-1,1],
                       reward ~ N(0,1), termination ~ Bernoulli(1/1000)
    kind = "microrts": obs ~ U{0,1} f32 (N,74,16,16) (CHW planes), GridNet actions
                       MultiDiscrete(tile(nvec, 256)) with action_plane_space
                       MultiDiscrete([6,4,4,4,4,7,49]), all-true action masks (N,256,78) from
                       get_action_mask(), K=3 rewards ~ N(0,1) (N,3), termination ~ Bernoulli(1/1000)
                       
    Truncations are always False (the reference treats them like terminations).

    Observation batches are drawn from a pool of `obs_pool` batches generated at construction
    (a uniformly chosen pool entry per step): the env's own cost would otherwise sit inside the
    timed rollout (numpy generates the 29 MB of uniform bytes of a 1024-env Pong step in ~45 ms,
    more than the whole device step) while saying nothing about the hot path.  Rewards and
    terminations are drawn fresh every step.  Returned observation arrays are shared with the
    pool: consumers copy them (the rollout stages them into pinned memory) and must not write.
    """

    def __init__(self, num_envs: int, kind: str = "cartpole", seed: int = 1,
                 term_prob: Optional[float] = None, obs_pool: Optional[int] = None):
        self.num_envs = int(num_envs)
        self.kind = kind
        self.rng = np.random.default_rng(seed)
        if kind == "cartpole":
            self.single_observation_space = Box(-np.inf, np.inf, (4,), np.float32)
            self.single_action_space = Discrete(2)
            self.term_prob = 1 / 200 if term_prob is None else term_prob
        elif kind == "pong":
            self.single_observation_space = Box(0, 255, (4, 84, 84), np.uint8)
            self.single_action_space = Discrete(6)
            self.term_prob = 1 / 1000 if term_prob is None else term_prob
        elif kind == "halfcheetah":
            self.single_observation_space = Box(-np.inf, np.inf, (17,), np.float32)
            self.single_action_space = Box(-1.0, 1.0, (6,), np.float32)
            self.term_prob = 1 / 1000 if term_prob is None else term_prob
        elif kind == "microrts":
            self.map_hw = (16, 16)
            cells = self.map_hw[0] * self.map_hw[1]
            self.single_observation_space = Box(0.0, 1.0, (74,) + self.map_hw, np.float32)
            self.action_plane_space = MultiDiscrete(MICRORTS_NVEC)
            self.single_action_space = MultiDiscrete(np.tile(MICRORTS_NVEC, cells))
            self.term_prob = 1 / 1000 if term_prob is None else term_prob
            self._mask = np.ones((self.num_envs, cells, int(sum(MICRORTS_NVEC))), dtype=np.bool_)
            self.get_action_mask = lambda: self._mask
        else:
            raise ValueError(f"unknown synthetic env kind {kind}")
        batch_bytes = self.num_envs * int(np.prod(self.single_observation_space.shape)) * \
            np.dtype(self.single_observation_space.dtype).itemsize
        if obs_pool is None:  # up to 16 batches within ~256 MB
            obs_pool = int(max(2, min(16, (256 << 20) // max(batch_bytes, 1))))
        self._pool = [self._draw_obs() for _ in range(int(obs_pool))]

    @property
    def unwrapped(self):
        return self

    def _obs(self) -> np.ndarray:
        return self._pool[int(self.rng.integers(len(self._pool)))]

    def _draw_obs(self) -> np.ndarray:
        N = self.num_envs
        shp = self.single_observation_space.shape
        if self.kind == "pong":
            return self.rng.integers(0, 256, size=(N,) + shp, dtype=np.uint8)
        if self.kind == "microrts":
            return (self.rng.random((N,) + shp, dtype=np.float32) < 0.5).astype(np.float32)
        return self.rng.standard_normal((N,) + shp, dtype=np.float32)

    def reset(self, **kwargs) -> Tuple[np.ndarray, Dict[str, Any]]:
        return self._obs(), {}

    def step(self, actions):
        N = self.num_envs
        obs = self._obs()
        if self.kind == "cartpole":
            rew = np.ones(N, dtype=np.float32)
        elif self.kind == "microrts":
            rew = self.rng.standard_normal((N, 3), dtype=np.float32)
        else:
            rew = self.rng.standard_normal(N, dtype=np.float32)
        term = self.rng.random(N) < self.term_prob
        trunc = np.zeros(N, dtype=np.bool_)
        return obs, rew, term, trunc, {}

    def close(self):
        pass


class CartPoleVecEnv:
    """Vectorised CartPole-v1 (gymnasium 0.29 public dynamics: Euler integration,
    tau=0.02, force 10, pole half-length 0.5, termination |x|>2.4 or
    |theta|>12deg, truncation at 500 steps, reward 1 per step, reset state
    ~ U(-0.05, 0.05)).  Same-step autoreset like gymnasium's vector envs; the
    finished episode's return/length arrive in info["episode"] with mask
    info["_episode"] (RecordEpisodeStatistics convention)."""

    gravity, masscart, masspole, length, force_mag, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    theta_threshold = 12 * 2 * np.pi / 360
    x_threshold = 2.4
    max_episode_steps = 500

    def __init__(self, num_envs: int, seed: int = 1):
        self.num_envs = int(num_envs)
        high = np.array([self.x_threshold * 2, np.finfo(np.float32).max,
                         self.theta_threshold * 2, np.finfo(np.float32).max], dtype=np.float32)
        self.single_observation_space = Box(-high, high, (4,), np.float32)
        self.single_action_space = Discrete(2)
        self.rngs = [np.random.default_rng(seed + i) for i in range(self.num_envs)]
        self.state = np.zeros((self.num_envs, 4), dtype=np.float64)
        self.steps = np.zeros(self.num_envs, dtype=np.int64)
        self.ep_return = np.zeros(self.num_envs, dtype=np.float64)

    @property
    def unwrapped(self):
        return self

    def _reset_idx(self, idx):
        for i in idx:
            self.state[i] = self.rngs[i].uniform(-0.05, 0.05, size=4)
        self.steps[idx] = 0
        self.ep_return[idx] = 0

    def reset(self, **kwargs):
        self._reset_idx(np.arange(self.num_envs))
        return self.state.astype(np.float32), {}

    def step(self, actions):
        a = np.asarray(actions).reshape(self.num_envs)
        x, x_dot, th, th_dot = self.state.T
        force = np.where(a == 1, self.force_mag, -self.force_mag)
        cos, sin = np.cos(th), np.sin(th)
        total_mass = self.masspole + self.masscart
        pml = self.masspole * self.length
        temp = (force + pml * th_dot ** 2 * sin) / total_mass
        th_acc = (self.gravity * sin - cos * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * cos ** 2 / total_mass))
        x_acc = temp - pml * th_acc * cos / total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * x_acc
        th = th + self.tau * th_dot
        th_dot = th_dot + self.tau * th_acc
        self.state = np.stack([x, x_dot, th, th_dot], axis=1)
        self.steps += 1
        term = (np.abs(x) > self.x_threshold) | (np.abs(th) > self.theta_threshold)
        trunc = (self.steps >= self.max_episode_steps) & ~term
        rew = np.ones(self.num_envs, dtype=np.float32)
        self.ep_return += 1.0
        done = term | trunc
        info: Dict[str, Any] = {}
        if done.any():
            idx = np.nonzero(done)[0]
            info["episode"] = {"r": np.where(done, self.ep_return, 0.0),
                               "l": np.where(done, self.steps, 0)}
            info["_episode"] = done.copy()
            self._reset_idx(idx)
        return self.state.astype(np.float32), rew, term, trunc, info

    def close(self):
        pass
