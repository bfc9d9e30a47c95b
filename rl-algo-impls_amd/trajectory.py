"""Per-trajectory rollout builders with their advantages computed on the GPU.

Mirrors rl_algo_impls/rollout/trajectory.py (Trajectory, TrajectoryBuilder, batch_actions) and
rl_algo_impls/rollout/discrete_skips_trajectory_builder.py (DiscreteSkipsTrajectoryBuilder): the
builders accumulate host-side exactly as the reference's do (they sit beside the host env loop of
the guided rollouts, rl_algo_impls/rollout/guided_learner_rollout.py:73-176 and
random_guided_learner_rollout.py:99-227), and `trajectory()` returns the same Trajectory.

The advantage recurrence runs in the gfx950 kernels rai_gae_trajectories / rai_gae_skips
(csrc/gae_traj.hip).  `build_trajectories` computes a whole rollout's trajectories — all of them,
any lengths — in ONE launch per builder kind instead of one numpy loop per trajectory; the
single-builder `trajectory()` is the same call with one trajectory.  Bit-identical to the
reference in exact mode (tests/golden/traj_cases.npz).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, TypeVar, Union

import numpy as np
import torch

from . import _lib
from .gae import EXACT

NumOrArray = Union[float, np.ndarray]


@dataclass
class Trajectory:  # trajectory.py:9-19
    obs: np.ndarray
    values: np.ndarray
    advantages: np.ndarray
    logprobs: np.ndarray
    actions: Union[np.ndarray, Dict[str, np.ndarray]]
    action_masks: Optional[Union[np.ndarray, Dict[str, np.ndarray]]]

    def __len__(self) -> int:
        return len(self.obs)


ND = TypeVar("ND", np.ndarray, Dict[str, np.ndarray], None)


def batch_actions(actions: List[ND]) -> ND:  # trajectory.py:98-103
    if isinstance(actions[0], dict):
        return {k: np.array([a[k] for a in actions]) for k in actions[0]}
    if actions[0] is None:
        return None
    return np.array(actions)


class TrajectoryBuilder:  # trajectory.py:22-92
    def __init__(self) -> None:
        self.reset()

    def __len__(self) -> int:
        return len(self.obs)

    def add(self, obs, reward, done: bool, value, logprob, action, action_mask) -> None:
        self.obs.append(obs)
        self.rewards.append(reward)
        self.dones.append(done)
        self.values.append(value)
        self.logprobs.append(logprob)
        self.actions.append(action)
        self.action_masks.append(action_mask)

    def reset(self) -> None:
        self.obs, self.rewards, self.dones, self.values = [], [], [], []
        self.logprobs, self.actions, self.action_masks = [], [], []

    def trajectory(self, gamma: NumOrArray, gae_lambda: NumOrArray, next_values: Optional[np.ndarray] = None,
                   device=None) -> Trajectory:
        return build_trajectories([self], gamma, gae_lambda, [next_values], device=device)[0]


class DiscreteSkipsTrajectoryBuilder:  # discrete_skips_trajectory_builder.py:11-109
    def __init__(self) -> None:
        self.reset()

    def __len__(self) -> int:
        return len(self.obs)

    def reset(self) -> None:
        self.obs, self.rewards, self.values, self.logprobs = [], [], [], []
        self.actions, self.action_masks, self.steps_elapsed = [], [], []
        self.done = False

    def step_no_add(self, reward, done: bool, gamma: NumOrArray) -> None:
        assert not self.done, "Shouldn't be stepping a done trajectory"
        # the skipped step's reward is discounted into the last added step's reward (host side,
        # like the env loop that calls this)
        if self.rewards:
            self.rewards[-1] += reward * gamma ** self.steps_elapsed[-1]
        if self.steps_elapsed:
            self.steps_elapsed[-1] += 1
        self.done = done

    def step_add(self, obs, reward, done: bool, value, logprob, action, action_mask, gamma: NumOrArray) -> None:
        assert not self.done, "Shouldn't be adding to a done trajectory"
        self.obs.append(obs)
        self.values.append(value)
        self.logprobs.append(logprob)
        self.actions.append(action)
        self.action_masks.append(action_mask)
        self.rewards.append(np.zeros_like(reward))
        self.steps_elapsed.append(0)
        self.step_no_add(reward, done, gamma)

    def trajectory(self, gamma: NumOrArray, gae_lambda: NumOrArray, next_values: Optional[np.ndarray] = None,
                   device=None) -> Trajectory:
        return build_trajectories([self], gamma, gae_lambda, [next_values], device=device)[0]


def _f32_values(values: list) -> np.ndarray:
    v = np.array(values)
    if v.dtype != np.float32:
        raise ValueError(f"trajectory values must be float32 (policy outputs), got {v.dtype}")
    return v


def _columns(shape, gamma: NumOrArray, gae_lambda: NumOrArray):
    """Per-column fp64 gamma/lambda (prepend_dims_to_match, tensor_utils.py:25-31)."""
    K = int(np.prod(shape)) if shape else 1
    if len(shape) > 1:
        raise NotImplementedError("value shape must be () or (K,)")
    if K > _lib.RAI_MAX_K:
        raise NotImplementedError(f"K={K} value columns exceeds RAI_MAX_K={_lib.RAI_MAX_K}")
    vec = isinstance(gamma, np.ndarray)
    for x in (gamma, gae_lambda):
        if isinstance(x, np.ndarray):
            assert x.shape == tuple(shape)[-len(x.shape):], f"Array {x.shape} must match later dims of {shape}"
    g = np.ascontiguousarray(np.broadcast_to(np.asarray(gamma, np.float64), (K,)))
    lam = np.ascontiguousarray(np.broadcast_to(np.asarray(gae_lambda, np.float64), (K,)))
    return K, g, lam, vec


def build_trajectories(builders: Sequence[Union[TrajectoryBuilder, DiscreteSkipsTrajectoryBuilder]],
                       gamma: NumOrArray, gae_lambda: NumOrArray,
                       next_values: Optional[Sequence[Optional[np.ndarray]]] = None,
                       device=None, mode: int = EXACT) -> List[Trajectory]:
    """Trajectories of many builders (one kind) with one device launch for all advantages.
    next_values[i] follows the reference's per-builder `trajectory(..., next_values=...)`."""
    if not builders:
        return []
    kinds = {type(b) for b in builders}
    if len(kinds) != 1 or not kinds <= {TrajectoryBuilder, DiscreteSkipsTrajectoryBuilder}:
        raise TypeError("build_trajectories takes builders of one kind")
    skips = isinstance(builders[0], DiscreteSkipsTrajectoryBuilder)
    nvs = list(next_values) if next_values is not None else [None] * len(builders)
    assert len(nvs) == len(builders)
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

    rews, vals, lens = [], [], []
    for b, nv in zip(builders, nvs):
        assert len(b) > 0, "empty trajectory"
        if skips:
            assert b.done or nv is not None, "Need next_values if trajectory isn't done"
        rews.append(np.array(b.rewards, dtype=np.float32))
        vals.append(_f32_values(b.values))
        lens.append(len(b))
    vshape = vals[0].shape[1:]
    if any(v.shape[1:] != vshape for v in vals) or any(r.shape != v.shape for r, v in zip(rews, vals)):
        raise ValueError("all trajectories need the same value shape, rewards shaped like values")
    K, g, lam, vec = _columns(vshape, gamma, gae_lambda)
    n = len(builders)
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    rew = np.concatenate(rews).reshape(-1, K)
    val = np.concatenate(vals).reshape(-1, K)
    nv_arr = np.zeros((n, K), dtype=np.float32)
    for i, nv in enumerate(nvs):
        if nv is not None:
            nv_arr[i] = np.asarray(nv, dtype=np.float32).reshape(K)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_rew, d_val, d_off, d_nv = t(rew), t(val), t(offsets), t(nv_arr)
    d_adv = torch.empty_like(d_val)
    st = _lib.stream_handle(dev)
    L = _lib.lib()
    if not skips:
        dones = np.concatenate([np.asarray(b.dones, dtype=np.bool_) for b in builders]).astype(np.uint8)
        d_dones = t(dones)
        rc = L.rai_gae_trajectories(d_rew.data_ptr(), d_val.data_ptr(), d_dones.data_ptr(), d_off.data_ptr(), n, K,
                                    d_nv.data_ptr(), g.ctypes.data_as(C.POINTER(C.c_double)),
                                    lam.ctypes.data_as(C.POINTER(C.c_double)), int(vec), int(mode),
                                    d_adv.data_ptr(), None, st)
        _lib.check(rc, "rai_gae_trajectories")
    else:
        steps = np.concatenate([np.asarray(b.steps_elapsed, dtype=np.int32) for b in builders])
        if steps.min() < 0:
            raise ValueError("negative steps_elapsed")
        max_s = int(steps.max())
        # gamma ** s exactly as the reference evaluates `gamma ** steps_elapsed[t]` (numpy pow on an
        # np.int32 exponent), and (gamma ** s) * gae_lambda in the reference's order
        gam = np.asarray(gamma, np.float64) if vec else gamma
        gk = np.empty((max_s + 1, K), np.float64)
        gkl = np.empty((max_s + 1, K), np.float64)
        for s in range(max_s + 1):
            p = gam ** np.int32(s)
            gk[s] = p
            gkl[s] = p * gae_lambda
        done = np.array([b.done for b in builders], dtype=np.uint8)
        d_steps, d_gk, d_gkl, d_done = t(steps), t(gk), t(gkl), t(done)
        rc = L.rai_gae_skips(d_rew.data_ptr(), d_val.data_ptr(), d_steps.data_ptr(), d_off.data_ptr(), n, K,
                             d_nv.data_ptr(), d_done.data_ptr(), d_gk.data_ptr(), d_gkl.data_ptr(), max_s,
                             int(mode), d_adv.data_ptr(), None, st)
        _lib.check(rc, "rai_gae_skips")
    adv = d_adv.cpu().numpy()
    out = []
    for i, b in enumerate(builders):
        a = adv[offsets[i]:offsets[i + 1]].reshape(rews[i].shape)
        out.append(Trajectory(obs=np.array(b.obs), values=vals[i], advantages=a, logprobs=np.array(b.logprobs),
                              actions=batch_actions(b.actions), action_masks=batch_actions(b.action_masks)))
    return out
