"""HBM-resident rollout buffer, GAE and minibatching behind the reference's
Rollout / RolloutGenerator / Batch contract.

Reference interfaces mirrored:
  Batch (field order, consumed positionally via astuple)   rl_algo_impls/rollout/rollout.py:23-72
  Rollout ABC (y_true, y_pred, total_steps, num_minibatches, minibatches, add_to_batch)
                                                            rl_algo_impls/rollout/rollout.py:78-103
  RolloutGenerator ABC (__init__(policy, vec_env, **kw), prepare, rollout)
                                                            rl_algo_impls/rollout/rollout.py:106-117
  SyncStepRolloutGenerator kwargs / loop                    rl_algo_impls/rollout/sync_step_rollout.py:14-216
  VecRollout (GAE, returns, minibatches)                    rl_algo_impls/rollout/vec_rollout.py:38-175

Design (MI355X-first): the (T, N, ...) buffers live in HBM for the whole update
(288 GB/GPU: the 3.7 GB Pong buffer fits with room for its permuted copy).  Per
env step the host obs go H2D into slot s, the policy head runs on the slot and a
fused HIP kernel samples the action and writes action / log-prob / value into the
slot; only the actions return to the host (the env steps there).  GAE and returns
run as one HIP reverse-scan over the resident buffers.  Each epoch's shuffle is a
single multi-field gather kernel into a permuted copy, after which every
minibatch is a contiguous slice (zero-copy views) instead of a fancy-index
gather per minibatch.
"""
from __future__ import annotations

import dataclasses
from abc import ABC, abstractmethod
from dataclasses import dataclass
from collections import deque
from typing import Callable, Deque, Dict, Iterator, List, Optional

import ctypes as C
import os
import weakref

import numpy as np
import torch

from . import _lib
from .envs import is_box, is_discrete
from .gae import EXACT, compute_advantages_device


@dataclass
class Batch:  # rollout.py:23-36 — field ORDER is part of the contract
    obs: torch.Tensor
    logprobs: Optional[torch.Tensor]
    actions: torch.Tensor
    action_masks: Optional[torch.Tensor]
    num_actions: Optional[torch.Tensor]
    values: torch.Tensor
    advantages: torch.Tensor
    returns: torch.Tensor
    additional: Dict[str, torch.Tensor] = dataclasses.field(default_factory=dict)

    @property
    def device(self) -> torch.device:
        return self.obs.device

    def to(self, device: torch.device) -> "Batch":
        if self.device == torch.device(device):
            return self
        mv = lambda t: None if t is None else t.to(device)
        return Batch(*(mv(getattr(self, f.name)) for f in dataclasses.fields(self)[:-1]),
                     {k: v.to(device) for k, v in self.additional.items()})

    def __getitem__(self, indices: torch.Tensor) -> "Batch":
        g = lambda t: None if t is None else t[indices]
        return Batch(self.obs[indices], g(self.logprobs), self.actions[indices], g(self.action_masks),
                     g(self.num_actions), self.values[indices], self.advantages[indices],
                     self.returns[indices], {k: v[indices] for k, v in self.additional.items()})

    def __len__(self) -> int:
        return self.obs.shape[0]


BatchMapFn = Callable[[Batch], Dict[str, torch.Tensor]]


class Rollout(ABC):
    @property
    @abstractmethod
    def y_true(self) -> np.ndarray: ...

    @property
    @abstractmethod
    def y_pred(self) -> np.ndarray: ...

    @property
    @abstractmethod
    def total_steps(self) -> int: ...

    @abstractmethod
    def num_minibatches(self, batch_size: int) -> int: ...

    @abstractmethod
    def minibatches(self, batch_size: int, shuffle: bool = True) -> Iterator[Batch]: ...

    def add_to_batch(self, map_fn: BatchMapFn, batch_size: int) -> None: ...


class RolloutGenerator(ABC):
    def __init__(self, policy, vec_env, **kwargs) -> None:
        super().__init__()
        self.policy = policy
        self.vec_env = vec_env

    def prepare(self) -> None:
        pass

    @abstractmethod
    def rollout(self, **kwargs) -> Rollout: ...


def _free_host_buffers(hosts: List[int]) -> None:
    for h in hosts:
        _lib.lib().rai_host_free(C.c_void_p(h))


def feistel_permutation(n: int, device: torch.device, key: Optional[int] = None) -> torch.Tensor:
    """The epoch shuffle: a keyed bijection of [0, n) computed on the device (rai_feistel_permutation;
    replaces torch.randperm(total_steps), rl_algo_impls/rollout/vec_rollout.py:166-170, whose device
    form is a radix sort).  The 64-bit key is drawn from torch's default CPU generator, so runs under
    torch.manual_seed repeat their shuffles."""
    if key is None:
        key = int(torch.randint(0, 2**63 - 1, (1,), dtype=torch.int64).item())
    out = torch.empty(n, dtype=torch.int64, device=device)
    rc = _lib.lib().rai_feistel_permutation(n, key & (2**64 - 1), out.data_ptr(), _lib.stream_handle(device))
    _lib.check(rc, "rai_feistel_permutation")
    return out


def gather_rows(srcs: List[torch.Tensor], dsts: List[torch.Tensor], idx: torch.Tensor) -> None:
    """dst_f[i] = src_f[idx[i]] for every field, one kernel launch (rai_gather_rows)."""
    n = len(srcs)
    assert 0 < n <= _lib.RAI_MAX_FIELDS and len(dsts) == n
    idx = idx.to(torch.int64).contiguous()
    rows = idx.shape[0]
    src_p = (C.c_void_p * n)(*[s.data_ptr() for s in srcs])
    dst_p = (C.c_void_p * n)(*[d.data_ptr() for d in dsts])
    rb = (C.c_int64 * n)(*[s[0].numel() * s.element_size() if s.shape[0] else 1 for s in srcs])
    for s, d in zip(srcs, dsts):
        assert s.is_contiguous() and d.is_contiguous() and s.dtype == d.dtype
        assert d.shape[0] >= rows and s.shape[1:] == d.shape[1:]
    rc = _lib.lib().rai_gather_rows(n, C.cast(src_p, C.c_void_p), C.cast(dst_p, C.c_void_p),
                                    C.cast(rb, C.c_void_p), idx.data_ptr(), rows,
                                    _lib.stream_handle(idx.device))
    _lib.check(rc, "rai_gather_rows")


def _num_actions(actions: torch.Tensor, action_masks: torch.Tensor, subaction_mask, action_plane_space):
    """rl_algo_impls/rollout/rollout.py:130-180 for per-position (GridNet) masks: (T, N) counts
    (gridnet.gridnet_num_actions).  subaction_mask is the YAML's {reference index: {index: value}}
    (ValueDependentMask.from_reference_index_to_index_to_value, vec_rollout.py:72-74)."""
    from .gridnet import ValueDependentMask, gridnet_num_actions

    if isinstance(action_masks, dict):
        raise NotImplementedError("pick_position (Lux) action masks are outside the hot path")
    if action_masks.dim() < 4:
        raise NotImplementedError("num_actions of flat (non-GridNet) action masks is outside the hot path")
    sub = ValueDependentMask.from_reference_index_to_index_to_value(subaction_mask) if subaction_mask else None
    if not sub:  # any over each cell's whole mask, the plane split unused (rollout.py:164-165)
        return gridnet_num_actions(None, action_masks, None, None)
    assert action_plane_space  # rollout.py:166
    return gridnet_num_actions(actions, action_masks, np.asarray(action_plane_space.nvec), sub)


class DeviceRollout(Rollout):
    """VecRollout equivalent over HBM-resident (T, N, ...) tensors."""

    def __init__(self, device: torch.device, next_episode_starts: torch.Tensor, next_values: torch.Tensor,
                 obs: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor,
                 episode_starts: torch.Tensor, values: torch.Tensor, logprobs: Optional[torch.Tensor],
                 action_masks: Optional[torch.Tensor], gamma, gae_lambda,
                 scale_advantage_by_values_accuracy: bool = False, gae_mode: int = EXACT,
                 perm_source: Optional[Callable[[int], torch.Tensor]] = None,
                 generator: Optional[torch.Generator] = None,
                 perm_keys: Optional[Callable[[], int]] = None,
                 subaction_mask: Optional[Dict[int, Dict[int, int]]] = None, action_plane_space=None) -> None:
        super().__init__()
        self.device = device
        self.obs, self.actions, self.rewards = obs, actions, rewards
        self.episode_starts, self.values, self.logprobs = episode_starts, values, logprobs
        self.action_masks = action_masks
        self.next_episode_starts, self.next_values = next_episode_starts, next_values
        self.num_actions = None
        if action_masks is not None:  # vec_rollout.py:69-76 -> rollout.py:130-180, one launch
            self.num_actions = _num_actions(actions, action_masks, subaction_mask, action_plane_space)
        self.advantages, self.returns = compute_advantages_device(
            rewards, values, episode_starts, next_episode_starts, next_values, gamma, gae_lambda,
            mode=gae_mode, want_returns=True)
        if scale_advantage_by_values_accuracy:  # vec_rollout.py:91-94
            ptp = self.returns.max() - self.returns.min()
            self.advantages *= torch.exp(-torch.abs(self.values - self.returns) / ptp)
        self._perm_source = perm_source
        self._generator = generator
        self._perm_keys = perm_keys
        self._flat: Optional[List[torch.Tensor]] = None
        self._perm_bufs: Dict[int, List[torch.Tensor]] = {}

    @classmethod
    def from_fields(cls, device: torch.device, obs: torch.Tensor, actions: torch.Tensor, values: torch.Tensor,
                    advantages: torch.Tensor, returns: torch.Tensor, logprobs: Optional[torch.Tensor],
                    action_masks: Optional[torch.Tensor] = None, num_actions: Optional[torch.Tensor] = None,
                    perm_keys: Optional[Callable[[], int]] = None,
                    perm_source: Optional[Callable[[int], torch.Tensor]] = None) -> "DeviceRollout":
        """A rollout over (T, N, ...) fields whose advantages / returns are already computed (GAE is
        independent per env column, so the column groups of several ranks' rollouts concatenate into the
        rollout of the whole env group: PPO's replicated data-parallel update, ppo.py).  Only what the
        update reads is set: the Batch fields, the epoch permutation source, the explained variance."""
        self = cls.__new__(cls)
        Rollout.__init__(self)
        self.device = device
        self.obs, self.actions, self.values, self.logprobs = obs, actions, values, logprobs
        self.advantages, self.returns = advantages, returns
        self.action_masks, self.num_actions = action_masks, num_actions
        self.rewards = self.episode_starts = self.next_episode_starts = self.next_values = None
        self._perm_source, self._generator, self._perm_keys = perm_source, None, perm_keys
        self._flat, self._perm_bufs = None, {}
        return self

    # -- Rollout API ---------------------------------------------------------------------
    @property
    def y_true(self) -> np.ndarray:
        return self.returns.reshape((-1,) + tuple(self.returns.shape[2:])).cpu().numpy()

    @property
    def y_pred(self) -> np.ndarray:
        return self.values.reshape((-1,) + tuple(self.values.shape[2:])).cpu().numpy()

    @property
    def total_steps(self) -> int:
        return int(self.values.shape[0] * self.values.shape[1])

    def num_minibatches(self, batch_size: int) -> int:
        return self.total_steps // batch_size + (1 if self.total_steps % batch_size else 0)

    def explained_variance(self) -> float:
        """1 - var(R - V)/var(R) (ppo.py:415-418), reduced on device, one host read."""
        y = self.returns.reshape(-1).double()
        p = self.values.reshape(-1).double()
        var_y = torch.var(y, unbiased=False)
        ev = 1 - torch.var(y - p, unbiased=False) / var_y
        var_y, ev = (float(x) for x in torch.stack([var_y, ev]).cpu())
        return float("nan") if var_y == 0 else ev

    def _flat_fields(self) -> List[torch.Tensor]:
        if self._flat is None:
            fl = lambda t: t.reshape((-1,) + tuple(t.shape[2:]))
            fields = [fl(self.obs), fl(self.actions), fl(self.values), fl(self.advantages), fl(self.returns)]
            if self.logprobs is not None:
                fields.append(fl(self.logprobs))
            if self.action_masks is not None:
                fields.append(fl(self.action_masks))
            self._flat = fields
        return self._flat

    def _epoch_fields(self) -> List[torch.Tensor]:
        """The fields an epoch's permuted copy carries: _flat_fields() (what the update's kernels read)
        plus Batch.num_actions when the rollout has action masks."""
        fields = self._flat_fields()
        if self.num_actions is not None:
            fields = fields + [self.num_actions.reshape(-1)]
        return fields

    def _batch_from(self, fields: List[torch.Tensor], sl: slice) -> Batch:
        """A Batch over rows sl of fields laid out as _epoch_fields() (num_actions optional)."""
        obs, actions, values, adv, ret = (f[sl] for f in fields[:5])
        i = 5
        logprobs = None
        if self.logprobs is not None:
            logprobs = fields[i][sl]
            i += 1
        masks = None
        if self.action_masks is not None:
            masks = fields[i][sl]
            i += 1
        num_actions = fields[i][sl] if len(fields) > i else None
        return Batch(obs, logprobs, actions, masks, num_actions, values, adv, ret)

    def permutation(self) -> torch.Tensor:
        if self._perm_source is not None:
            return self._perm_source(self.total_steps).to(self.device)
        if self._generator is not None:
            return torch.randperm(self.total_steps, device=self.device, generator=self._generator)
        return feistel_permutation(self.total_steps, self.device,
                                   key=self._perm_keys() if self._perm_keys is not None else None)

    def alloc_epoch_buffers(self, slot: int = 0) -> None:
        """Allocate the permuted copy `slot` (on the current stream) ahead of an epoch_batch that
        will run on another stream."""
        if slot not in self._perm_bufs:
            self._perm_bufs[slot] = [torch.empty_like(f) for f in self._epoch_fields()]

    def epoch_batch(self, shuffle: bool = True, slot: int = 0) -> Batch:
        """The whole rollout as one flat Batch, permuted for this epoch (one gather
        kernel); minibatch i is rows [i*batch_size, (i+1)*batch_size).  slot selects the
        permuted copy written (two slots: the next epoch's batch is prepared while the current
        one is read)."""
        flat = self._epoch_fields()
        if shuffle:
            self.alloc_epoch_buffers(slot)
            gather_rows(flat, self._perm_bufs[slot], self.permutation())
            src = self._perm_bufs[slot]
        else:
            src = flat
        return self._batch_from(src, slice(0, self.total_steps))

    def minibatches(self, batch_size: int, shuffle: bool = True) -> Iterator[Batch]:
        full = self.epoch_batch(shuffle)
        for i in range(0, self.total_steps, batch_size):
            sl = slice(i, i + batch_size)
            g = lambda t: None if t is None else t[sl]
            yield Batch(full.obs[sl], g(full.logprobs), full.actions[sl], g(full.action_masks), g(full.num_actions),
                        full.values[sl], full.advantages[sl], full.returns[sl])

    def add_to_batch(self, map_fn: BatchMapFn, batch_size: int) -> None:
        raise NotImplementedError("teacher-KL additional batch fields are outside the hot-path scope")


_UNSUPPORTED_GEN_KW = ("sde_sample_freq", "num_envs_reset_every_rollout", "rolling_num_envs_reset_every_rollout",
                       "random_num_envs_reset_every_rollout", "prepare_steps",
                       "rolling_num_envs_reset_every_prepare_step")


class SyncStepRolloutGenerator(RolloutGenerator):
    """Device-resident SyncStepRolloutGenerator (sync_step_rollout.py:14-216)."""

    def __init__(self, policy, vec_env, n_steps: int = 2048, sde_sample_freq: int = -1,
                 scale_advantage_by_values_accuracy: bool = False, full_batch_off_accelerator: bool = False,
                 include_logp: bool = True, subaction_mask=None, num_envs_reset_every_rollout: int = 0,
                 rolling_num_envs_reset_every_rollout: int = 0, random_num_envs_reset_every_rollout: int = 0,
                 prepare_steps: int = 0, rolling_num_envs_reset_every_prepare_step: int = 0,
                 gae_mode: int = EXACT, seed: Optional[int] = None) -> None:
        super().__init__(policy, vec_env)
        bad = [k for k, v, d in [("sde_sample_freq", sde_sample_freq, -1),
                                 ("num_envs_reset_every_rollout", num_envs_reset_every_rollout, 0),
                                 ("rolling_num_envs_reset_every_rollout", rolling_num_envs_reset_every_rollout, 0),
                                 ("random_num_envs_reset_every_rollout", random_num_envs_reset_every_rollout, 0),
                                 ("prepare_steps", prepare_steps, 0),
                                 ("rolling_num_envs_reset_every_prepare_step",
                                  rolling_num_envs_reset_every_prepare_step, 0)] if v != d]
        if bad or full_batch_off_accelerator:
            raise NotImplementedError(f"rollout options outside the hot-path scope: {bad or 'full_batch_off_accelerator'}")
        # rl_algo_impls/runner/train.py:159-162 copies the policy's subaction_mask into these kwargs; it
        # gates Batch.num_actions (sync_step_rollout.py:39,177 -> vec_rollout.py:69-76)
        self.subaction_mask = subaction_mask
        self.action_plane_space = getattr(vec_env, "action_plane_space", None)
        self.gridnet = bool(getattr(policy, "gridnet", False))
        self.get_action_mask = getattr(vec_env, "get_action_mask", None)
        if self.get_action_mask is not None and not self.gridnet:
            raise NotImplementedError("action masks are on the hot path for GridNet (squeeze_unet) policies only")
        if self.gridnet and self.get_action_mask is None:
            raise AssertionError("GridNet policies need the env's get_action_mask()")
        self.n_steps = n_steps
        self.include_logp = include_logp
        self.scale_advantage_by_values_accuracy = scale_advantage_by_values_accuracy
        self.gae_mode = gae_mode
        self.device = policy.device
        self.seed = int(torch.initial_seed() if seed is None else seed) & 0xFFFFFFFFFFFF
        self.rng_offset = 0
        self.perm_source: Optional[Callable[[int], torch.Tensor]] = None
        self.perm_count = 0  # epoch shuffles drawn: key (seed, count), like the samplers' (seed, offset)

        N = vec_env.num_envs
        T = n_steps
        obs_space, act_space = vec_env.single_observation_space, vec_env.single_action_space
        self.num_envs = N
        dev = self.device
        tdt = lambda d: torch.from_numpy(np.zeros((), dtype=d)).dtype
        self.obs_dtype = tdt(obs_space.dtype)
        self.discrete = is_discrete(act_space)
        if not (self.discrete or is_box(act_space) or self.gridnet):
            raise NotImplementedError(f"action space {act_space} is outside the hot-path scope")
        # GridNet (MicroRTS): per-position actions (map cells, planes) i64, K critic columns
        self.act_shape = tuple(policy.action_shape) if self.gridnet else (() if self.discrete else
                                                                          tuple(act_space.shape))
        act_dtype = torch.int64 if (self.discrete or self.gridnet) else torch.float32
        vshape = tuple(policy.value_shape)
        self.obs = torch.zeros((T, N) + tuple(obs_space.shape), dtype=self.obs_dtype, device=dev)
        self.rewards = torch.zeros((T, N) + vshape, dtype=torch.float32, device=dev)
        self.episode_starts = torch.zeros((T, N), dtype=torch.bool, device=dev)
        self.values = torch.zeros((T, N) + vshape, dtype=torch.float32, device=dev)
        self.action_masks = None
        self.rollout_graph = os.environ.get("RAI_ROLLOUT_GRAPH", "1") == "1" and self.device.type == "cuda"
        self._fwd_graph = None
        if self.gridnet:  # sync_step_rollout.py:119-131: (T, N, cells, sum(nvec)) bool
            m0 = np.asarray(self.get_action_mask())
            self.action_masks = torch.zeros((T,) + m0.shape, dtype=torch.bool, device=dev)
            self.h_mask = torch.zeros(m0.shape, dtype=torch.bool).pin_memory()
            self.next_masks_dev = torch.zeros(m0.shape, dtype=torch.bool, device=dev)
        self.logprobs = torch.zeros((T, N), dtype=torch.float32, device=dev)
        self.actions = torch.zeros((T, N) + self.act_shape, dtype=act_dtype, device=dev)
        self.clamped = torch.zeros((N,) + self.act_shape, dtype=act_dtype, device=dev)
        if not (self.discrete or self.gridnet):
            self.act_low = torch.as_tensor(np.asarray(act_space.low, np.float32), device=dev)
            self.act_high = torch.as_tensor(np.asarray(act_space.high, np.float32), device=dev)
        # pinned host staging (H2D obs/rewards/dones, D2H actions)
        self.h_obs = torch.zeros((N,) + tuple(obs_space.shape), dtype=self.obs_dtype).pin_memory()
        self.h_rew = torch.zeros((N,) + vshape, dtype=torch.float32).pin_memory()
        self.h_done = torch.zeros((N,), dtype=torch.bool).pin_memory()
        self.h_act = torch.zeros((N,) + self.act_shape, dtype=act_dtype).pin_memory()
        self.next_obs_dev = torch.zeros((N,) + tuple(obs_space.shape), dtype=self.obs_dtype, device=dev)
        # finished episodes' returns / lengths (gymnasium RecordEpisodeStatistics convention
        # info["episode"], info["_episode"]; what EpisodeStatsWriter logs as train_rolling/*,
        # rl_algo_impls/wrappers/episode_stats_writer.py:65-112), last 100
        self.episode_returns: Deque[float] = deque(maxlen=100)
        self.episode_lengths: Deque[int] = deque(maxlen=100)
        self.next_episode_starts = torch.ones((N,), dtype=torch.bool, device=dev)
        self._act_ready = torch.cuda.Event()
        # CartPole-class MLP policies: one fused launch per env step (rai_mlp_policy_step)
        from .policy import mlp_actor_critic_spec

        self.fused_step = None
        spec = mlp_actor_critic_spec(policy)
        if spec is not None and self.discrete and self.obs_dtype == torch.float32 and len(obs_space.shape) == 1:
            self.fused_step = spec
        # wide-MLP policies (HalfCheetah class): the rollout forward as rai_mlp_wide_dist_params (3
        # launches) instead of the PyTorch module; RAI_ROLLOUT_WIDE=0 keeps the module
        self._wide_fwd = None
        if (self.fused_step is None and not self.gridnet and self.device.type == "cuda"
                and os.environ.get("RAI_ROLLOUT_WIDE", "1") != "0" and len(obs_space.shape) == 1):
            from .mlp_wide import WideRolloutForward, wide_mlp_spec

            if wide_mlp_spec(policy) is not None and N <= _lib.RAI_WIDE_MAX_B:
                self._wide_fwd = WideRolloutForward(policy, dev, N)
        obs, _ = vec_env.reset()
        self._stage_obs(obs)
        self._stage_masks()

    def _stage_masks(self) -> None:
        if self.action_masks is not None:
            np.copyto(self.h_mask.numpy(), np.asarray(self.get_action_mask()))
            self.next_masks_dev.copy_(self.h_mask, non_blocking=True)

    def _policy_forward(self, fn):
        """The policy forward of one env step, fn(next_obs_dev) with next_obs_dev a fixed buffer,
        replayed from a hipGraph captured on first use: a CNN or MLP forward at rollout batch sizes
        is tens of small kernels, launch-bound when issued one by one (squeeze-U-Net: ~100).
        RAI_ROLLOUT_GRAPH=0 runs it eagerly.  The parameters are updated in place (flat buffer
        views), so the graph stays valid across updates."""
        if not self.rollout_graph:
            return fn(self.next_obs_dev)
        if self._fwd_graph is None:
            cur = torch.cuda.current_stream(self.device)
            side = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for _ in range(2):  # warm-up outside capture (solver selection, workspaces)
                    fn(self.next_obs_dev)
            cur.wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._g_out = fn(self.next_obs_dev)
            self._fwd_graph = g
        self._fwd_graph.replay()
        return self._g_out

    def _gridnet_step(self, s: int) -> None:
        """backbone_actor_critic.py:194-223 + gridnet.py sample: per-position actions, the fused
        GridNet sample + log-prob kernel, K critic values, written into slot s."""
        logits, v = self._policy_forward(self.policy.network.logits_and_value)
        pi = self.policy.network.distribution(logits, self.next_masks_dev)
        a, logp = pi.sample_with_logp(self.seed, self.rng_offset)
        self.rng_offset += 1
        self.actions[s].copy_(a.view(self.actions[s].shape))
        self.logprobs[s].copy_(logp)
        self.values[s].copy_(v)

    def _layer_ptrs(self):
        """The two networks' six weight / bias pointers as ctypes arrays, rebuilt only when a
        parameter's storage moved (the flat-buffer views keep theirs across updates)."""
        ps = list(self.policy.parameters())
        key = tuple(p.data_ptr() for p in ps)
        cached = getattr(self, "_ptrs_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        for p in ps:
            assert p.is_contiguous() and p.dtype == torch.float32
        arr = lambda xs: (C.c_void_p * 6)(*[x.data_ptr() for x in xs])
        out = (arr(ps[:6]), arr(ps[6:12]))
        self._ptrs_cache = (key, out)
        return out

    def _fused_step(self, s: Optional[int]) -> None:
        """Actor + critic forward, sample and slot writes for env step s (s None: bootstrap values
        of next_obs_dev into self._next_values)."""
        L = _lib.lib()
        sp = self.fused_step
        pi, v = self._layer_ptrs()
        N = self.num_envs
        st = _lib.stream_handle(self.device)
        if s is None:
            rc = L.rai_mlp_policy_step(None, v, self.next_obs_dev.data_ptr(), N, sp["in_dim"], 64, sp["n_act"],
                                       sp["activation"], self.seed, self.rng_offset, None, None,
                                       self._next_values.data_ptr(), st)
        else:
            rc = L.rai_mlp_policy_step(pi, v, self.obs[s].data_ptr(), N, sp["in_dim"], 64, sp["n_act"],
                                       sp["activation"], self.seed, self.rng_offset, self.actions[s].data_ptr(),
                                       self.logprobs[s].data_ptr(), self.values[s].data_ptr(), st)
            self.rng_offset += 1
        _lib.check(rc, "rai_mlp_policy_step")

    # an observation batch at least this large goes host -> device straight from the env's array
    _DIRECT_OBS_BYTES = 1 << 20

    def _stage_obs(self, obs: np.ndarray, dst: Optional[torch.Tensor] = None) -> None:
        """The next observation batch into next_obs_dev.  Large batches (C3 Pong: 1024 x 4x84x84 u8,
        29 MB) are copied straight from the env's pageable array: HIP's pageable path (~0.54 ms,
        ~53 GB/s, returns when the copy is done) is as fast as the DMA from pinned memory alone,
        while staging through the pinned buffer first costs a single-threaded host memcpy of the
        whole batch (1.35 ms; profiles/r2s_rollout_timing.txt).  Small batches keep the pinned
        buffer and an asynchronous copy."""
        dst = self.next_obs_dev if dst is None else dst
        if (obs.nbytes >= self._DIRECT_OBS_BYTES and isinstance(obs, np.ndarray) and obs.flags.c_contiguous
                and obs.flags.writeable and torch.from_numpy(obs[:0]).dtype == self.obs_dtype
                and obs.shape == tuple(dst.shape)):
            dst.copy_(torch.from_numpy(obs))
            return
        np.copyto(self.h_obs.numpy(), obs, casting="same_kind")
        dst.copy_(self.h_obs, non_blocking=True)

    def _sample(self, params: torch.Tensor, v: torch.Tensor, s: int) -> None:
        L = _lib.lib()
        st = _lib.stream_handle(self.device)
        N = self.num_envs
        params = params.contiguous().float()
        v = v.contiguous().float()
        if self.discrete:
            rc = L.rai_categorical_sample(params.data_ptr(), None, N, params.shape[-1], self.seed,
                                          self.rng_offset, self.actions[s].data_ptr(), self.logprobs[s].data_ptr(),
                                          v.data_ptr(), self.values[s].data_ptr(), 1, st)
            _lib.check(rc, "rai_categorical_sample")
        else:
            log_std = self.policy.network._pi.log_std.detach().contiguous()
            rc = L.rai_gaussian_sample(params.data_ptr(), log_std.data_ptr(), N, params.shape[-1],
                                       self.act_low.data_ptr(), self.act_high.data_ptr(), self.seed,
                                       self.rng_offset, self.actions[s].data_ptr(), self.clamped.data_ptr(),
                                       self.logprobs[s].data_ptr(), v.data_ptr(), self.values[s].data_ptr(), 1, st)
            _lib.check(rc, "rai_gaussian_sample")
        self.rng_offset += 1

    @torch.no_grad()
    def _rollout(self, output_next_values: bool) -> Optional[torch.Tensor]:
        self.policy.eval()
        net = self.policy.network
        # the fused CartPole-class step reads its slot directly: each step's next observations and episode
        # starts go host -> device straight into slot s + 1 (two device copies per step fewer); the other
        # policies' graph-replayed forwards read the fixed next_obs_dev buffer, so they keep the slot copy
        direct = self.fused_step is not None and os.environ.get("RAI_ROLLOUT_DIRECT", "1") != "0"
        if direct and self.action_masks is None and os.environ.get("RAI_ROLLOUT_NATIVE", "1") != "0":
            if os.environ.get("RAI_ROLLOUT_MAPPED", "1") != "0" and self.obs_dtype == torch.float32:
                self._fused_step_loop_mapped()
            else:
                self._fused_step_loop()
            return self._finish_rollout(output_next_values)
        for s in range(self.n_steps):
            if not direct or s == 0:
                self.obs[s].copy_(self.next_obs_dev)
                self.episode_starts[s].copy_(self.next_episode_starts)
            if self.action_masks is not None:
                self.action_masks[s].copy_(self.next_masks_dev)
            if self.fused_step is not None:
                self._fused_step(s)
            elif self.gridnet:
                self._gridnet_step(s)
            else:
                params, v = self._policy_forward(self._wide_fwd if self._wide_fwd is not None
                                                 else net.dist_params_and_value)
                self._sample(params, v, s)
            src = self.actions[s] if (self.discrete or self.gridnet) else self.clamped
            self.h_act.copy_(src, non_blocking=True)
            self._act_ready.record()
            self._act_ready.synchronize()
            obs, rew, term, trunc, info = self.vec_env.step(self.h_act.numpy())
            if info and "episode" in info:
                done_mask = np.asarray(info.get("_episode", np.ones(self.num_envs, dtype=bool)))
                self.episode_returns.extend(np.asarray(info["episode"]["r"])[done_mask].tolist())
                self.episode_lengths.extend(np.asarray(info["episode"]["l"])[done_mask].tolist())
            np.copyto(self.h_rew.numpy(), rew, casting="same_kind")
            np.logical_or(term, trunc, out=self.h_done.numpy())
            self.rewards[s].copy_(self.h_rew, non_blocking=True)
            into_slot = direct and s + 1 < self.n_steps
            (self.episode_starts[s + 1] if into_slot else self.next_episode_starts).copy_(self.h_done,
                                                                                           non_blocking=True)
            self._stage_obs(obs, self.obs[s + 1] if into_slot else None)
            self._stage_masks()
        return self._finish_rollout(output_next_values)

    def _fused_step_loop(self) -> None:
        """The CartPole-class env-step loop with one native call per host <-> device hand-off: the fused
        policy step (forward, sample, slot writes) into slot s, the actions copied to the pinned host
        buffer and waited for (rai_copy_d2h_sync), the host env step, then the rewards, terminations and
        next observations copied straight into their slots (rai_copy_h2d_multi).  Same kernels, same
        sampler stream and the same slot contents as the generic loop above (RAI_ROLLOUT_NATIVE=0); the
        per-step torch copy / event dispatches it replaces cost ~45 us of the ~95 us step at C2."""
        L = _lib.lib()
        sp = self.fused_step
        pi, v = self._layer_ptrs()
        st = _lib.stream_handle(self.device)
        N, T = self.num_envs, self.n_steps
        self.obs[0].copy_(self.next_obs_dev)
        self.episode_starts[0].copy_(self.next_episode_starts)
        slot = lambda t: (t.data_ptr(), t[0].numel() * t.element_size())  # base, bytes per step slot
        (ob, obs_b), (ab, act_b), (lb, lp_b), (vb, v_b), (rb, rew_b), (eb, es_b) = (
            slot(self.obs), slot(self.actions), slot(self.logprobs), slot(self.values), slot(self.rewards),
            slot(self.episode_starts))
        h_act, h_rew, h_done, h_obs = self.h_act, self.h_rew, self.h_done, self.h_obs
        assert h_act.numel() * h_act.element_size() == act_b and h_obs.numel() * h_obs.element_size() == obs_b
        h_act_np, h_rew_np, h_done_np, h_obs_np = h_act.numpy(), h_rew.numpy(), h_done.numpy(), h_obs.numpy()
        dst = (C.c_void_p * 3)()
        src = (C.c_void_p * 3)(h_rew.data_ptr(), h_done.data_ptr(), h_obs.data_ptr())
        nbytes = (C.c_int64 * 3)(rew_b, es_b, obs_b)
        last = (self.next_episode_starts.data_ptr(), self.next_obs_dev.data_ptr())
        in_dim, n_act, act_fn = sp["in_dim"], sp["n_act"], sp["activation"]
        for s in range(T):
            rc = L.rai_mlp_policy_step(pi, v, ob + s * obs_b, N, in_dim, 64, n_act, act_fn, self.seed, self.rng_offset,
                                       ab + s * act_b, lb + s * lp_b, vb + s * v_b, st)
            if rc:
                _lib.check(rc, "rai_mlp_policy_step")
            self.rng_offset += 1
            rc = L.rai_copy_d2h_sync(ab + s * act_b, h_act_np.ctypes.data, act_b, st)
            if rc:
                _lib.check(rc, "rai_copy_d2h_sync")
            obs, rew, term, trunc, info = self.vec_env.step(h_act_np)
            if info and "episode" in info:
                done_mask = np.asarray(info.get("_episode", np.ones(self.num_envs, dtype=bool)))
                self.episode_returns.extend(np.asarray(info["episode"]["r"])[done_mask].tolist())
                self.episode_lengths.extend(np.asarray(info["episode"]["l"])[done_mask].tolist())
            np.copyto(h_rew_np, rew, casting="same_kind")
            np.logical_or(term, trunc, out=h_done_np)
            np.copyto(h_obs_np, obs, casting="same_kind")
            dst[0] = rb + s * rew_b
            if s + 1 < T:
                dst[1], dst[2] = eb + (s + 1) * es_b, ob + (s + 1) * obs_b
            else:
                dst[1], dst[2] = last
            rc = L.rai_copy_h2d_multi(3, dst, src, nbytes, st)
            if rc:
                _lib.check(rc, "rai_copy_h2d_multi")

    def _mapped_buffers(self) -> Dict[str, tuple]:
        """Host-mapped pinned staging buffers (rai_host_alloc: coherent host memory the policy-step kernel
        reads and writes directly) for the env hand-off: name -> (host address, device address, numpy view)."""
        if getattr(self, "_mapped", None) is None:
            L = _lib.lib()
            N = self.num_envs
            in_dim = int(np.prod(self.obs.shape[2:]))
            bufs: Dict[str, tuple] = {}
            for name, n, dt in (("obs", N * in_dim, np.float32), ("rew", N, np.float32), ("done", N, np.uint8),
                                ("act", N, np.int64)):
                nbytes = n * np.dtype(dt).itemsize
                h, d = C.c_void_p(), C.c_void_p()
                rc = L.rai_host_alloc(nbytes, C.byref(h), C.byref(d))
                if rc:
                    for hh, _, _ in bufs.values():
                        L.rai_host_free(C.c_void_p(hh))
                    _lib.check(rc, "rai_host_alloc")
                arr = np.frombuffer((C.c_char * nbytes).from_address(h.value), dtype=dt)
                bufs[name] = (h.value, d.value, arr)
            bufs["obs"] = bufs["obs"][:2] + (bufs["obs"][2].reshape(N, in_dim),)
            weakref.finalize(self, _free_host_buffers, [b[0] for b in bufs.values()])
            self._mapped = bufs
        return self._mapped

    def _fused_step_loop_mapped(self) -> None:
        """The CartPole-class env-step loop with ONE launch and one stream wait per env step: the policy
        step kernel reads the env's next observations, rewards and terminations straight from host-mapped
        pinned memory into their slots and writes the sampled actions to host-mapped memory too
        (rai_mlp_policy_step_mapped), so no per-step copy is issued.  Same kernel arithmetic and sampler
        stream as _fused_step_loop (RAI_ROLLOUT_MAPPED=0), bit-identical buffers."""
        L = _lib.lib()
        sp = self.fused_step
        pi, v = self._layer_ptrs()
        st = _lib.stream_handle(self.device)
        N, T = self.num_envs, self.n_steps
        m = self._mapped_buffers()
        (obs_h, obs_d, obs_np), (rew_h, rew_d, rew_np), (done_h, done_d, done_np), (act_h, act_d, act_np) = (
            m["obs"], m["rew"], m["done"], m["act"])
        self.obs[0].copy_(self.next_obs_dev)
        self.episode_starts[0].copy_(self.next_episode_starts)
        slot = lambda t: (t.data_ptr(), t[0].numel() * t.element_size())
        (ob, obs_b), (ab, act_b), (lb, lp_b), (vb, v_b), (rb, rew_b), (eb, es_b) = (
            slot(self.obs), slot(self.actions), slot(self.logprobs), slot(self.values), slot(self.rewards),
            slot(self.episode_starts))
        assert obs_np.nbytes == obs_b and act_np.nbytes == act_b and rew_np.nbytes == rew_b and done_np.nbytes == es_b
        in_dim, n_act, act_fn = sp["in_dim"], sp["n_act"], sp["activation"]
        for s in range(T):
            if s == 0:  # slot 0 already holds next_obs_dev / next_episode_starts (device copies above)
                rc = L.rai_mlp_policy_step_mapped(pi, v, None, ob, N, in_dim, 64, n_act, act_fn, self.seed,
                                                  self.rng_offset, ab, lb, vb, act_d, None, None, None, None, st)
            else:  # step s - 1's env results: observations -> obs slot s, rewards -> slot s - 1, starts -> slot s
                rc = L.rai_mlp_policy_step_mapped(pi, v, obs_d, ob + s * obs_b, N, in_dim, 64, n_act, act_fn,
                                                  self.seed, self.rng_offset, ab + s * act_b, lb + s * lp_b,
                                                  vb + s * v_b, act_d, rew_d, rb + (s - 1) * rew_b, done_d,
                                                  eb + s * es_b, st)
            if rc:
                _lib.check(rc, "rai_mlp_policy_step_mapped")
            self.rng_offset += 1
            rc = L.rai_stream_sync(st)
            if rc:
                _lib.check(rc, "rai_stream_sync")
            obs, rew, term, trunc, info = self.vec_env.step(act_np)
            if info and "episode" in info:
                done_mask = np.asarray(info.get("_episode", np.ones(self.num_envs, dtype=bool)))
                self.episode_returns.extend(np.asarray(info["episode"]["r"])[done_mask].tolist())
                self.episode_lengths.extend(np.asarray(info["episode"]["l"])[done_mask].tolist())
            np.copyto(rew_np, rew, casting="same_kind")
            np.logical_or(term, trunc, out=done_np)
            np.copyto(obs_np, obs.reshape(obs_np.shape), casting="same_kind")
        # the last step's results: rewards -> slot T - 1, starts / observations -> next_* (async copies from
        # the mapped buffers; the next rollout writes them only after its first stream wait)
        dst = (C.c_void_p * 3)(rb + (T - 1) * rew_b, self.next_episode_starts.data_ptr(), self.next_obs_dev.data_ptr())
        src = (C.c_void_p * 3)(rew_h, done_h, obs_h)
        nbytes = (C.c_int64 * 3)(rew_b, es_b, obs_b)
        _lib.check(L.rai_copy_h2d_multi(3, dst, src, nbytes, st), "rai_copy_h2d_multi")

    def _finish_rollout(self, output_next_values: bool) -> Optional[torch.Tensor]:
        net = self.policy.network
        next_values = None
        if output_next_values:
            if self.fused_step is not None:
                self._next_values = torch.empty((self.num_envs,), dtype=torch.float32, device=self.device)
                self._fused_step(None)
                next_values = self._next_values
            else:
                next_values = net.value(self.next_obs_dev).float()
        self.policy.train()
        return next_values

    def _perm_key(self) -> int:
        k = (self.seed << 16) ^ self.perm_count
        self.perm_count += 1
        return k

    def rollout(self, gamma, gae_lambda) -> DeviceRollout:
        next_values = self._rollout(output_next_values=True)
        return DeviceRollout(
            self.device, self.next_episode_starts.clone(), next_values, self.obs, self.actions, self.rewards,
            self.episode_starts, self.values, self.logprobs if self.include_logp else None, self.action_masks, gamma,
            gae_lambda, self.scale_advantage_by_values_accuracy, self.gae_mode, self.perm_source,
            perm_keys=self._perm_key, subaction_mask=self.subaction_mask, action_plane_space=self.action_plane_space)
