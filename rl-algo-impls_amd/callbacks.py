"""Training callbacks on the update path: the hyperparameter schedule.

Mirrors rl_algo_impls/shared/callbacks/callback.py (Callback) and
rl_algo_impls/shared/callbacks/hyperparam_transitions.py:46-197 (HyperparamTransitions), with
rl_algo_impls/utils/interpolate.py:7-29 (linear / cosine interpolation).  `PPO.learn_epoch` calls
`on_step(timesteps_elapsed=<rollout steps>, train_stats=...)` after each update
(rl_algo_impls/ppo/ppo.py:430-438); the schedule writes the algorithm's mutable attributes
(learning_rate, clip_range, ent_coef, gamma, ...), which the next update uploads to the device.

LearningRateByKLDivergence (rl_algo_impls/ppo/learning_rate_by_kl_divergence.py:10-103) is the
host-side learning-rate controller SURVEY.md §2 row 2 marks on the path: after each update it scales
`algo.learning_rate` toward a target approx_kl (the next update uploads the new rate).  The schedule's
phases may set its `target_kl` (hyperparam_transitions.py:41-43,124-127,184-197), as the `*-lr-by-kl`
YAML configs do (rl_algo_impls/hyperparams/ppo.yml:302-335).  The Lux reward-weights hook is outside
this build's hot path: a phase naming it raises ValueError like any other unsupported key.
"""
from __future__ import annotations

from enum import Enum
from typing import Any, Dict, List, Optional, Union

import numpy as np

# hyperparam_transitions.py:19-31 (the attributes the schedule may set on the algorithm)
ALGO_SET_NAMES = {
    "gae_lambda", "multi_reward_weights", "vf_coef", "switch_range", "guide_probability", "learning_rate",
    "clip_range", "clip_range_vf", "ent_coef", "gamma", "teacher_kl_loss_coef",
}
ALGO_BOOL_NAMES = {"freeze_policy_head", "freeze_value_head", "freeze_backbone"}
ROLLOUT_GENERATOR_NAMES = {"rolling_num_envs_reset_every_rollout", "random_num_envs_reset_every_rollout"}
LEARNING_RATE_BY_KL_DIVERGENCE_NAMES = {"target_kl"}  # hyperparam_transitions.py:41-43


class InterpolateMethod(Enum):
    LINEAR = 0
    COSINE = 1


def lerp(start, end, progress: float):
    return start + (end - start) * progress


def cosine_interpolate(start, end, progress: float):
    # np.cos makes this an np.float64 for float inputs (SURVEY.md §8a A16 notes the NEP 50 effect
    # on a scheduled gamma; the GAE entry point keeps the reference's promotion either way)
    return (1 - np.cos(progress * np.pi)) / 2 * (end - start) + start


def interpolate(start, end, progress: float, method: InterpolateMethod):
    if method == InterpolateMethod.LINEAR:
        return lerp(start, end, progress)
    if method == InterpolateMethod.COSINE:
        return cosine_interpolate(start, end, progress)
    raise ValueError(f"{method} not valid")


def num_or_array(v: Union[float, List[float]]):
    """rl_algo_impls/shared/tensor_utils.py:38-41."""
    return np.array(v) if isinstance(v, list) else v


class Callback:
    def __init__(self) -> None:
        self.timesteps_elapsed = 0

    def on_step(self, timesteps_elapsed: int = 1, **kwargs) -> bool:
        self.timesteps_elapsed += timesteps_elapsed
        return True


class HyperparamTransitions(Callback):
    """Phases of hyperparameter overrides with interpolated transitions between them.

    `durations` has 2·len(phases) − 1 entries summing to 1: phase 0, transition 0→1, phase 1, ...
    Progress = timesteps_elapsed / total_train_timesteps.  `config` is anything with
    `n_timesteps` (the reference passes its runner Config); `total_train_timesteps` may be given
    directly instead.
    """

    def __init__(self, config, env, algo, rollout_generator, phases: List[Dict[str, Any]],
                 durations: List[float], start_timesteps: int = 0, interpolate_method: str = "linear",
                 lr_by_kl_callback=None, total_train_timesteps: Optional[int] = None) -> None:
        super().__init__()
        self.env = env
        self.algo = algo
        self.rollout_generator = rollout_generator
        self.lr_by_kl_callback = lr_by_kl_callback
        self.phases = phases
        assert len(durations) == len(phases) * 2 - 1, (
            "Durations expected to be 2*len(phases)-1 to account for transitions between phases")
        assert np.isclose(np.sum(durations), 1)
        self.durations = durations
        self.total_train_timesteps = (total_train_timesteps if total_train_timesteps is not None
                                      else config.n_timesteps)
        self.timesteps_elapsed = start_timesteps
        self.interpolate_method = InterpolateMethod[interpolate_method.upper()]
        self.current_phase_idx: Optional[int] = None
        self.update()

    def on_step(self, timesteps_elapsed: int = 1, **kwargs) -> bool:
        super().on_step(timesteps_elapsed)
        self.update()
        return True

    def update(self) -> None:
        progress = self.timesteps_elapsed / self.total_train_timesteps
        prior = 0.0
        acc = 0.0
        for idx, d in enumerate(self.durations):
            acc += d
            if progress < acc:
                if idx % 2 == 0:
                    self.maybe_update_phase(idx // 2)
                else:
                    self.update_phase_transition(idx // 2, (progress - prior) / d)
                return
            prior = acc
        self.maybe_update_phase(len(self.phases) - 1)

    def _target(self, k: str):
        if k in ALGO_SET_NAMES or k in ALGO_BOOL_NAMES:
            assert hasattr(self.algo, k), f"{type(self.algo).__name__} has no attribute {k}"
            return self.algo
        if k in ROLLOUT_GENERATOR_NAMES:
            assert hasattr(self.rollout_generator, k)
            return self.rollout_generator
        if k in LEARNING_RATE_BY_KL_DIVERGENCE_NAMES:
            assert self.lr_by_kl_callback is not None
            assert hasattr(self.lr_by_kl_callback, k)
            return self.lr_by_kl_callback
        raise ValueError(f"{k} not supported in {self.__class__.__name__}")

    def maybe_update_phase(self, phase_idx: int) -> None:
        if phase_idx == self.current_phase_idx:
            return
        self.current_phase_idx = phase_idx
        phase = self.phases[phase_idx]
        print(f"{self.timesteps_elapsed}: Entering phase {phase_idx}: {phase}")
        for k, v in phase.items():
            target = self._target(k)
            plain = k in ALGO_BOOL_NAMES or k in ROLLOUT_GENERATOR_NAMES or k in LEARNING_RATE_BY_KL_DIVERGENCE_NAMES
            setattr(target, k, v if plain else num_or_array(v))

    def update_phase_transition(self, prior_phase_idx: int, transition_progress: float) -> None:
        if self.current_phase_idx is not None:
            print(f"{self.timesteps_elapsed}: Exiting phase {self.current_phase_idx}")
        self.current_phase_idx = None
        prior_phase = self.phases[prior_phase_idx]
        next_phase = self.phases[prior_phase_idx + 1]
        assert set(prior_phase.keys()) == set(next_phase.keys()), "An override has to be specified in every phase"
        for k, next_v in next_phase.items():
            old_v = prior_phase[k]
            target = self._target(k)
            if k in ALGO_BOOL_NAMES:
                setattr(target, k, old_v)
            elif k in ROLLOUT_GENERATOR_NAMES:
                v_type = type(getattr(target, k))
                setattr(target, k, v_type(interpolate(old_v, next_v, transition_progress, self.interpolate_method)))
            elif k in LEARNING_RATE_BY_KL_DIVERGENCE_NAMES:  # raw values, no num_or_array (:184-197)
                setattr(target, k, interpolate(old_v, next_v, transition_progress, self.interpolate_method))
            else:
                setattr(target, k, interpolate(num_or_array(old_v), num_or_array(next_v), transition_progress,
                                               self.interpolate_method))


class LearningRateByKLDivergence(Callback):
    """rl_algo_impls/ppo/learning_rate_by_kl_divergence.py:10-103.  After each update: an exponential
    moving mean of approx_kl (window `moving_window_size`); once more updates than the window have
    passed, learning_rate *= clip(target_kl / |mean kl|, min_decrease_fraction, max_increase_fraction).
    The increase cap shrinks while the fast/slow moving ratio of the value loss exceeds
    v_loss_threshold, and drops to 1 when no_increase_on_max_grad_norm and the update's mean gradient
    norm exceeded algo.max_grad_norm; min_lr / max_lr bound the result.  Host-side fp64 (numpy), like
    the reference; the device kernels read the new rate at the next update's upload."""

    def __init__(self, algo, target_kl: float, moving_window_size: int = 5, max_increase_fraction: float = 1.02,
                 min_decrease_fraction: float = 0.5, v_loss_threshold: Optional[float] = None,
                 v_loss_fast_moving_window_size: int = 10, v_loss_slow_moving_window_size: int = 50,
                 no_increase_on_max_grad_norm: bool = False, min_lr: Optional[float] = None,
                 max_lr: Optional[float] = None) -> None:
        from .wrappers import ExponentialMovingMeanVar

        super().__init__()
        self.algo = algo
        self.target_kl = target_kl
        self.max_increase_fraction = max_increase_fraction
        self.min_decrease_fraction = min_decrease_fraction
        self.rms_kl = ExponentialMovingMeanVar(window_size=moving_window_size)
        self.num_updates = 0
        self.v_loss_threshold = v_loss_threshold
        if v_loss_threshold is not None:
            self.slow_v_loss_rms = ExponentialMovingMeanVar(window_size=v_loss_slow_moving_window_size)
            self.fast_v_loss_rms = ExponentialMovingMeanVar(window_size=v_loss_fast_moving_window_size)
        self.no_increase_on_max_grad_norm = no_increase_on_max_grad_norm
        self.min_lr = min_lr
        self.max_lr = max_lr
        if min_lr is not None:
            assert self.algo.learning_rate >= min_lr, "Algo's learning rate is already below min_lr"
        if max_lr is not None:
            assert self.algo.learning_rate <= max_lr, "Algo's learning rate is already above max_lr"

    def on_step(self, train_stats, timesteps_elapsed: int = 1, **kwargs) -> bool:
        super().on_step(timesteps_elapsed)
        self.rms_kl.update(np.array([train_stats.approx_kl]))
        self.num_updates += 1
        if self.v_loss_threshold is not None:
            v_loss = np.array([np.mean(train_stats.v_loss)])
            self.slow_v_loss_rms.update(v_loss)
            self.fast_v_loss_rms.update(v_loss)

        lo, hi = self.min_decrease_fraction, self.max_increase_fraction
        if self.v_loss_threshold is not None and self.num_updates > self.slow_v_loss_rms.window_size:
            ratio = self.fast_v_loss_rms.mean.item() / self.slow_v_loss_rms.mean.item()
            if ratio > self.v_loss_threshold:  # value loss rising fast: cap the increase
                hi = max(hi - (ratio - self.v_loss_threshold), lo)
        if self.no_increase_on_max_grad_norm and train_stats.grad_norm > self.algo.max_grad_norm:
            hi = min(hi, 1.0)
        if self.num_updates > self.rms_kl.window_size:
            kl = self.rms_kl.mean.item()
            self.algo.learning_rate *= np.clip(self.target_kl / np.abs(kl), lo, hi)
        if self.min_lr is not None:
            self.algo.learning_rate = max(self.algo.learning_rate, self.min_lr)
        if self.max_lr is not None:
            self.algo.learning_rate = min(self.algo.learning_rate, self.max_lr)
        return True
