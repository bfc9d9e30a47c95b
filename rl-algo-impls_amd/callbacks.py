"""Training callbacks on the update path: the hyperparameter schedule.

Mirrors rl_algo_impls/shared/callbacks/callback.py (Callback) and
rl_algo_impls/shared/callbacks/hyperparam_transitions.py:46-197 (HyperparamTransitions), with
rl_algo_impls/utils/interpolate.py:7-29 (linear / cosine interpolation).  `PPO.learn_epoch` calls
`on_step(timesteps_elapsed=<rollout steps>, train_stats=...)` after each update
(rl_algo_impls/ppo/ppo.py:430-438); the schedule writes the algorithm's mutable attributes
(learning_rate, clip_range, ent_coef, gamma, ...), which the next update uploads to the device.

The Lux reward-weights and LearningRateByKLDivergence hooks are outside this build's hot path
(SURVEY.md §2): a phase naming them raises ValueError like any other unsupported key.
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
        raise ValueError(f"{k} not supported in {self.__class__.__name__}")

    def maybe_update_phase(self, phase_idx: int) -> None:
        if phase_idx == self.current_phase_idx:
            return
        self.current_phase_idx = phase_idx
        phase = self.phases[phase_idx]
        print(f"{self.timesteps_elapsed}: Entering phase {phase_idx}: {phase}")
        for k, v in phase.items():
            target = self._target(k)
            setattr(target, k, v if (k in ALGO_BOOL_NAMES or k in ROLLOUT_GENERATOR_NAMES) else num_or_array(v))

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
            else:
                setattr(target, k, interpolate(num_or_array(old_v), num_or_array(next_v), transition_progress,
                                               self.interpolate_method))
