"""Host-side VectorEnv wrappers on the rollout path: observation / reward normalisation and
episode statistics.

Env stepping stays on the host behind the reference's VectorEnv API (north star), so these are
numpy wrappers with the reference's arithmetic:
  * RunningMeanStd / ExponentialMovingMeanVar / HybridMovingMeanVar
    — rl_algo_impls/utils/running_mean_std.py:10-199
  * NormalizeObservation / NormalizeReward — rl_algo_impls/wrappers/normalize.py:18-122
  * EpisodeStatsWriter (+ Episode, Statistic, EpisodesStats) — rl_algo_impls/wrappers/
    episode_stats_writer.py:16-112, rl_algo_impls/shared/stats.py:22-190
  * get_info / get_infos — rl_algo_impls/wrappers/vector_wrapper.py:35-57

Data parallel: each rank steps its own env group, but the reference normalises
with ONE running estimate over all envs.  `RunningMeanStd(group=...)` reproduces that: every
update all-gathers the ranks' (count, mean, M2) of their batch rows over a CPU (gloo)
process group, merges them in rank order (Chan et al.'s pairwise formula) into the global
batch's mean and population variance, and applies the reference's update to that — every rank
holds the identical statistics, equal to the single-process estimate over the concatenated
envs up to fp64 rounding.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np


# ---------------------------------------------------------------------------------------------
# info helpers (vector_wrapper.py:35-57)
def _get_dict_idx(d: Dict[str, Any], env_idx: int) -> Any:
    return {k: (_get_dict_idx(v, env_idx) if isinstance(v, dict) else v[env_idx]) for k, v in d.items()}


def get_info(infos: dict, key: Any, env_idx: int) -> Any:
    if key in infos:
        if isinstance(infos[key], dict):
            return _get_dict_idx(infos[key], env_idx)
        return infos[key][env_idx]
    return None


def get_infos(infos: dict, key: Any, num_envs: int, default_value: Any) -> List[Any]:
    if key in infos:
        assert len(infos[f"_{key}"]) == num_envs
        return [get_info(infos, key, i) if is_set else default_value for i, is_set in enumerate(infos[f"_{key}"])]
    return [default_value for _ in range(num_envs)]


def find_wrapper(env, wrapper_class):
    """vector_wrapper.py:26-32: the outermost wrapper of `wrapper_class` in env's chain."""
    current = env
    while current is not None and current is not getattr(current, "unwrapped", current):
        if isinstance(current, wrapper_class):
            return current
        current = getattr(current, "env", None)
    return None


class VectorWrapper:
    """Attribute-forwarding base (gymnasium VectorWrapper semantics the reference relies on)."""

    def __init__(self, env) -> None:
        self.env = env
        self.num_envs = env.num_envs
        self.single_observation_space = env.single_observation_space
        self.single_action_space = env.single_action_space

    def __getattr__(self, name: str):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def step(self, actions):
        return self.env.step(actions)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def close(self):
        return self.env.close()


# ---------------------------------------------------------------------------------------------
# running statistics (running_mean_std.py)
def _merge_batch_moments(group, x: np.ndarray) -> Tuple[np.ndarray, np.ndarray, int]:
    """Global batch (mean, population var, count) of the rows every rank of `group` holds."""
    import torch
    import torch.distributed as dist

    n = x.shape[0]
    mean = np.mean(x, axis=0, dtype=np.float64)
    m2 = np.var(x, axis=0, dtype=np.float64) * n
    mine = torch.from_numpy(np.concatenate([[float(n)], np.ravel(mean), np.ravel(m2)]).astype(np.float64))
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, mine, group=group)
    d = mean.size
    shape = mean.shape
    tot_n, tot_mean, tot_m2 = 0.0, np.zeros(shape), np.zeros(shape)
    for p in parts:  # rank order: bit-identical result on every rank
        p = p.numpy()
        nb, mb, m2b = p[0], p[1:1 + d].reshape(shape), p[1 + d:].reshape(shape)
        if nb == 0:
            continue
        if tot_n == 0:
            tot_n, tot_mean, tot_m2 = nb, mb.copy(), m2b.copy()
            continue
        delta = mb - tot_mean
        new_n = tot_n + nb
        tot_mean = tot_mean + delta * nb / new_n
        tot_m2 = tot_m2 + m2b + np.square(delta) * tot_n * nb / new_n
        tot_n = new_n
    return tot_mean, tot_m2 / tot_n, int(tot_n)


class RunningMeanStd:
    def __init__(self, epsilon: float = 1e-4, shape: Tuple[int, ...] = (), group=None) -> None:
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon
        self.group = group  # torch.distributed CPU group: merge every update across ranks

    def update(self, x: np.ndarray) -> None:
        if self.group is not None:
            batch_mean, batch_var, batch_count = _merge_batch_moments(self.group, np.asarray(x))
        else:
            batch_mean = np.mean(x, axis=0)
            batch_var = np.var(x, axis=0)
            batch_count = x.shape[0]
        delta = batch_mean - self.mean
        total_count = self.count + batch_count
        self.mean += delta * batch_count / total_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        M2 = m_a + m_b + np.square(delta) * self.count * batch_count / total_count
        self.var = M2 / total_count
        self.count = total_count

    def save(self, path: str) -> None:
        np.savez_compressed(path, mean=self.mean, var=self.var, count=self.count)

    def load(self, path: str, count_override: Optional[int] = None) -> None:
        data = np.load(path)
        self.mean = data["mean"]
        self.var = data["var"]
        self.count = data.get("count") if count_override is None else count_override

    def load_from(self, existing: "RunningMeanStd") -> None:
        self.mean = np.copy(existing.mean)
        self.var = np.copy(existing.var)
        self.count = np.copy(existing.count)


class ExponentialMovingMeanVar:
    def __init__(self, alpha: Optional[float] = None, window_size: Optional[Union[int, float]] = None,
                 shape: Tuple[int, ...] = ()) -> None:
        assert alpha is None or window_size is None, (
            f"Only one of alpha ({alpha}) or window_size ({window_size}) can be specified")
        if window_size is not None:
            alpha = 2 / (window_size + 1)
        assert alpha is not None, "Either alpha or window_size must be specified"
        assert 0 < alpha < 1, f"alpha ({alpha}) must be between 0 and 1 (exclusive)"
        self.alpha = alpha
        self.window_size = window_size if window_size is not None else (2 / alpha - 1)
        self.mean = np.zeros(shape, np.float64)
        self.squared_mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.initialized = False

    def update(self, x: np.ndarray) -> None:
        if not self.initialized:
            self.mean = np.mean(x, axis=0, dtype=np.float64)
            self.squared_mean = np.mean(x ** 2, axis=0, dtype=np.float64)
            self.var = np.var(x, axis=0, dtype=np.float64)
            self.initialized = True
            return
        w = (self.alpha * ((1 - self.alpha) ** np.arange(x.shape[0] - 1, -1, -1)))[:, None]
        self.mean = np.sum(w * x, axis=0) + (1 - np.sum(w)) * self.mean
        self.squared_mean = np.sum(w * (x ** 2), axis=0) + (1 - np.sum(w)) * self.squared_mean
        self.var = self.squared_mean - self.mean ** 2

    def save(self, path: str) -> None:
        np.savez_compressed(path, mean=self.mean, var=self.var, initialized=self.initialized)

    def load(self, path: str, count_override: Optional[int] = None) -> None:
        data = np.load(path)
        self.mean = data["mean"]
        self.var = data["var"]
        self.squared_mean = self.var + self.mean ** 2
        self.initialized = data["initialized"].item()

    def load_from(self, existing: "ExponentialMovingMeanVar") -> None:
        self.mean = np.copy(existing.mean)
        self.var = np.copy(existing.var)
        self.initialized = np.copy(existing.initialized)


class HybridMovingMeanVar:
    def __init__(self, alpha: Optional[float] = None, window_size: Optional[Union[int, float]] = None,
                 shape: Tuple[int, ...] = ()) -> None:
        self.rms = RunningMeanStd(shape=shape)
        self.emmv = ExponentialMovingMeanVar(alpha=alpha, window_size=window_size, shape=shape)

    def _frac(self) -> float:
        return self.rms.count / self.emmv.window_size

    @property
    def mean(self) -> np.ndarray:
        f = self._frac()
        return self.emmv.mean if f >= 1 else self.rms.mean * (1 - f) + self.emmv.mean * f

    @property
    def var(self) -> np.ndarray:
        f = self._frac()
        return self.emmv.var if f >= 1 else self.rms.var * (1 - f) + self.emmv.var * f

    def update(self, x: np.ndarray) -> None:
        self.rms.update(x)
        self.emmv.update(x)

    def save(self, path: str) -> None:
        self.rms.save(path + "-rms.npz")
        self.emmv.save(path + "-emmv.npz")

    def load(self, path: str, count_override: Optional[int] = None) -> None:
        self.rms.load(path + "-rms.npz", count_override=count_override)
        self.emmv.load(path + "-emmv.npz", count_override=count_override)

    def load_from(self, existing: "HybridMovingMeanVar") -> None:
        self.rms.load_from(existing.rms)
        self.emmv.load_from(existing.emmv)


# ---------------------------------------------------------------------------------------------
# normalisation wrappers (normalize.py)
class NormalizeObservation(VectorWrapper):
    def __init__(self, env, training: bool = True, epsilon: float = 1e-8, clip: float = 10.0, group=None) -> None:
        super().__init__(env)
        self.rms = RunningMeanStd(shape=env.single_observation_space.shape, group=group)
        self.training = training
        self.epsilon = epsilon
        self.clip = clip

    def step(self, action):
        obs, reward, terminations, truncations, info = self.env.step(action)
        return self.normalize(obs), reward, terminations, truncations, info

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        return self.normalize(obs), info

    def normalize(self, obs: np.ndarray) -> np.ndarray:
        if self.training:
            self.rms.update(obs)
        return np.clip((obs - self.rms.mean) / np.sqrt(self.rms.var + self.epsilon), -self.clip, self.clip)

    def save(self, path: str) -> None:
        self.rms.save(path)

    def load(self, path: str) -> None:
        self.rms.load(path)

    def load_from(self, existing: "NormalizeObservation") -> None:
        self.rms.load_from(existing.rms)


class NormalizeReward(VectorWrapper):
    def __init__(self, env, training: bool = True, gamma: float = 0.99, epsilon: float = 1e-8, clip: float = 10.0,
                 shape: Tuple[int, ...] = (), exponential_moving_mean_var: bool = False,
                 emv_window_size: Optional[Union[int, float]] = None, group=None) -> None:
        super().__init__(env)
        if exponential_moving_mean_var:
            if group is not None:
                raise NotImplementedError("cross-rank merge of the exponential moving estimate")
            self.rms = HybridMovingMeanVar(window_size=emv_window_size, shape=shape)
        else:
            self.rms = RunningMeanStd(shape=shape, group=group)
        self.training = training
        self.gamma = gamma
        self.epsilon = epsilon
        self.clip = clip
        self.returns = np.zeros((self.num_envs,) + shape)

    def step(self, action):
        obs, reward, terminations, truncations, info = self.env.step(action)
        reward = self.normalize(reward)
        self.returns[terminations | truncations] = 0
        return obs, reward, terminations, truncations, info

    def reset(self, **kwargs):
        self.returns = np.zeros_like(self.returns)
        return self.env.reset(**kwargs)

    def masked_reset(self, env_mask: np.ndarray):
        self.returns[env_mask] = 0
        return self.env.masked_reset(env_mask)

    def normalize(self, rewards):
        if self.training:
            self.returns = self.returns * self.gamma + rewards
            self.rms.update(self.returns)
        return np.clip(rewards / np.sqrt(self.rms.var + self.epsilon), -self.clip, self.clip)

    def save(self, path: str) -> None:
        self.rms.save(path)

    def load(self, path: str) -> None:
        self.rms.load(path)

    def load_from(self, existing: "NormalizeReward") -> None:
        self.rms.load_from(existing.rms)


# ---------------------------------------------------------------------------------------------
# episode statistics (shared/stats.py, wrappers/episode_stats_writer.py)
@dataclass
class Episode:
    score: float = 0
    length: int = 0
    info: Dict[str, Any] = field(default_factory=dict)


@dataclass
class Statistic:
    values: np.ndarray
    round_digits: int = 2
    score_function: str = "mean-std"

    @property
    def mean(self) -> float:
        return np.mean(self.values).item()

    @property
    def std(self) -> float:
        return np.std(self.values).item()

    @property
    def min(self) -> float:
        return np.min(self.values).item()

    @property
    def max(self) -> float:
        return np.max(self.values).item()

    def __len__(self) -> int:
        return len(self.values)

    def score(self) -> float:
        if self.score_function == "mean-std":
            return self.mean - self.std
        if self.score_function == "mean":
            return self.mean
        raise NotImplementedError(f"Only mean-std and mean score_functions supported ({self.score_function})")

    def __repr__(self) -> str:
        mean = round(self.mean, self.round_digits)
        if self.round_digits == 0:
            mean = int(mean)
        if self.score_function == "mean":
            return f"{mean}"
        std = round(self.std, self.round_digits)
        if self.round_digits == 0:
            std = int(std)
        return f"{mean} +/- {std}"


def _add_info_values(values: Dict[str, List], info: Dict[str, Any], path: Tuple[str, ...] = ()) -> None:
    for k, v in info.items():
        if isinstance(v, dict):
            _add_info_values(values, v, path=(*path, k))
        else:
            values.setdefault("_".join((*path, k)), []).append(v)


class EpisodesStats:
    def __init__(self, episodes: Sequence[Episode], simple: bool = False, score_function: str = "mean-std") -> None:
        self.episodes = episodes
        self.simple = simple
        self.score = Statistic(np.array([e.score for e in episodes]), score_function=score_function)
        self.length = Statistic(np.array([e.length for e in episodes]), round_digits=0)
        additional: Dict[str, List] = {}
        for e in episodes:
            if e.info:
                _add_info_values(additional, e.info)
        self.additional_stats = {k: Statistic(np.array(v)) for k, v in additional.items()}

    def __len__(self) -> int:
        return len(self.episodes)

    def __repr__(self) -> str:
        mean, score = self.score.mean, self.score.score()
        if mean != score:
            return f"Score: {self.score} ({round(score)}) | Length: {self.length}"
        return f"Score: {self.score} | Length: {self.length}"

    def write_to_tensorboard(self, tb_writer, main_tag: str) -> None:
        stats = {"mean": self.score.mean}
        if not self.simple:
            stats.update({"min": self.score.min, "max": self.score.max, "result": self.score.score(),
                          "n_episodes": len(self.episodes), "length": self.length.mean})
            for k, s in self.additional_stats.items():
                stats[k] = s.mean
        if tb_writer is None:
            return
        for name, value in stats.items():
            tb_writer.add_scalar(f"{main_tag}/{name}", value)


class EpisodeStatsWriter(VectorWrapper):
    """Logs finished episodes as `train/mean` and `train_rolling/{mean,min,max,result,n_episodes,
    length}` over the last `rolling_length` episodes (episode_stats_writer.py:65-112).  Reads the
    RecordEpisodeStatistics convention: info["episode"] with mask info["_episode"], or the
    same-step-autoreset info["final_info"][i]["episode"]."""

    def __init__(self, env, tb_writer, training: bool = True, rolling_length: int = 100,
                 additional_keys_to_log: Optional[List[str]] = None) -> None:
        super().__init__(env)
        self.training = training
        self.tb_writer = tb_writer
        self.rolling_length = rolling_length
        self.episodes: deque = deque(maxlen=rolling_length)
        self.total_steps = 0
        self.episode_cnt = 0
        self.last_episode_cnt_print = 0
        self.additional_keys_to_log = additional_keys_to_log or []
        self._steps_per_step: Optional[int] = None
        self._record_stats_enabled = True

    def step(self, actions):
        obs, rewards, terminations, truncations, infos = self.env.step(actions)
        self._record_stats(infos)
        return obs, rewards, terminations, truncations, infos

    def reset(self, **kwargs):
        obs, infos = self.env.reset(**kwargs)
        self._record_stats(infos)
        return obs, infos

    @property
    def steps_per_step(self) -> int:
        return getattr(self.env, "num_envs", 1) if self._steps_per_step is None else self._steps_per_step

    @steps_per_step.setter
    def steps_per_step(self, v: int) -> None:
        self._steps_per_step = v

    def disable_record_stats(self) -> None:
        self._record_stats_enabled = False

    def enable_record_stats(self) -> None:
        self._record_stats_enabled = True

    def _record_stats(self, infos: dict) -> None:
        if not self._record_stats_enabled:
            return
        self.total_steps += self.steps_per_step
        step_episodes = []
        if "episode" not in infos:
            for final_info in get_infos(infos, "final_info", self.num_envs, {}):
                if final_info and "episode" in final_info:
                    ep = Episode(np.asarray(final_info["episode"]["r"]).item(),
                                 np.asarray(final_info["episode"]["l"]).item(),
                                 info={k: final_info[k] for k in self.additional_keys_to_log})
                    step_episodes.append(ep)
                    self.episodes.append(ep)
        else:
            for env_idx, ep_info in enumerate(get_infos(infos, "episode", self.num_envs, {})):
                if ep_info:
                    ep = Episode(ep_info["r"], ep_info["l"],
                                 info={k: get_info(infos, k, env_idx) for k in self.additional_keys_to_log})
                    step_episodes.append(ep)
                    self.episodes.append(ep)
        if step_episodes:
            tag = "train" if self.training else "eval"
            EpisodesStats(step_episodes, simple=True).write_to_tensorboard(self.tb_writer, tag)
            rolling = EpisodesStats(self.episodes)
            rolling.write_to_tensorboard(self.tb_writer, f"{tag}_rolling")
            self.episode_cnt += len(step_episodes)
            if self.episode_cnt >= self.last_episode_cnt_print + self.rolling_length:
                print(f"Episode: {self.episode_cnt} | Steps: {self.total_steps} | {rolling}")
                self.last_episode_cnt_print += self.rolling_length
