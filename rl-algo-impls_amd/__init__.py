"""rl_algo_impls_amd — MI355X (gfx950) PPO/A2C rollout+update hot path.

Drop-in behind toldo4/rl-algo-impls' plugin points (ALGOS / POLICIES /
DEFAULT_ROLLOUT_GENERATORS, the Rollout/Batch contract, compute_advantages and
the VectorEnv API).  Submodules are imported lazily so that host-only pieces
(envs, schedules) do not load the HIP library.
"""
from __future__ import annotations

import importlib

__version__ = "0.1.0"

_LAZY = {
    "compute_advantages": "gae",
    "compute_advantages_device": "gae",
    "PPO": "ppo",
    "A2C": "a2c",
    "ActorCritic": "policy",
    "SyncStepRolloutGenerator": "rollout",
    "DeviceRollout": "rollout",
    "Batch": "rollout",
    "ALGOS": "registry",
    "POLICIES": "registry",
    "DEFAULT_ROLLOUT_GENERATORS": "registry",
}


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError(name)
    return getattr(importlib.import_module(f"{__name__}.{mod}"), name)
