"""Plugin registries under the reference's names (rl_algo_impls/runner/running_utils.py:38-55),
so `--algo ppo|a2c|acbc` hyperparameters resolve to the MI355X implementations."""
from __future__ import annotations

from .a2c import A2C
from .acbc import ACBC
from .policy import ActorCritic
from .ppo import PPO
from .rollout import SyncStepRolloutGenerator

ALGOS = {"ppo": PPO, "a2c": A2C, "acbc": ACBC}
POLICIES = {"ppo": ActorCritic, "a2c": ActorCritic, "acbc": ActorCritic}
DEFAULT_ROLLOUT_GENERATORS = {"ppo": SyncStepRolloutGenerator, "a2c": SyncStepRolloutGenerator,
                              "acbc": SyncStepRolloutGenerator}
