"""Diagnostic: CartPole-v1 learning curve of the fused path per kernel layout and seed
(RAI_MLP_LAYOUT).  Prints the first step count at which the rolling mean of the last 100
episode returns passes 475, or the best mean reached in 100k steps.  Not part of the tests."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd.envs import CartPoleVecEnv  # noqa: E402
from rl_algo_impls_amd.policy import ActorCritic  # noqa: E402
from rl_algo_impls_amd.ppo import PPO  # noqa: E402
from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator  # noqa: E402

dev = torch.device("cuda", 0)
for seed in [int(s) for s in os.environ.get("SEEDS", "1,2,3,4").split(",")]:
    torch.manual_seed(seed)
    env = CartPoleVecEnv(8, seed=seed)
    policy = ActorCritic(env).to(dev)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=32, seed=seed)
    algo = PPO(policy, dev, None, batch_size=256, n_epochs=20, learning_rate=1e-3, gamma=0.98, gae_lambda=0.8,
               clip_range=0.2, ent_coef=0.0)
    best, steps, hit = 0.0, 0, None
    while steps < 100_000:
        # the YAML's hyperparam_transitions: lr 1e-3 -> 0 and clip 0.2 -> 0, linear in progress
        # (rl_algo_impls/shared/callbacks/hyperparam_transitions.py:85-100, interpolate "linear")
        prog = steps / 100_000
        algo.learning_rate, algo.clip_range = 1e-3 * (1 - prog), 0.2 * (1 - prog)
        steps, _ = algo.learn_epoch(steps, 100_000, gen, None)
        if len(gen.episode_returns) >= 20:
            best = max(best, float(np.mean(gen.episode_returns)))
        if best > 475 and hit is None:
            hit = steps
    print(f"layout={os.environ.get('RAI_MLP_LAYOUT', 'default')} seed={seed} best={best:.1f} "
          f"passed_475_at={hit}", flush=True)
