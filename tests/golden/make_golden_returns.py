"""Episode-return reference curves: the REFERENCE'S OWN PPO trained on CartPole-v1.

Runs rl_algo_impls' PPO.learn (rl_algo_impls/ppo/ppo.py:192-212,214-447) with its
SyncStepRolloutGenerator (rl_algo_impls/rollout/sync_step_rollout.py), its
EpisodeStatsWriter (rl_algo_impls/wrappers/episode_stats_writer.py:65-112, rolling deque of 100)
and its HyperparamTransitions (rl_algo_impls/shared/callbacks/hyperparam_transitions.py:46-197)
with the YAML CartPole-v1 hyperparameters (rl_algo_impls/hyperparams/ppo.yml:1-23), on CPU,
imported with ./stubs exactly as make_golden.py does.

The environment is the build's own envs.CartPoleVecEnv (gymnasium 0.29's public CartPole-v1
dynamics; gymnasium is not installed here) behind the stub VectorEnv, so the build's GPU trainer
can be run on the identical env, seeds and hyperparameters (tests/test_gpu_returns.py).

Written: returns_cartpole.json -- per config and seed, the per-update (timesteps, rolling mean of
the last 100 training episode returns) curve, the final rolling mean, and a 10-episode
deterministic evaluation (rl_algo_impls/shared/callbacks/eval_callback.py:79-240) of the final
policy on a fresh CartPoleVecEnv(8, seed + 1000).  Only outputs are stored.

    python tests/golden/make_golden_returns.py                 # all configs and seeds
    python tests/golden/make_golden_returns.py c2_4096x128     # one config; other configs' runs kept
    python tests/golden/make_golden_returns.py c2_4096x128_8u --add-seeds 4 5 6 7 8
                                                               # more seeds, the config's runs kept
"""
from __future__ import annotations

import json
import multiprocessing as mp
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]

CONFIGS = {
    # the YAML's CartPole-v1 entry (8 envs x 32 steps, 1e5 timesteps)
    "yaml_8x32": dict(n_envs=8, n_steps=32, n_timesteps=100_000),
    # BASELINE configs[0]: the reference CPU path at num_envs=8, n_steps=128
    "c1_8x128": dict(n_envs=8, n_steps=128, n_timesteps=100_000),
    # BASELINE configs[1] / the north star's headline config: 4096 envs x 128 steps, the YAML's
    # batch_size 256 x 20 epochs (40,960 optimizer steps per update), 4 updates with the YAML's
    # linear lr / clip decay over them.  ~3 min of CPU per update per process.
    "c2_4096x128": dict(n_envs=4096, n_steps=128, n_timesteps=4 * 4096 * 128),
    # the same config run twice as long (8 updates, the lr / clip decay spread over 8): closer to
    # convergence, where the return populations are tighter
    "c2_4096x128_8u": dict(n_envs=4096, n_steps=128, n_timesteps=8 * 4096 * 128),
}
# seeds per config (the C2 runs are ~40x the CPU time of the 8-env ones)
CONFIG_SEEDS = {"yaml_8x32": (1, 2, 3, 4, 5), "c1_8x128": (1, 2, 3, 4, 5), "c2_4096x128": (1, 2, 3),
                "c2_4096x128_8u": (1, 2, 3, 4, 5, 6, 7, 8)}  # 4-8 added in round 6 (--add-seeds)
ALGO_KW = dict(batch_size=256, n_epochs=20, gae_lambda=0.8, gamma=0.98, ent_coef=0.0,
               learning_rate=0.001, clip_range=0.2)
PHASES = [{"learning_rate": 0.001, "clip_range": 0.2}, {"learning_rate": 0.0, "clip_range": 0.0}]
DURATIONS = [0.0, 1.0, 0.0]
EVAL_EPISODES = 10


def run_one(args):
    cfg_name, seed = args
    import torch

    torch.set_num_threads(1)
    sys.path.insert(0, str(HERE))
    sys.path.insert(0, str(REPO))
    import make_golden as mg  # imports the reference with the stubs
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd import envs
    import gymnasium.spaces as gs
    from gymnasium.experimental.vector.vector_env import VectorEnv
    from types import SimpleNamespace

    from rl_algo_impls.ppo.ppo import PPO
    from rl_algo_impls.rollout.sync_step_rollout import SyncStepRolloutGenerator
    from rl_algo_impls.shared.callbacks.callback import Callback
    from rl_algo_impls.shared.callbacks.eval_callback import evaluate
    from rl_algo_impls.shared.callbacks.hyperparam_transitions import HyperparamTransitions
    from rl_algo_impls.shared.callbacks.summary_wrapper import SummaryWrapper
    from rl_algo_impls.shared.policy.actor_critic import ActorCritic
    from rl_algo_impls.wrappers.episode_stats_writer import EpisodeStatsWriter

    class RefCartPole(VectorEnv):
        """The build's CartPoleVecEnv with gymnasium (stub) spaces for the reference's policy."""

        def __init__(self, n, seed):
            self.inner = envs.CartPoleVecEnv(n, seed=seed)
            self.num_envs = n
            sp = self.inner.single_observation_space
            self.single_observation_space = gs.Box(sp.low, sp.high, (4,), np.float32)
            self.single_action_space = gs.Discrete(2)

        def reset(self, **kw):
            return self.inner.reset(**kw)

        def step(self, actions):
            return self.inner.step(actions)

    c = CONFIGS[cfg_name]
    # rl_algo_impls/runner/running_utils.py:175-180 set_seeds (its module imports wandb, absent here)
    import random

    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    writer = mg.SummaryWriter()
    tbw = SummaryWrapper(writer)
    inner = RefCartPole(c["n_envs"], seed)
    env = EpisodeStatsWriter(inner, tbw, rolling_length=100)
    # the stub VectorWrapper's class-level space attributes shadow __getattr__
    env.single_observation_space = inner.single_observation_space
    env.single_action_space = inner.single_action_space
    env.num_envs = inner.num_envs
    policy = ActorCritic(env).to(torch.device("cpu"))
    algo = PPO(policy, torch.device("cpu"), tbw, **ALGO_KW)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=c["n_steps"])
    config = SimpleNamespace(n_timesteps=c["n_timesteps"])
    ht = HyperparamTransitions(config, env, algo, gen, PHASES, DURATIONS)
    curve = []

    class Record(Callback):
        def on_step(self, timesteps_elapsed=1, **kw):
            super().on_step(timesteps_elapsed)
            eps = list(env.episodes)
            curve.append([int(self.timesteps_elapsed),
                          float(np.mean([e.score for e in eps])) if eps else 0.0, len(eps)])
            print(cfg_name, seed, curve[-1], flush=True)
            return True

    algo.learn(c["n_timesteps"], gen, callbacks=[ht, Record()])
    ev_env = RefCartPole(8, seed + 1000)
    st = evaluate(ev_env, policy, EVAL_EPISODES, deterministic=True, print_returns=False)
    return cfg_name, seed, dict(curve=curve, final_rolling_mean=curve[-1][1],
                                eval_mean=float(st.score.mean), eval_std=float(st.score.std))


def main():
    argv = sys.argv[1:]
    add = None
    if "--add-seeds" in argv:
        i = argv.index("--add-seeds")
        add = [int(x) for x in argv[i + 1:]]
        argv = argv[:i]
    names = argv or list(CONFIGS)
    jobs = [(c, s) for c in names for s in (add if add is not None else CONFIG_SEEDS[c])]
    with mp.get_context("spawn").Pool(min(int(__import__("os").environ.get("RETURNS_PROCS", "4")), len(jobs))) as pool:
        res = pool.map(run_one, jobs)
    path = HERE / "returns_cartpole.json"
    out = json.loads(path.read_text()) if path.exists() else dict(runs={})
    out.update(configs={k: CONFIGS[k] for k in set(out["runs"]) | set(names)}, algo_kw=ALGO_KW, phases=PHASES,
               durations=DURATIONS, eval_episodes=EVAL_EPISODES)
    for c in names:
        if add is None:
            out["runs"][c] = {}
    for cfg, seed, r in res:
        out["runs"].setdefault(cfg, {})[str(seed)] = r
        print(cfg, seed, "final rolling", round(r["final_rolling_mean"], 1), "eval", r["eval_mean"])
    path.write_text(json.dumps(out))


if __name__ == "__main__":
    main()
