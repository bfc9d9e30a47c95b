"""Diagnostic: the C2 (CartPole 4096 envs x 128 steps) rollout's per-env-step wall time split by host
timers: the whole rollout, then each phase of the step loop alone (env.step, the fused policy step, the
D2H action copy + wait, the three H2D copies).  Not part of the product or the tests.

    python tools/c2_rollout_timing.py
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
import bench  # noqa: E402
from rl_algo_impls_amd.envs import SyntheticVecEnv  # noqa: E402
from rl_algo_impls_amd.policy import ActorCritic  # noqa: E402
from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator  # noqa: E402

cfg = bench.CONFIGS["cartpole"]
N, T = cfg["num_envs"], cfg["n_steps"]
dev = torch.device("cuda", 0)
torch.manual_seed(1)
env = SyntheticVecEnv(N, cfg["env"], seed=1)
policy = ActorCritic(env, **cfg["policy"]).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=T, seed=1234)
sync = torch.cuda.synchronize
for _ in range(3):
    gen.rollout(0.98, 0.8)
sync()
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    gen.rollout(0.98, 0.8)
sync()
whole = (time.perf_counter() - t0) / reps
print(f"whole rollout (incl. GAE) {T} x {N}: {whole * 1e3:.2f} ms = {whole * 1e6 / T:.1f} us/step")
t0 = time.perf_counter()
for _ in range(reps):
    gen._rollout(False)
sync()
loop = (time.perf_counter() - t0) / reps
print(f"step loop alone: {loop * 1e3:.2f} ms = {loop * 1e6 / T:.1f} us/step")


def timed(name, fn, n=T * reps):
    for _ in range(10):
        fn()
    sync()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    sync()
    us = (time.perf_counter() - t) * 1e6 / n
    print(f"  {name:40s} {us:8.1f} us")


acts = gen.h_act.numpy().copy()
timed("env.step (host, numpy)", lambda: env.step(acts))
timed("fused policy step (launch, async)", lambda: gen._fused_step(0))
timed("fused policy step + sync", lambda: (gen._fused_step(0), sync()))


def d2h():
    gen.h_act.copy_(gen.actions[0], non_blocking=True)
    gen._act_ready.record()
    gen._act_ready.synchronize()


timed("D2H actions + event wait", d2h)
obs, rew, term, trunc, info = env.step(acts)
timed("3 H2D copies (rew, done, obs)", lambda: (gen.rewards[0].copy_(gen.h_rew, non_blocking=True),
                                                gen.episode_starts[1].copy_(gen.h_done, non_blocking=True),
                                                gen._stage_obs(obs, gen.obs[1])))
timed("np.copyto rew + logical_or done", lambda: (np.copyto(gen.h_rew.numpy(), rew, casting="same_kind"),
                                                  np.logical_or(term, trunc, out=gen.h_done.numpy())))
