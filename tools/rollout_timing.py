"""Diagnostic: where one env step of a bench config's rollout spends its wall time (host timers with
a device synchronize after every phase), next to the unsynchronised rollout, plus the host->device
staging alternatives for the step's observation batch.  Not part of the product or the tests.

    python tools/rollout_timing.py --config pong --steps 64
"""
import argparse
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
from rl_algo_impls_amd.running_utils import set_device_optimizations  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="pong")
p.add_argument("--num-envs", type=int, default=None)
p.add_argument("--steps", type=int, default=64)
args = p.parse_args()
cfg = bench.CONFIGS[args.config]
N, T = args.num_envs or cfg["num_envs"], cfg["n_steps"]
dev = torch.device("cuda", 0)
set_device_optimizations(dev, use_deterministic_algorithms=False)
torch.backends.cudnn.benchmark = True
torch.manual_seed(1)
env = SyntheticVecEnv(N, cfg["env"], seed=1)
policy = ActorCritic(env, **cfg["policy"]).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=T, seed=1234)
sync = torch.cuda.synchronize

for _ in range(2):
    gen.rollout(0.99, 0.95)
sync()
t0 = time.perf_counter()
gen.rollout(0.99, 0.95)
sync()
whole = time.perf_counter() - t0
print(f"whole rollout {T} steps x {N} envs: {whole * 1e3:.1f} ms = {whole * 1e3 / T:.3f} ms/step", flush=True)

# phase split of the generic (non-fused, non-GridNet) step, synchronising after every phase
net = policy.network
ph = {k: [] for k in ("slot copies", "forward graph", "sample", "D2H act + sync", "env.step",
                      "reward/done H2D", "stage obs (+ masks)")}
policy.eval()
with torch.no_grad():
    for s in range(args.steps):
        s_ = s % T
        t = [time.perf_counter()]
        gen.obs[s_].copy_(gen.next_obs_dev)
        gen.episode_starts[s_].copy_(gen.next_episode_starts)
        sync(); t.append(time.perf_counter())
        if gen.action_masks is not None:
            gen.action_masks[s_].copy_(gen.next_masks_dev)
        if gen.fused_step is not None:  # CartPole class: forward + sample in one launch
            gen._fused_step(s_)
            sync(); t.append(time.perf_counter())
        elif gen.gridnet:  # forward graph + GridNet sample in one phase, nothing in "sample"
            gen._gridnet_step(s_)
            sync(); t.append(time.perf_counter())
        else:
            params, v = gen._policy_forward(net.dist_params_and_value)
            sync(); t.append(time.perf_counter())
            gen._sample(params, v, s_)
        sync(); t.append(time.perf_counter())
        gen.h_act.copy_(gen.actions[s_] if (gen.discrete or gen.gridnet) else gen.clamped, non_blocking=True)
        gen._act_ready.record()
        gen._act_ready.synchronize()
        t.append(time.perf_counter())
        obs, rew, term, trunc, info = env.step(gen.h_act.numpy())
        np.copyto(gen.h_rew.numpy(), rew, casting="same_kind")
        np.logical_or(term, trunc, out=gen.h_done.numpy())
        t.append(time.perf_counter())
        gen.rewards[s_].copy_(gen.h_rew, non_blocking=True)
        gen.next_episode_starts.copy_(gen.h_done, non_blocking=True)
        sync(); t.append(time.perf_counter())
        gen._stage_obs(obs)
        gen._stage_masks()
        sync(); t.append(time.perf_counter())
        for k, a, b in zip(ph, t[:-1], t[1:]):
            ph[k].append(b - a)
tot = 0.0
for k, v in ph.items():
    m = float(np.median(v)) * 1e3
    tot += m
    print(f"  {k:24s} median {m:7.3f} ms", flush=True)
print(f"  {'sum of medians':24s}        {tot:7.3f} ms", flush=True)

# staging alternatives for one observation batch (median of 20)
obs = env._obs()
h = gen.h_obs
d = gen.next_obs_dev


def med(fn, n=20):
    xs = []
    for i in range(n):
        o = env._pool[i % len(env._pool)]
        sync()
        a = time.perf_counter()
        fn(o)
        sync()
        xs.append(time.perf_counter() - a)
    return float(np.median(xs)) * 1e3


print(f"obs batch {obs.nbytes / 1e6:.1f} MB, torch threads {torch.get_num_threads()}", flush=True)
print(f"  np.copyto -> pinned                 {med(lambda o: np.copyto(h.numpy(), o)):7.3f} ms", flush=True)
print(f"  torch copy_ -> pinned               {med(lambda o: h.copy_(torch.from_numpy(o))):7.3f} ms", flush=True)
print(f"  pinned -> device (H2D)              {med(lambda o: d.copy_(h, non_blocking=True)):7.3f} ms", flush=True)
print(f"  np.copyto + H2D                     "
      f"{med(lambda o: (np.copyto(h.numpy(), o), d.copy_(h, non_blocking=True))):7.3f} ms", flush=True)
print(f"  torch copy_ + H2D                   "
      f"{med(lambda o: (h.copy_(torch.from_numpy(o)), d.copy_(h, non_blocking=True))):7.3f} ms", flush=True)
print(f"  pageable -> device (direct)         {med(lambda o: d.copy_(torch.from_numpy(o))):7.3f} ms", flush=True)
H = N // 2


def halves(o):
    ot = torch.from_numpy(o)
    h[:H].copy_(ot[:H])
    d[:H].copy_(h[:H], non_blocking=True)
    h[H:].copy_(ot[H:])
    d[H:].copy_(h[H:], non_blocking=True)


print(f"  torch copy_ + H2D in two halves      {med(halves):7.3f} ms", flush=True)
