"""Diagnostic: wall time of consecutive PPO updates of a bench config and the device time of each
graph-replayed minibatch step (HIP events around MinibatchStepGraph.run), to find where a slow
update spends its time.  Not part of the product or the tests.

    python tools/replay_timing.py --config pong --updates 3
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
from rl_algo_impls_amd import graphs  # noqa: E402
from rl_algo_impls_amd.envs import SyntheticVecEnv  # noqa: E402
from rl_algo_impls_amd.policy import ActorCritic  # noqa: E402
from rl_algo_impls_amd.ppo import PPO  # noqa: E402
from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator  # noqa: E402
from rl_algo_impls_amd.running_utils import set_device_optimizations  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="pong")
p.add_argument("--num-envs", type=int, default=None)
p.add_argument("--updates", type=int, default=3)
p.add_argument("--deterministic", type=int, default=0)
args = p.parse_args()
cfg = bench.CONFIGS[args.config]
N, T = args.num_envs or cfg["num_envs"], cfg["n_steps"]
dev = torch.device("cuda", 0)
set_device_optimizations(dev, use_deterministic_algorithms=bool(args.deterministic))
torch.manual_seed(1)
env = SyntheticVecEnv(N, cfg["env"], seed=1)
policy = ActorCritic(env, **cfg["policy"]).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=T, seed=1234)
algo = PPO(policy, dev, None, **dict(cfg["algo"]))

events = []
orig_run = graphs.MinibatchStepGraph.run


def timed_run(self, desc, stream, step):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    t0 = time.perf_counter()
    orig_run(self, desc, stream, step)
    t1 = time.perf_counter()
    e1.record(stream)
    events.append((e0, e1, t1 - t0, self.graph is not None))


graphs.MinibatchStepGraph.run = timed_run
for u in range(args.updates):
    events.clear()
    t0 = time.perf_counter()
    algo.learn_epoch(0, 1, gen, None)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = np.array([a.elapsed_time(b) for a, b, _, _ in events])
    host_ms = np.array([h * 1e3 for _, _, h, _ in events])
    graphed = np.array([g for *_, g in events])
    print(f"update {u}: {wall:.2f} s (rollout {algo.last_rollout_seconds:.2f} s), {len(events)} minibatch steps, "
          f"graphed {int(graphed.sum())}", flush=True)
    if len(dev_ms):
        q = np.percentile(dev_ms, [0, 50, 90, 99, 100])
        print(f"  device ms per step: min {q[0]:.3f} p50 {q[1]:.3f} p90 {q[2]:.3f} p99 {q[3]:.3f} max {q[4]:.3f} "
              f"sum {dev_ms.sum():.1f}", flush=True)
        print(f"  host ms per launch: p50 {np.median(host_ms):.3f} max {host_ms.max():.1f} sum {host_ms.sum():.1f}",
              flush=True)
        slow = np.argsort(-dev_ms)[:8]
        print("  slowest steps (index, device ms):", [(int(i), round(float(dev_ms[i]), 2)) for i in slow], flush=True)
