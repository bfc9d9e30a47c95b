"""Diagnostic: torch.profiler op table of one PPO update (rollout + update) for a bench config, to
attribute GPU kernels (e.g. non-vectorised elementwise copies) to the aten ops that issue them.
Not part of the product or the tests.

    python tools/torch_prof.py --config microrts --num-envs 64 > gpurun_out/torch_prof.txt
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
import bench  # noqa: E402
from rl_algo_impls_amd.envs import SyntheticVecEnv  # noqa: E402
from rl_algo_impls_amd.policy import ActorCritic  # noqa: E402
from rl_algo_impls_amd.ppo import PPO  # noqa: E402
from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="microrts")
p.add_argument("--num-envs", type=int, default=64)
p.add_argument("--rows", type=int, default=30)
p.add_argument("--deterministic", type=int, default=0)
args = p.parse_args()
cfg = bench.CONFIGS[args.config]
N, T = args.num_envs, cfg["n_steps"]
algo_kw = dict(cfg["algo"])
if args.config == "microrts":
    algo_kw["batch_size"] = max(1, algo_kw["batch_size"] * N // cfg["num_envs"])
dev = torch.device("cuda", 0)
from rl_algo_impls_amd.running_utils import set_device_optimizations  # noqa: E402

set_device_optimizations(dev, use_deterministic_algorithms=bool(args.deterministic))
torch.manual_seed(1)
env = SyntheticVecEnv(N, cfg["env"], seed=1)
policy = ActorCritic(env, **cfg["policy"]).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=T, seed=1234)
algo = PPO(policy, dev, None, **algo_kw)
algo.learn_epoch(0, 1, gen, None)  # warm-up: solver selection, graph capture
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
    algo.learn_epoch(0, 1, gen, None)
    torch.cuda.synchronize()
print(f"rollout {algo.last_rollout_seconds:.3f} s of {algo.last_update_seconds:.3f} s")
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=args.rows, max_name_column_width=60))
# aten ops by the device time of the kernels they issued (CUDA total), with input shapes
ops = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")]
ops.sort(key=lambda e: -e.device_time_total)
for e in ops[:args.rows]:
    print(f"{e.device_time_total / 1e3:9.1f} ms  n={e.count:6d}  {e.key:32s} {str(e.input_shapes)[:110]}")
