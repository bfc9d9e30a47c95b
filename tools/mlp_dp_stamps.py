"""Diagnostic: per-phase cycles of the multi-CU kernel on the data-parallel step path
(rai_mlp_ppo_epoch_dp over a 1-rank RCCL group), summed over all launches of one epoch.
Loads the stamps build (lib/librai_amd_stamps.so).  Not part of the product or the tests."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ["RAI_AMD_LIB"] = str(ROOT / "rl-algo-impls_amd" / "lib" / "librai_amd_stamps.so")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd import _lib  # noqa: E402
from rl_algo_impls_amd.envs import SyntheticVecEnv  # noqa: E402
from rl_algo_impls_amd.policy import ActorCritic  # noqa: E402
from rl_algo_impls_amd.ppo import PPO  # noqa: E402
from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator  # noqa: E402

NAMES = {1: "forward", 2: "loss + dZ2", 3: "dH1 + partials", 4: "P_B dW2 + sums", 5: "publish + counter",
         6: "reduce", 7: "stats/exchange", 8: "adam (epoch mode)", 9: "-", 10: "prologue (weights, m/v)",
         11: "apply prev step", 12: "after loop", 13: "epilogue (stats rows, writeback)",
         14: "pro: weights -> LDS", 15: "pro: m/v -> regs", 16: "pro: prefetch/pw/barrier",
         17: "apply: global |g|^2", 18: "apply: Adam"}
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
torch.manual_seed(1)
env = SyntheticVecEnv(int(os.environ.get("N", "1024")), "cartpole", seed=1)
policy = ActorCritic(env).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=128)
algo = PPO(policy, dev, None, batch_size=256, n_epochs=1, learning_rate=1e-3, gamma=0.98, gae_lambda=0.8)
algo.enable_data_parallel()
r = gen.rollout(gamma=0.98, gae_lambda=0.8)
algo.update(r)  # warm
torch.cuda.synchronize()
out0 = (C.c_ulonglong * 64)()
assert _lib.lib().rai_mlp_debug_stamps(out0) == 0
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
algo.update(r)
ev1.record()
ev1.synchronize()
out1 = (C.c_ulonglong * 64)()
assert _lib.lib().rai_mlp_debug_stamps(out1) == 0
st = (np.array(out1, dtype=np.float64) - np.array(out0, dtype=np.float64)).reshape(2, 32)
nmb = r.total_steps // 256
launches = nmb + 1
print(f"epoch {ev0.elapsed_time(ev1):.2f} ms, {nmb} steps, {launches} launches -> "
      f"{ev0.elapsed_time(ev1) * 1e3 / nmb:.2f} us/step")
for net in range(2):
    tot = st[net, 1:14].sum() + st[net, 14:19].sum()
    print(f"--- network {net}: {tot / launches:.0f} ticks per launch")
    for i in range(1, 19):
        if st[net, i]:
            print(f"  {NAMES[i]:34s} {st[net, i] / launches:10.1f} ticks/launch")
torch.distributed.destroy_process_group()
