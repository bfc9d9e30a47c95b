"""Diagnostic: per-phase shader-clock breakdown of the C4 whole-epoch kernel (rai_mlp_wide_epoch,
csrc/mlp_wide_epoch.hip).  Loads the stamps build (lib/librai_amd_stamps.so, -DRAI_STAMPS) and
runs one epoch of the HalfCheetah-shaped update (256 envs x 512 steps, batch 64).  Not part of the
product or the tests."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ["RAI_AMD_LIB"] = str(ROOT / "rl-algo-impls_amd" / "lib" / "librai_amd_stamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd import _lib  # noqa: E402
from rl_algo_impls_amd.envs import SyntheticVecEnv  # noqa: E402
from rl_algo_impls_amd.policy import ActorCritic  # noqa: E402
from rl_algo_impls_amd.ppo import PPO  # noqa: E402
from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator  # noqa: E402

NAMES = ["X + fwd1 + publish H1", "A wait (after the deferred Adam)", "gather H1", "fwd2 tile",
         "partials + publish P", "B wait", "load partials", "loss compute (wave 0)", "loss LDS out + barrier",
         "bwd2 dZ2 + publish", "small grads", "dW2 rows", "C wait", "gather dZ2", "dH1 + dZ1", "-", "dW1",
         "db1 (wave 3)", "norm share + drain", "prefetch issue", "D wait (wave 1: stats)", "clip + Adam",
         "A: arrival + deferred W2 Adam"]
lib = _lib.lib()
fn = getattr(lib, "rai_wide_epoch_debug_stamps")
fn.restype = C.c_int
fn.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
torch.manual_seed(1)
N, T = int(os.environ.get("N", "256")), int(os.environ.get("T", "512"))
env = SyntheticVecEnv(N, "halfcheetah", seed=1)
policy = ActorCritic(env, pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256], activation_fn="relu",
                     log_std_init=-2, init_layers_orthogonal=False).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=T)
algo = PPO(policy, dev, None, batch_size=64, n_epochs=1, learning_rate=2e-5, gamma=0.98, gae_lambda=0.92,
           clip_range=0.1, ent_coef=0.0004, max_grad_norm=0.8, vf_coef=0.58)
r = gen.rollout(gamma=0.98, gae_lambda=0.92)
algo.update(r)  # warm
torch.cuda.synchronize()
out0 = (C.c_ulonglong * 48)()
assert fn(out0) == 0
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
algo.update(r)
ev1.record()
ev1.synchronize()
out = (C.c_ulonglong * 48)()
assert fn(out) == 0
st = (np.array(out, dtype=np.float64) - np.array(out0, dtype=np.float64)).reshape(2, 24)
nmb = (r.total_steps + 63) // 64
assert algo._we_ws is not None, "whole-epoch kernel not used"
print(f"epoch {ev0.elapsed_time(ev1):.2f} ms for {nmb} minibatches -> {ev0.elapsed_time(ev1) * 1e3 / nmb:.2f} us/mb")
# slot 23: launches whose network ran on one XCC (plain-store hand-offs)
print(f"one-XCC store form: actor {st[0, 23]:.0f}, critic {st[1, 23]:.0f} of 1 launch")
for net in range(2):
    tot = st[net, :len(NAMES)].sum()
    print(f"--- workgroup 0 of the {'actor' if net == 0 else 'critic'}: {tot / nmb:.0f} ticks/mb")
    for i, n in enumerate(NAMES):
        print(f"  {n:44s} {st[net, i] / nmb:10.1f} ticks/mb  {100 * st[net, i] / tot:5.1f}%")
