"""Diagnostic: per-phase cycle breakdown of the fused MLP PPO epoch kernel.
Loads the stamps build (lib/librai_amd_stamps.so, -DRAI_STAMPS) and runs one epoch of
the CartPole 4096x128 / batch 256 workload.  Not part of the product or the tests."""
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

LAYOUT = os.environ.get("RAI_MLP_LAYOUT", "mc8")
NAMES = {
    "mc8": ["F1 (own columns) + barrier", "F2 + output partials + barrier", "loss + dZ2 + barrier",
            "dH1 + dZ1 + partials + barrier", "P_B dW2 + sums + barrier", "round 1: publish + counter wait",
            "share sum + round 2 publish + wait", "all-gather + norm + adam + barrier"],
    "mc4": ["F1+F2 forward", "out layer + loss + dZ2", "dH1 + partials + barrier", "P_B dW2 + sums",
           "publish + counter wait", "reduce G slots + |g|^2", "stats + norm exchange", "adam"],
    "rows": ["F1 layer1 (wave-local)", "F2 layer2 + epilogue", "out layer + loss + dZ2", "dH1 MFMA",
             "dZ1/partials + barrier", "P_B dW2 MFMA", "E2 owner sums + norm", "E3 stats + exchange",
             "E4 adam"],
}[LAYOUT]
dev = torch.device("cuda", 0)
torch.manual_seed(1)
env = SyntheticVecEnv(4096, "cartpole", seed=1)
policy = ActorCritic(env).to(dev)
gen = SyncStepRolloutGenerator(policy, env, n_steps=int(os.environ.get("T", "128")))
algo = PPO(policy, dev, None, batch_size=256, n_epochs=1, learning_rate=1e-3, gamma=0.98, gae_lambda=0.8)
r = gen.rollout(gamma=0.98, gae_lambda=0.8)
algo.update(r)  # warm
torch.cuda.synchronize()
out0 = (C.c_ulonglong * 64)()
assert _lib.lib().rai_mlp_debug_stamps(out0) == 0  # the kernels accumulate: take the difference
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
algo.update(r)
ev1.record()
ev1.synchronize()
out = (C.c_ulonglong * 64)()
rc = _lib.lib().rai_mlp_debug_stamps(out)
assert rc == 0, rc
st = (np.array(out, dtype=np.float64) - np.array(out0, dtype=np.float64)).reshape(2, 32)
nmb = r.total_steps // 256
print(f"epoch {ev0.elapsed_time(ev1):.2f} ms for {nmb} minibatches -> {ev0.elapsed_time(ev1) * 1e3 / nmb:.2f} us/mb")
# mc8: STAMP(15..19) close each compute phase's work and STAMP(1..5) the barrier wait after it; the exchange
# phases are split by STAMP(9..14).  Every stamp is the time since the previous one, so a phase's time is
# the sum of its work and wait stamps and the % column is over all of them (work plus waits).
MC8_PARTS = [(15, 1), (16, 2), (17, 3), (18, 4), (19, 5), (9, 10, 6), (11, 12, 13, 7), (14, 8)]
if LAYOUT == "mc8":  # slot 31: launches whose network ran on one XCC (plain-store hand-offs)
    print(f"one-XCC store form: actor {st[0, 31]:.0f}, critic {st[1, 31]:.0f} of 1 launch")
for net in range(2):
    if LAYOUT == "mc8":
        ph = [sum(st[net, i] for i in parts) for parts in MC8_PARTS]
    else:
        ph = [st[net, i + 1] for i in range(len(NAMES))]
    tot = sum(ph)
    print(f"--- workgroup {net} ({'actor' if net == 0 else 'critic'}): {tot / nmb:.0f} stamp-ticks/mb")
    for n, v in zip(NAMES, ph):
        print(f"  {n:36s} {v / nmb:10.1f} ticks/mb  {100 * v / tot:5.1f}%")
    if LAYOUT == "mc8":  # compute phases split into work and barrier wait
        for i, n in ((15, "F1 work"), (16, "F2 work"), (17, "loss work"), (18, "dH1 work"), (19, "P_B work")):
            print(f"  {n:34s} {st[net, i] / nmb:10.1f} ticks/mb (+ barrier {st[net, i - 14] / nmb:.1f})")
        for i, n in ((9, "  r1: wave-0 partial stores + drain"), (10, "  r1: barrier (other waves' drains)"),
                     (6, "  r1: counter wait + stats"), (11, "  r2: share-sum loads (+ xGMI)"),
                     (12, "  r2: share store + norm + drain"), (13, "  r2: barrier (other waves' drains)"),
                     (7, "  r2: counter wait (both networks)"), (14, "  ag: gradient + norm loads, norm sum"),
                     (8, "  ag: clip + adam + barrier")):
            print(f"  {n:34s} {st[net, i] / nmb:10.1f} ticks/mb")
