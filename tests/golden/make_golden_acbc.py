"""Golden vectors for ACBC (Actor-Critic Behavior Cloning with critic bootstrapping,
rl_algo_impls/acbc/acbc.py:29-165): the third algorithm on the rollout + GAE hot path.

Runs the REFERENCE ITSELF in this container (stub imports as make_golden.py) on fixed minibatches
through ACBC.learn: per-optimizer-step pre-clip grads, grad norms, params, the per-step loss,
pi_loss and v_loss (which learn() only logs as means), and the Adam state.  Inputs and outputs
only are written (acbc_steps.npz).

    python tests/golden/make_golden_acbc.py
"""
from __future__ import annotations

import json

import numpy as np
import torch

import make_golden as mg  # noqa: E402  (imports the reference with the stubs)
from rl_algo_impls.acbc import acbc as acbc_mod  # noqa: E402
from rl_algo_impls.acbc.acbc import ACBC  # noqa: E402
from rl_algo_impls.shared.callbacks.summary_wrapper import SummaryWrapper  # noqa: E402
from rl_algo_impls.shared.policy.actor_critic import ActorCritic  # noqa: E402


def run(policy, batches, kw, n_epochs):
    writer = mg.SummaryWriter()
    algo = ACBC(policy, torch.device("cpu"), SummaryWrapper(writer), n_epochs=n_epochs, **kw)
    rec = dict(grads=[], norms=[], params=[], step_stats=[])

    def optimizer_step():
        ps = [p for p in policy.parameters()]
        rec["grads"].append(mg.flat([p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]))
        # clip_grad_norm_'s total norm (ACBC.optimizer_step does not return it)
        rec["norms"].append(float(torch.norm(torch.stack([torch.norm(p.grad.detach(), 2) for p in ps]), 2)))
        torch.nn.utils.clip_grad_norm_(policy.parameters(), algo.max_grad_norm)
        algo.optimizer.step()
        algo.optimizer.zero_grad()
        rec["params"].append(mg.flat(policy.parameters()))

    algo.optimizer_step = optimizer_step
    real_ts = acbc_mod.TrainStats

    def ts(step_stats, explained_var):  # the last epoch's per-step dicts
        rec["step_stats"] = [dict(s) for s in step_stats]
        return real_ts(step_stats, explained_var)

    acbc_mod.TrainStats = ts
    try:
        r = mg.FixedRollout(batches)
        algo.learn(r.total_steps, mg.FixedGen(r))
    finally:
        acbc_mod.TrainStats = real_ts
    opt = algo.optimizer.state_dict()
    st = [opt["state"][i] for i in sorted(opt["state"])]
    rec["opt_state1"] = mg.flat([s["exp_avg"] for s in st])
    rec["opt_state2"] = mg.flat([s["exp_avg_sq"] for s in st])
    rec["opt_step"] = float(st[0]["step"])
    rec["scalars"] = [(t, v) for t, v, _ in writer.scalars]
    return rec


def main():
    arrays, index = {}, {}
    cases = {
        "cp_acbc": dict(n=3, B=128, epochs=2, kw=dict(learning_rate=1e-3, batch_size=128, vf_coef=0.25)),
        "cp_acbc_gradacc": dict(n=2, B=64, epochs=2, kw=dict(learning_rate=3e-4, batch_size=64, vf_coef=0.5,
                                                              gradient_accumulation=True)),
    }
    for name, c in cases.items():
        torch.manual_seed(13)
        rng = np.random.default_rng(17)
        policy = ActorCritic(mg.cartpole_env())
        init = mg.flat(policy.parameters())
        batches = [mg.make_batch(policy, c["B"], rng, (4,), discrete_n=2) for _ in range(c["n"])]
        rec = run(policy, batches, c["kw"], c["epochs"])
        p = name + "/"
        for i, b in enumerate(batches):
            for f in ("obs", "actions", "values", "advantages", "returns"):
                arrays[f"{p}b{i}_{f}"] = getattr(b, f).numpy()
        arrays[p + "init"] = init
        arrays[p + "grads"] = np.stack(rec["grads"])
        arrays[p + "norms"] = np.array(rec["norms"], np.float64)
        arrays[p + "params"] = np.stack(rec["params"])
        arrays[p + "last_epoch_stats"] = np.array(
            [[s["loss"], s["pi_loss"], float(np.asarray(s["v_loss"]).reshape(-1)[0])] for s in rec["step_stats"]],
            np.float64)
        arrays[p + "opt_state1"] = rec["opt_state1"]
        arrays[p + "opt_state2"] = rec["opt_state2"]
        index[name] = dict(n=c["n"], B=c["B"], epochs=c["epochs"], kw=c["kw"], opt_step=rec["opt_step"],
                           scalars=rec["scalars"])
    arrays["index"] = np.array(json.dumps(index))
    np.savez_compressed(mg.HERE / "acbc_steps.npz", **arrays)
    print(f"acbc_steps.npz: {list(cases)}")


if __name__ == "__main__":
    main()
