"""Golden vectors for LearningRateByKLDivergence (★ host-side schedule), generated
by running the REFERENCE ITSELF (read-only /root/reference, imported with ./stubs exactly as
make_golden.py does).  Only inputs and outputs are written (lr_by_kl.json).

    python tests/golden/make_golden_lr_by_kl.py

  LearningRateByKLDivergence      rl_algo_impls/ppo/learning_rate_by_kl_divergence.py:10-103
  target_kl phases                 rl_algo_impls/shared/callbacks/hyperparam_transitions.py:41-43,124-127,184-197
  callback order (lr_by_kl first)  rl_algo_impls/runner/train.py:193-213
  the *-lr-by-kl YAML              rl_algo_impls/hyperparams/ppo.yml:302-335

Per case: a scripted sequence of per-update train stats (approx_kl, v_loss scalar or K = 3 vector,
grad_norm), the callback kwargs, the algorithm's initial learning_rate / max_grad_norm, optional
HyperparamTransitions phases, and after every update the algorithm's learning_rate and the
callback's target_kl.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

CASES = [
    dict(name="defaults", lr=1e-3, max_grad_norm=0.5, kwargs=dict(target_kl=0.01), n=30, kl_scale=0.01),
    # the Atari *-lr-by-kl configs (ppo.yml:302-335) with their target_kl schedule 0.01 -> 0.001
    dict(name="atari_lr_by_kl", lr=2.5e-4, max_grad_norm=0.5,
         kwargs=dict(target_kl=0.01, min_decrease_fraction=0.9, max_increase_fraction=1.05,
                     no_increase_on_max_grad_norm=True),
         phases=[{"target_kl": 0.01}, {"target_kl": 0.001}], durations=[0.8, 0.2, 0], n=40, kl_scale=0.006),
    dict(name="vloss_threshold_bounds", lr=3e-4, max_grad_norm=0.8,
         kwargs=dict(target_kl=0.02, moving_window_size=3, v_loss_threshold=1.1, v_loss_fast_moving_window_size=3,
                     v_loss_slow_moving_window_size=8, min_lr=1e-4, max_lr=6e-4), n=40, kl_scale=0.01, k3=True),
    dict(name="cosine_phases", lr=5e-4, max_grad_norm=0.5,
         kwargs=dict(target_kl=0.02, max_increase_fraction=1.1),
         phases=[{"target_kl": 0.02}, {"target_kl": 0.005}], durations=[0.3, 0.5, 0.2], interpolate="cosine",
         n=25, kl_scale=0.02),
]


def main():
    import make_golden as mg  # noqa: F401  (stubs + reference on sys.path)
    from rl_algo_impls.ppo.learning_rate_by_kl_divergence import LearningRateByKLDivergence
    from rl_algo_impls.shared.callbacks.hyperparam_transitions import HyperparamTransitions

    rng = np.random.default_rng(17)
    out = []
    for c in CASES:
        n = c["n"]
        kl = (c["kl_scale"] * rng.lognormal(0.0, 0.6, n)).tolist()
        if c.get("k3"):
            v_loss = (np.linspace(1.0, 3.0, n)[:, None] * rng.lognormal(0.0, 0.3, (n, 3))).tolist()
        else:
            v_loss = rng.lognormal(0.0, 0.5, n).tolist()
        grad_norm = (c["max_grad_norm"] * rng.lognormal(0.0, 0.4, n)).tolist()
        algo = SimpleNamespace(learning_rate=c["lr"], max_grad_norm=c["max_grad_norm"])
        cb = LearningRateByKLDivergence(algo, **c["kwargs"])
        callbacks = [cb]
        steps_per_update = 1000
        if "phases" in c:
            cfg = SimpleNamespace(n_timesteps=n * steps_per_update)
            callbacks.append(HyperparamTransitions(cfg, None, algo, None, c["phases"], c["durations"],
                                                   interpolate_method=c.get("interpolate", "linear"),
                                                   lr_by_kl_callback=cb))
        lrs, tks = [], []
        for i in range(n):
            ts = SimpleNamespace(approx_kl=kl[i], v_loss=np.array(v_loss[i]) if c.get("k3") else v_loss[i],
                                 grad_norm=grad_norm[i])
            for callback in callbacks:  # PPO.learn's order (rl_algo_impls/ppo/ppo.py:430-438)
                callback.on_step(timesteps_elapsed=steps_per_update, train_stats=ts)
            lrs.append(float(algo.learning_rate))
            tks.append(float(cb.target_kl))
        out.append(dict(c, approx_kl=kl, v_loss=v_loss, grad_norm=grad_norm, steps_per_update=steps_per_update,
                        learning_rate=lrs, target_kl=tks))
        print(c["name"], lrs[-1], tks[-1])
    (HERE / "lr_by_kl.json").write_text(json.dumps(out))


if __name__ == "__main__":
    main()
