"""LearningRateByKLDivergence (rl_algo_impls/ppo/learning_rate_by_kl_divergence.py:10-103) and the
schedule's target_kl phases (hyperparam_transitions.py:41-43,124-127,184-197) against the reference's
own outputs over scripted per-update train stats (tests/golden/lr_by_kl.json,
tests/golden/make_golden_lr_by_kl.py): the learning rate and target_kl after every update, bit-exact
(the same fp64 numpy expressions in the same order)."""
import json
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import GOLDEN

CASES = json.loads((GOLDEN / "lr_by_kl.json").read_text())


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_lr_by_kl_matches_reference(case):
    from rl_algo_impls_amd.callbacks import HyperparamTransitions, LearningRateByKLDivergence

    algo = SimpleNamespace(learning_rate=case["lr"], max_grad_norm=case["max_grad_norm"])
    cb = LearningRateByKLDivergence(algo, **case["kwargs"])
    callbacks = [cb]
    if "phases" in case:
        cfg = SimpleNamespace(n_timesteps=case["n"] * case["steps_per_update"])
        callbacks.append(HyperparamTransitions(cfg, None, algo, None, case["phases"], case["durations"],
                                               interpolate_method=case.get("interpolate", "linear"),
                                               lr_by_kl_callback=cb))
    lrs, tks = [], []
    for i in range(case["n"]):
        v = np.array(case["v_loss"][i]) if case.get("k3") else case["v_loss"][i]
        ts = SimpleNamespace(approx_kl=case["approx_kl"][i], v_loss=v, grad_norm=case["grad_norm"][i])
        for c in callbacks:
            c.on_step(timesteps_elapsed=case["steps_per_update"], train_stats=ts)
        lrs.append(float(algo.learning_rate))
        tks.append(float(cb.target_kl))
    assert lrs == case["learning_rate"]
    assert tks == case["target_kl"]


def test_lr_by_kl_bounds_are_checked():
    from rl_algo_impls_amd.callbacks import LearningRateByKLDivergence

    with pytest.raises(AssertionError, match="below min_lr"):
        LearningRateByKLDivergence(SimpleNamespace(learning_rate=1e-5, max_grad_norm=0.5), 0.01, min_lr=1e-4)
    with pytest.raises(AssertionError, match="above max_lr"):
        LearningRateByKLDivergence(SimpleNamespace(learning_rate=1e-3, max_grad_norm=0.5), 0.01, max_lr=1e-4)


def test_target_kl_phase_needs_the_callback():
    from rl_algo_impls_amd.callbacks import HyperparamTransitions

    algo = SimpleNamespace(learning_rate=1e-3)
    with pytest.raises(AssertionError):
        HyperparamTransitions(SimpleNamespace(n_timesteps=10), None, algo, None, [{"target_kl": 0.01}], [1.0])
