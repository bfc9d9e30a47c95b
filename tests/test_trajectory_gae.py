"""Per-trajectory GAE operators: TrajectoryBuilder
(rl_algo_impls/rollout/trajectory.py:56-92) and DiscreteSkipsTrajectoryBuilder
(rl_algo_impls/rollout/discrete_skips_trajectory_builder.py:26-109).

CPU: the oracle restatements against the reference-generated fixtures (traj_cases.npz,
tests/golden/make_golden_traj.py).  GPU: the builders of rl_algo_impls_amd.trajectory, driven with
the fixtures' inputs, against the same fixtures (bit-exact in exact mode) — one launch for all
trajectories of a case — plus large ragged batches against the oracle and the edge cases.
"""
import json

import numpy as np
import pytest
import torch

from conftest import ROOT

import oracle as O

GOLD = ROOT / "tests" / "golden"


@pytest.fixture(scope="module")
def traj():
    return np.load(GOLD / "traj_cases.npz"), json.loads((GOLD / "traj_cases.json").read_text())


def _g(v):
    return np.array(v, dtype=np.float64) if isinstance(v, list) else v


def test_oracle_trajectory_builder_bit_exact(traj):
    d, meta = traj
    for c in meta["cases"]:
        for j in range(c["n"]):
            p = f"{c['name']}_{j}_"
            nv = d[p + "nv"] if p + "nv" in d else None
            a = O.trajectory_advantages(d[p + "rew"], d[p + "val"], d[p + "dones"], _g(c["gamma"]),
                                        _g(c["gae_lambda"]), nv)
            np.testing.assert_array_equal(a, d[p + "adv"], err_msg=p)


def test_oracle_skips_builder_bit_exact(traj):
    d, meta = traj
    for c in meta["skip_cases"]:
        for j in range(c["n"]):
            p = f"{c['name']}_{j}_"
            nv = d[p + "nv"] if p + "nv" in d else None
            a = O.skips_advantages(d[p + "acc_rew"], d[p + "val"], d[p + "steps"], bool(d[p + "done"]),
                                   _g(c["gamma"]), _g(c["gae_lambda"]), nv)
            np.testing.assert_array_equal(a, d[p + "adv"], err_msg=p)


def _skips_builder(d, p, K, gamma):
    """Replay a fixture's step_add / step_no_add script into our builder (host accumulation)."""
    from rl_algo_impls_amd.trajectory import DiscreteSkipsTrajectoryBuilder

    rew, val, skips, done_end = d[p + "rew_in"], d[p + "val"], d[p + "skips"], bool(d[p + "done"])
    rew_in = [float(x) for x in rew] if K == 0 else list(rew)
    b = DiscreteSkipsTrajectoryBuilder()
    i, n_add = 0, len(val)
    for a_i in range(n_add):
        last_add = a_i == n_add - 1
        v = np.float32(val[a_i]) if K == 0 else val[a_i]
        b.step_add(np.zeros(2, np.float32), rew_in[i], done_end and last_add and skips[a_i] == 0, v,
                   np.float32(0), np.int64(0), None, gamma)
        i += 1
        for s_i in range(int(skips[a_i])):
            b.step_no_add(rew_in[i], done_end and last_add and s_i == skips[a_i] - 1, gamma)
            i += 1
    return b


def test_skips_builder_host_accumulation_matches_reference(traj):
    """The host-side reward discounting of step_no_add (CPU only, no kernel)."""
    d, meta = traj
    for c in meta["skip_cases"]:
        for j in range(c["n"]):
            p = f"{c['name']}_{j}_"
            b = _skips_builder(d, p, c["K"], _g(c["gamma"]))
            np.testing.assert_array_equal(np.array(b.rewards, dtype=np.float32), d[p + "acc_rew"], err_msg=p)
            np.testing.assert_array_equal(np.array(b.steps_elapsed, dtype=np.int32), d[p + "steps"])
            assert b.done == bool(d[p + "done"])


@pytest.mark.gpu
def test_trajectory_builder_kernel_bit_exact(traj):
    from rl_algo_impls_amd.trajectory import TrajectoryBuilder, build_trajectories

    d, meta = traj
    for c in meta["cases"]:
        builders, nvs, want = [], [], []
        for j in range(c["n"]):
            p = f"{c['name']}_{j}_"
            b = TrajectoryBuilder()
            rew, val, dones = d[p + "rew"], d[p + "val"], d[p + "dones"]
            for t in range(len(rew)):
                v = np.float32(val[t]) if c["K"] == 0 else val[t]
                b.add(np.zeros(2, np.float32), rew[t], bool(dones[t]), v, np.float32(0), np.int64(0), None)
            builders.append(b)
            nvs.append(d[p + "nv"] if p + "nv" in d else None)
            want.append(d[p + "adv"])
        # one launch for the whole case
        trs = build_trajectories(builders, _g(c["gamma"]), _g(c["gae_lambda"]), nvs)
        for tr, w in zip(trs, want):
            assert tr.advantages.shape == w.shape
            np.testing.assert_array_equal(tr.advantages, w, err_msg=c["name"])
        # the per-builder reference call
        tr0 = builders[-1].trajectory(_g(c["gamma"]), _g(c["gae_lambda"]), next_values=nvs[-1])
        np.testing.assert_array_equal(tr0.advantages, want[-1])


@pytest.mark.gpu
def test_skips_builder_kernel_bit_exact(traj):
    from rl_algo_impls_amd.trajectory import build_trajectories

    d, meta = traj
    for c in meta["skip_cases"]:
        builders, nvs, want = [], [], []
        for j in range(c["n"]):
            p = f"{c['name']}_{j}_"
            builders.append(_skips_builder(d, p, c["K"], _g(c["gamma"])))
            nvs.append(d[p + "nv"] if p + "nv" in d else None)
            want.append(d[p + "adv"])
        trs = build_trajectories(builders, _g(c["gamma"]), _g(c["gae_lambda"]), nvs)
        for tr, w in zip(trs, want):
            np.testing.assert_array_equal(tr.advantages, w, err_msg=c["name"])


@pytest.mark.gpu
@pytest.mark.parametrize("K,vec", [(0, False), (3, True), (3, False)])
def test_large_ragged_batches_vs_oracle(K, vec):
    """1,000 trajectories of 1..700 rows (one launch) against the oracle, exact and fast modes."""
    from rl_algo_impls_amd.trajectory import DiscreteSkipsTrajectoryBuilder, TrajectoryBuilder, build_trajectories
    from rl_algo_impls_amd.gae import FAST

    rng = np.random.default_rng(K + 10 * vec)
    shape = () if K == 0 else (K,)
    gamma = np.array([0.99, 0.995, 0.999]) if vec else 0.99
    lam = np.array([0.95, 0.9, 0.99]) if vec else 0.95
    lens = rng.integers(1, 700, 1000)
    lens[:3] = [1, 64, 65]
    tbs, sks, nvs = [], [], []
    for i, L in enumerate(lens):
        rew = rng.standard_normal((L,) + shape).astype(np.float32)
        val = rng.standard_normal((L,) + shape).astype(np.float32)
        dones = rng.random(L) < 0.02
        tb, sk = TrajectoryBuilder(), DiscreteSkipsTrajectoryBuilder()
        for t in range(L):
            v = np.float32(val[t]) if K == 0 else val[t]
            tb.add(None, rew[t], bool(dones[t]), v, 0.0, 0, None)
            sk.step_add(None, rew[t], bool(i % 2 == 0 and t == L - 1), v, 0.0, 0, None, gamma)
            for _ in range(int(rng.integers(0, 4))):
                if sk.done:
                    break
                sk.step_no_add(rew[t] * 0.5, False, gamma)
        tbs.append(tb)
        sks.append(sk)
        nvs.append(rng.standard_normal(shape).astype(np.float32))
    got = build_trajectories(tbs, gamma, lam, nvs)
    for b, nv, tr in zip(tbs, nvs, got):
        want = O.trajectory_advantages(np.array(b.rewards, np.float32), np.array(b.values), np.array(b.dones),
                                       gamma, lam, nv)
        np.testing.assert_array_equal(tr.advantages, want)
    got = build_trajectories(sks, gamma, lam, nvs)
    fast = build_trajectories(sks, gamma, lam, nvs, mode=FAST)
    for b, nv, tr, tf in zip(sks, nvs, got, fast):
        args = (np.array(b.rewards, np.float32), np.array(b.values), np.array(b.steps_elapsed, np.int32), b.done,
                gamma, lam, nv)
        np.testing.assert_array_equal(tr.advantages, O.skips_advantages(*args))
        if K and not vec:  # fast mode = numpy<2 legacy promotion for K columns + scalar gamma
            np.testing.assert_array_equal(tf.advantages, O.skips_advantages(*args, legacy_promotion=True))
        else:
            np.testing.assert_allclose(tf.advantages, tr.advantages, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_trajectory_edge_cases_and_errors():
    from rl_algo_impls_amd.trajectory import DiscreteSkipsTrajectoryBuilder, TrajectoryBuilder, build_trajectories

    assert build_trajectories([], 0.99, 0.95) == []
    b = TrajectoryBuilder()
    b.add(None, 1.0, True, np.float32(0.5), 0.0, 0, None)  # single terminal step: adv = r - V
    tr = b.trajectory(0.99, 0.95)
    assert tr.advantages.dtype == np.float32 and tr.advantages[0] == np.float32(0.5)
    sk = DiscreteSkipsTrajectoryBuilder()
    sk.step_add(None, 1.0, False, np.float32(0.0), 0.0, 0, None, 0.99)
    with pytest.raises(AssertionError, match="next_values"):
        sk.trajectory(0.99, 0.95)
    bad = TrajectoryBuilder()
    bad.add(None, 1.0, False, 0.5, 0.0, 0, None)  # Python float value -> float64 array
    with pytest.raises(ValueError, match="float32"):
        bad.trajectory(0.99, 0.95)
    with pytest.raises(TypeError):
        build_trajectories([b, sk], 0.99, 0.95)
