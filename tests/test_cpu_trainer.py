"""The CPU leg of bench.py (oracle/cpu_trainer.py, the "port" timed as `cpu_baseline`)
pinned to the reference's own outputs: a whole PPO learn_epoch on the CartPole MLP
(learn_epoch_cartpole.npz) and three NatureCNN minibatch steps at the Pong shape
(pong_steps.npz).  CPU only."""
import json
import sys

import numpy as np
import torch

from conftest import GOLDEN

import cpu_trainer
import oracle

sys.path.insert(0, str(GOLDEN))
from make_golden_pong import pong_init  # noqa: E402


def test_cpu_trainer_learn_epoch_matches_reference(golden):
    z = golden("learn_epoch_cartpole.npz")
    kw = json.loads(str(z["kw"]))
    adv = oracle.compute_advantages(z["rewards"], z["values"], z["episode_starts"], z["next_episode_starts"],
                                    z["next_values"], kw["gamma"], kw["gae_lambda"])
    np.testing.assert_array_equal(adv, z["advantages"])
    np.testing.assert_array_equal(adv + z["values"], z["returns"])
    torch.manual_seed(0)
    pol = cpu_trainer.MLPActorCritic()
    cpu_trainer.load_flat(pol, z["init"])
    ppo = cpu_trainer.CpuPPO(pol, lr=kw["learning_rate"], batch_size=kw["batch_size"], n_epochs=kw["n_epochs"],
                             clip_range=kw["clip_range"], ent_coef=kw["ent_coef"])
    fl = lambda a: torch.as_tensor(np.asarray(a).reshape((-1,) + np.asarray(a).shape[2:]))
    b = dict(obs=fl(z["obs"]), logprobs=fl(z["logprobs"]), actions=fl(z["actions"]), values=fl(z["values"]),
             advantages=fl(adv), returns=fl(adv + z["values"]))
    rows, means = ppo.update(b, perms=list(z["perms"]))
    np.testing.assert_allclose(rows[:, 6], z["grad_norms"], rtol=1e-5)
    np.testing.assert_allclose(cpu_trainer.flat_params(pol), z["params"], rtol=2e-4, atol=1e-6)
    ev = cpu_trainer.explained_variance(adv + z["values"], z["values"])
    got = [means[k] for k in ("loss", "pi_loss", "v_loss", "entropy_loss", "approx_kl", "clipped_frac")]
    got += [ev, means["grad_norm"]]
    np.testing.assert_allclose(got, z["losses"], rtol=2e-4, atol=1e-7)


def test_cpu_trainer_long_horizon_matches_reference(golden):
    """The oracle's CPU restatement over 2,048 DEPENDENT optimizer steps (learn_epoch_long.npz, the reference's
    own learn_epoch: 256 envs x 128 steps, batch 256 x 16 epochs): its GAE bit-exact, its first 64 gradient
    norms to 1e-5 and its final weights within 4x the reference's own one-ulp drift floor (the fixture's
    params_ulp) -- the same rule the device path meets in tests/test_gpu_trainer.py."""
    z = golden("learn_epoch_long.npz")
    kw = json.loads(str(z["kw"]))
    adv = oracle.compute_advantages(z["rewards"], z["values"], z["episode_starts"], z["next_episode_starts"],
                                    z["next_values"], kw["gamma"], kw["gae_lambda"])
    np.testing.assert_array_equal(adv, z["advantages"])
    torch.manual_seed(0)
    pol = cpu_trainer.MLPActorCritic()
    cpu_trainer.load_flat(pol, z["init"])
    ppo = cpu_trainer.CpuPPO(pol, lr=kw["learning_rate"], batch_size=kw["batch_size"], n_epochs=kw["n_epochs"],
                             clip_range=kw["clip_range"], ent_coef=kw["ent_coef"])
    fl = lambda a: torch.as_tensor(np.asarray(a).reshape((-1,) + np.asarray(a).shape[2:]))
    b = dict(obs=fl(z["obs"]), logprobs=fl(z["logprobs"]), actions=fl(z["actions"]), values=fl(z["values"]),
             advantages=fl(adv), returns=fl(adv + z["values"]))
    rows, _ = ppo.update(b, perms=[p.astype(np.int64) for p in z["perms"]])
    assert len(rows) == len(z["grad_norms"]) == 2048
    np.testing.assert_allclose(rows[:64, 6], z["grad_norms"][:64], rtol=1e-5)
    pr, pu = z["params"].astype(np.float64), z["params_ulp"].astype(np.float64)
    got = cpu_trainer.flat_params(pol).astype(np.float64)
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))
    drift, floor = rel(got, pr), rel(pu, pr)
    assert drift <= max(4 * floor, 1e-6), (drift, floor)


def test_cpu_trainer_pong_steps_match_reference(golden):
    z = golden("pong_steps.npz")
    meta = json.loads(str(z["index"]))
    kw = meta["kw"]
    pol = cpu_trainer.NatureCnnActorCritic()
    assert [list(p.shape) for p in pol.parameters()] == meta["shapes"]
    init = pong_init([tuple(s) for s in meta["shapes"]], meta["init_seed"])
    cpu_trainer.load_flat(pol, init)
    ppo = cpu_trainer.CpuPPO(pol, lr=kw["learning_rate"], batch_size=kw["batch_size"], n_epochs=1,
                             clip_range=kw["clip_range"], ent_coef=kw["ent_coef"], vf_coef=kw["vf_coef"])
    n = meta["n"]
    cat = lambda f: torch.as_tensor(np.concatenate([z[f"b{i}_{f}"] for i in range(n)]))
    b = {f: cat(f) for f in ("obs", "logprobs", "actions", "values", "advantages", "returns")}
    rows, _ = ppo.update(b, perms=[np.arange(n * meta["B"])])
    np.testing.assert_allclose(rows[:, 6], z["norms"], rtol=1e-5)
    ref = z["stats"]
    np.testing.assert_allclose(rows[:, [0, 1, 3, 4, 5, 2]], ref[:, :6], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(cpu_trainer.flat_params(pol), z["params"], rtol=1e-5, atol=1e-8)


def test_cpu_trainer_scaled_batch_matches_reference(golden):
    """SURVEY 8(d) batch policy (b) (batch = T*N/4): the CPU leg against the reference's own learn_epoch
    at four minibatches per epoch (learn_epoch_scaled.npz, make_golden_scaled.py)."""
    z = golden("learn_epoch_scaled.npz")
    p = "scaled/"
    kw = json.loads(str(z[p + "kw"]))
    adv = oracle.compute_advantages(z[p + "rewards"], z[p + "values"], z[p + "episode_starts"],
                                    z[p + "next_episode_starts"], z[p + "next_values"], kw["gamma"], kw["gae_lambda"])
    np.testing.assert_array_equal(adv, z[p + "advantages"])
    pol = cpu_trainer.MLPActorCritic()
    cpu_trainer.load_flat(pol, z[p + "init"])
    ppo = cpu_trainer.CpuPPO(pol, lr=kw["learning_rate"], batch_size=kw["batch_size"], n_epochs=kw["n_epochs"],
                             clip_range=kw["clip_range"], ent_coef=kw["ent_coef"])
    fl = lambda a: torch.as_tensor(np.asarray(a).reshape((-1,) + np.asarray(a).shape[2:]))
    b = dict(obs=fl(z[p + "obs"]), logprobs=fl(z[p + "logprobs"]), actions=fl(z[p + "actions"]),
             values=fl(z[p + "values"]), advantages=fl(adv), returns=fl(adv + z[p + "values"]))
    rows, means = ppo.update(b, perms=list(z[p + "perms"]))
    assert len(rows) == 8  # 2 epochs x 4 minibatches
    np.testing.assert_allclose(rows[:, 6], z[p + "grad_norms"], rtol=1e-5)
    np.testing.assert_allclose(cpu_trainer.flat_params(pol), z[p + "params"], rtol=2e-4, atol=1e-6)
