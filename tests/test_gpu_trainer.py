"""End-to-end parity of the MI355X PPO/A2C update with the reference's own
PPO.learn_epoch / A2C.learn (golden fixtures from tests/golden/make_golden.py),
through the C ABI kernels + PyTorch-ROCm network."""
import json

import numpy as np
import pytest
import torch

from rl_algo_impls_amd.a2c import A2C
from rl_algo_impls_amd.ppo import PPO
from rl_algo_impls_amd.rollout import Batch, DeviceRollout, SyncStepRolloutGenerator
import make_golden_networks as nets

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class Recorder:
    def __init__(self):
        self.scalars = {}

    def add_scalar(self, tag, value, global_step=None):
        self.scalars[tag] = float(value)


class FixedDeviceRollout:
    def __init__(self, batches):
        self.batches = batches

    @property
    def total_steps(self):
        return sum(len(b) for b in self.batches)

    def num_minibatches(self, bs):
        return len(self.batches)

    def minibatches(self, bs, shuffle=True):
        return iter(self.batches)

    def explained_variance(self):
        y = torch.cat([b.returns for b in self.batches]).double()
        p = torch.cat([b.values for b in self.batches]).double()
        return float(1 - torch.var(y - p, unbiased=False) / torch.var(y, unbiased=False))


class EpochFixedRollout(FixedDeviceRollout):
    """The fixed minibatches as one epoch copy in order (no shuffle): the whole-epoch kernels
    (rai_mlp_wide_epoch) take minibatch i as rows [i B, (i + 1) B) of it."""

    def epoch_batch(self, shuffle=True):
        cat = lambda f: torch.cat([getattr(b, f) for b in self.batches]).contiguous()
        return Batch(cat("obs"), cat("logprobs"), cat("actions"), None, None, cat("values"), cat("advantages"),
                     cat("returns"))


def _device_batches(z, name, n, with_logp=True):
    out = []
    for i in range(n):
        p = f"{name}/b{i}_"
        t = lambda k: torch.from_numpy(z[p + k]).to(DEV)
        out.append(Batch(t("obs"), t("logprobs") if with_logp else None, t("actions"), None, None, t("values"),
                         t("advantages"), t("returns")))
    return out


@pytest.mark.parametrize("wide", [True, False, "epoch"], ids=["wide_kernels", "pytorch_network", "wide_epoch"])
@pytest.mark.parametrize("name", ["cp_default", "cp_vclip_ent", "cp_gradacc", "cp_klcut", "hc_gauss", "mc_mrw",
                                  "mc_after", "mc_huber_w"])
def test_ppo_minibatch_steps_match_reference(golden, name, wide):
    """Per-minibatch path against the reference's PPO steps.  The MLP cases (cp_*, hc_gauss: 64-wide
    actor/critic) run through the fused wide-MLP kernels (mlp_wide.py) or the PyTorch network +
    autograd; the multi-critic cases (mc_*) always take the PyTorch network.  wide_epoch: the same
    minibatches as ONE whole-epoch launch (rai_mlp_wide_epoch, csrc/mlp_wide_epoch.hip) where its
    scope covers the case (hc_gauss: B = 64, Gaussian head, Adam, no gradient accumulation)."""
    if wide == "epoch" and name != "hc_gauss":
        pytest.skip("outside rai_mlp_wide_epoch's scope (B > 64, gradient accumulation, kl_cutoff or K > 1)")
    z = golden("ppo_steps.npz")
    meta = json.loads(str(z["index"]))[name]
    policy = nets.build(meta["policy"])
    nets.load_flat(policy, z[f"{name}/init"])
    policy = policy.to(DEV)
    kw = dict(meta["kw"])
    algo = PPO(policy, DEV, Recorder(), n_epochs=1, **kw)
    algo.use_wide = bool(wide)
    bs = _device_batches(z, name, meta["n"])
    r = EpochFixedRollout(bs) if wide == "epoch" else FixedDeviceRollout(bs)
    stats, norms, K = algo.update(r)
    assert (getattr(algo, "_we_ws", None) is not None) == (wide == "epoch"), "whole-epoch kernel path"
    ref_params = z[f"{name}/params"]
    got = algo.flat.flat.cpu().numpy()
    # Adam's first steps normalise g/|g|; tolerance covers fp32 reduction-order
    # differences between the CPU reference and the GPU network/backward.
    np.testing.assert_allclose(got, ref_params[-1], rtol=1e-4, atol=float(kw["learning_rate"]) * 2e-3,
                               err_msg=name)
    np.testing.assert_allclose(norms, z[f"{name}/norms"], rtol=1e-4, err_msg=name)
    ref_stats = z[f"{name}/stats"]
    np.testing.assert_allclose(stats[:, :5], ref_stats[:, :5], rtol=2e-4, atol=2e-6, err_msg=name)
    np.testing.assert_allclose(stats[:, 5:5 + K] if meta["kw"].get("vf_weights") is None else
                               stats[:, 5:5 + K] @ np.asarray(meta["kw"]["vf_weights"])[:, None],
                               ref_stats[:, 5:5 + (K if meta["kw"].get("vf_weights") is None else 1)],
                               rtol=2e-4, atol=2e-6, err_msg=name)
    sd = algo.optimizer.state_dict()
    assert float(sd["state"][0]["step"]) == meta["opt_step"]
    s1 = torch.cat([s["exp_avg"].reshape(-1) for s in sd["state"].values()]).cpu().numpy()
    np.testing.assert_allclose(s1, z[f"{name}/opt_state1"], rtol=2e-3, atol=2e-7, err_msg=name)
    assert (algo._wide not in (None, False)) == (wide and not name.startswith("mc_")), "wide path not taken"


@pytest.mark.parametrize("generic", [False, True], ids=["fused_mlp_kernel", "generic_path"])
def test_learn_epoch_matches_reference_with_injected_rollout(golden, generic):
    z = golden("learn_epoch_cartpole.npz")
    kw = json.loads(str(z["kw"]))
    policy = nets.build("cartpole")
    nets.load_flat(policy, z["init"])
    policy = policy.to(DEV)
    rec = Recorder()
    algo = PPO(policy, DEV, rec, **kw)
    algo.force_generic = generic
    assert (algo.fused_mlp_spec() is None) == generic
    perms = list(z["perms"])
    t = lambda k: torch.from_numpy(z[k]).to(DEV)
    r = DeviceRollout(DEV, t("next_episode_starts"), t("next_values"), t("obs"), t("actions"), t("rewards"),
                      t("episode_starts"), t("values"), t("logprobs"), None, kw["gamma"], kw["gae_lambda"],
                      perm_source=lambda n: torch.from_numpy(perms.pop(0)))
    np.testing.assert_array_equal(r.advantages.cpu().numpy(), z["advantages"])
    np.testing.assert_array_equal(r.returns.cpu().numpy(), z["returns"])

    class Gen:
        def rollout(self, gamma, gae_lambda):
            return r

    algo.learn_epoch(0, 256, Gen(), None)
    assert not perms
    np.testing.assert_allclose(algo.flat.flat.cpu().numpy(), z["params"], rtol=2e-4, atol=5e-6)
    names = ("loss", "pi_loss", "v_loss", "entropy_loss", "approx_kl", "clipped_frac", "explained_var", "grad_norm")
    got = np.array([rec.scalars[f"losses/{k}"] for k in names])
    np.testing.assert_allclose(got, z["losses"], rtol=2e-4, atol=2e-6)
    assert rec.scalars["train/steps_per_second"] > 0


class FixedEpochRollout(FixedDeviceRollout):
    """Exposes epoch_batch() so PPO takes the fused rai_mlp_ppo_epoch path."""

    def epoch_batch(self, shuffle=True):
        cat = lambda f: torch.cat([getattr(b, f) for b in self.batches])
        return Batch(cat("obs"), cat("logprobs"), cat("actions"), None, None, cat("values"), cat("advantages"),
                     cat("returns"))


@pytest.mark.parametrize("name", ["cp_default", "cp_vclip_ent"])
def test_fused_mlp_kernel_matches_reference_steps(golden, name):
    z = golden("ppo_steps.npz")
    meta = json.loads(str(z["index"]))[name]
    policy = nets.build(meta["policy"])
    nets.load_flat(policy, z[f"{name}/init"])
    policy = policy.to(DEV)
    algo = PPO(policy, DEV, Recorder(), n_epochs=1, **meta["kw"])
    assert algo.fused_mlp_spec() is not None
    r = FixedEpochRollout(_device_batches(z, name, meta["n"]))
    stats, norms, K = algo.update(r)
    np.testing.assert_allclose(algo.flat.flat.cpu().numpy(), z[f"{name}/params"][-1], rtol=1e-4,
                               atol=float(meta["kw"]["learning_rate"]) * 2e-3)
    np.testing.assert_allclose(norms, z[f"{name}/norms"], rtol=1e-4)
    np.testing.assert_allclose(stats[:, :6], z[f"{name}/stats"][:, :6], rtol=2e-4, atol=2e-6)
    np.testing.assert_allclose(algo.optimizer.state1.cpu().numpy(), z[f"{name}/opt_state1"], rtol=2e-3, atol=2e-7)
    assert algo.optimizer.step_count == meta["opt_step"]


def test_fused_matches_generic_on_large_rollout():
    """Same permutations, same rollout: fused single-launch epoch vs the per-minibatch
    PyTorch path, 4096 envs x 16 steps, batch 256 (256 optimizer steps)."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    results = []
    for generic in (False, True):
        torch.manual_seed(3)
        env = SyntheticVecEnv(4096, "cartpole", seed=5)
        policy = ActorCritic(env).to(DEV)
        gen = SyncStepRolloutGenerator(policy, env, n_steps=16, seed=11)
        algo = PPO(policy, DEV, None, batch_size=256, n_epochs=1, learning_rate=1e-4, gamma=0.98, gae_lambda=0.8)
        algo.force_generic = generic
        r = gen.rollout(gamma=0.98, gae_lambda=0.8)
        g = torch.Generator(device=DEV)
        g.manual_seed(123)
        r._perm_source = lambda n: torch.randperm(n, device=DEV, generator=g)
        stats, norms, _ = algo.update(r)
        results.append((algo.flat.flat.cpu().numpy(), stats, norms))
    (pf, sf, nf), (pg, sg, ng) = results
    np.testing.assert_allclose(nf, ng, rtol=1e-3)
    np.testing.assert_allclose(sf[:, :6], sg[:, :6], rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(pf, pg, rtol=2e-3, atol=2e-5)


def test_fused_epoch_full_c2_horizon_drift():
    """Config C2's whole update — 4096 envs x 128 steps, batch 256, 20 epochs = 40,960 dependent
    optimizer steps (rl_algo_impls/hyperparams/ppo.yml:1-23 at the BASELINE shape) — through the
    fused epoch kernel vs the generic graph-replayed path, identical rollout and permutations.

    Over 40,960 steps no fp32 implementation tracks another to a fixed tolerance: any rounding
    difference (summation order in the network, the loss reductions, Adam's sqrt/divide) is
    carried forward by the optimiser.  The bound is therefore relative to the trajectory's own
    sensitivity: the generic path re-run from weights perturbed by one ulp sets the noise floor,
    and the fused kernel may drift from the generic path by no more than a small multiple of it.
    The measured figures are printed for DESIGN.md."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(3)
    env = SyntheticVecEnv(4096, "cartpole", seed=5)
    policy = ActorCritic(env).to(DEV)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=128, seed=11)
    r = gen.rollout(gamma=0.98, gae_lambda=0.8)
    p0 = torch.nn.utils.parameters_to_vector(policy.parameters()).detach().clone()
    runs = {}
    for name, generic, perturb in (("fused", False, False), ("generic", True, False),
                                   ("generic_ulp", True, True)):
        start = p0.clone()
        if perturb:
            start = torch.nextafter(start, torch.full_like(start, float("inf")))
        torch.nn.utils.vector_to_parameters(start, policy.parameters())
        algo = PPO(policy, DEV, None, batch_size=256, n_epochs=20, learning_rate=1e-3, gamma=0.98,
                   gae_lambda=0.8, clip_range=0.2, ent_coef=0.0)
        algo.force_generic = generic
        assert (algo.fused_mlp_spec() is None) == generic
        g = torch.Generator(device=DEV)
        g.manual_seed(123)
        r._perm_source = lambda n: torch.randperm(n, device=DEV, generator=g)
        stats, norms, _ = algo.update(r)
        torch.cuda.synchronize()
        assert algo.optimizer.step_count == 40960
        runs[name] = (algo.flat.flat.detach().cpu().double().numpy(), stats.astype(np.float64), norms)
    pf, sf, nf = runs["fused"]
    pg, sg, ng = runs["generic"]
    pu, su, nu = runs["generic_ulp"]
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))
    drift, floor = rel(pf, pg), rel(pu, pg)
    last = slice(-2048, None)  # the last epoch's 2,048 minibatch stats (what TrainStats reports)
    stat_drift = np.abs(sf[last, :6].mean(0) - sg[last, :6].mean(0))
    stat_floor = np.abs(su[last, :6].mean(0) - sg[last, :6].mean(0))
    print(f"C2 horizon: |p_fused - p_generic|/|p| = {drift:.3e}, ulp floor {floor:.3e}; "
          f"max abs param diff fused {np.abs(pf - pg).max():.3e} floor {np.abs(pu - pg).max():.3e}; "
          f"last-epoch mean stats diff fused {stat_drift} floor {stat_floor}")
    assert np.isfinite(pf).all() and np.isfinite(sf).all()
    assert drift <= max(4 * floor, 1e-5), (drift, floor)
    # the reported TrainStats (means over the last epoch) agree within the same floor
    assert (stat_drift <= np.maximum(4 * stat_floor, 1e-4 * (1 + np.abs(sg[last, :6].mean(0))))).all()


def _long_fixture_update(z, generic, ulp=False):
    """The reference's rollout and permutations of learn_epoch_long.npz through PPO.learn_epoch on the
    device (fused epoch kernel or generic path); returns (final params f64, per-step norms, losses)."""
    kw = json.loads(str(z["kw"]))
    policy = nets.build("cartpole")
    init = torch.from_numpy(z["init"])
    if ulp:
        init = torch.nextafter(init, torch.full_like(init, float("inf")))
    nets.load_flat(policy, init.numpy())
    policy = policy.to(DEV)
    rec = Recorder()
    algo = PPO(policy, DEV, rec, **kw)
    algo.force_generic = generic
    assert (algo.fused_mlp_spec() is None) == generic
    perms = [p.astype(np.int64) for p in z["perms"]]
    t = lambda k: torch.from_numpy(z[k]).to(DEV)
    r = DeviceRollout(DEV, t("next_episode_starts"), t("next_values"), t("obs"), t("actions"), t("rewards"),
                      t("episode_starts"), t("values"), t("logprobs"), None, kw["gamma"], kw["gae_lambda"],
                      perm_source=lambda n: torch.from_numpy(perms.pop(0)))
    np.testing.assert_array_equal(r.advantages.cpu().numpy(), z["advantages"])
    np.testing.assert_array_equal(r.returns.cpu().numpy(), z["returns"])
    captured = []
    real_update = algo.update

    def update(rr):
        out = real_update(rr)
        captured.append(np.asarray(out[1], np.float64))
        return out

    algo.update = update

    class Gen:
        def rollout(self, gamma, gae_lambda):
            return r

    algo.learn_epoch(0, r.total_steps, Gen(), None)
    torch.cuda.synchronize()
    assert not perms and algo.optimizer.step_count == len(z["grad_norms"]) == 2048
    names = ("loss", "pi_loss", "v_loss", "entropy_loss", "approx_kl", "clipped_frac", "explained_var", "grad_norm")
    losses = np.array([rec.scalars[f"losses/{k}"] for k in names])
    return algo.flat.flat.detach().cpu().double().numpy(), captured[0], losses


@pytest.mark.parametrize("generic", [False, True], ids=["fused_mlp_kernel", "generic_path"])
def test_long_horizon_matches_reference_learn_epoch(golden, generic):
    """2,048 DEPENDENT optimizer steps pinned to the reference itself (learn_epoch_long.npz, made by
    tests/golden/make_golden_long.py from rl_algo_impls/ppo/ppo.py:214-447): 256 envs x 128 steps at the
    YAML minibatch (256 rows; the default C2 epoch kernel's geometry), 16 epochs, the reference's rollout
    and permutations injected.  The bound is the trajectory's own sensitivity: the reference re-run from
    weights one ulp up (stored in the fixture) and the device path re-run the same way; the device update
    may drift from the reference by no more than a small multiple of the larger floor."""
    z = golden("learn_epoch_long.npz")
    pd, nd, ld = _long_fixture_update(z, generic)
    pu, nu, lu = _long_fixture_update(z, generic, ulp=True)
    pr, pr_u = z["params"].astype(np.float64), z["params_ulp"].astype(np.float64)
    nr, nr_u = z["grad_norms"], z["grad_norms_ulp"]
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))
    drift, floor_ref, floor_dev = rel(pd, pr), rel(pr_u, pr), rel(pu, pd)
    floor = max(floor_ref, floor_dev)
    norm_drift = np.abs(nd - nr) / nr
    norm_floor = np.maximum(np.abs(nr_u - nr) / nr, np.abs(nu - nd) / nd)
    print(f"long horizon ({'generic' if generic else 'fused'}): |p_dev - p_ref|/|p_ref| = {drift:.3e}, ulp floors "
          f"ref {floor_ref:.3e} dev {floor_dev:.3e}; max abs param diff {np.abs(pd - pr).max():.3e}; "
          f"grad-norm rel diff first 64 max {norm_drift[:64].max():.3e}, last 128 mean {norm_drift[-128:].mean():.3e} "
          f"(floor {norm_floor[-128:].mean():.3e}); losses {ld} vs {z['losses']}")
    assert np.isfinite(pd).all()
    assert drift <= max(4 * floor, 1e-5), (drift, floor_ref, floor_dev)
    np.testing.assert_allclose(nd[:64], nr[:64], rtol=1e-4)
    assert norm_drift[-128:].mean() <= max(4 * norm_floor[-128:].mean(), 1e-4)
    # the logged losses (TrainStats means over the last epoch, ppo.py:379-427)
    loss_floor = np.abs(lu - ld)
    assert (np.abs(ld - z["losses"]) <= np.maximum(4 * loss_floor, 2e-4 * (1 + np.abs(z["losses"])))).all(), \
        (ld, z["losses"], lu)


def _long_wide_update(z, ulp=False):
    """learn_epoch_long_wide.npz's rollout and permutations through PPO.learn_epoch on the device: the C4
    policy ([256, 256] ReLU, Gaussian head), whose epochs run as ONE rai_mlp_wide_epoch launch each."""
    from rl_algo_impls_amd.policy import ActorCritic

    kw = json.loads(str(z["kw"]))
    policy = ActorCritic(nets.halfcheetah_env(), **json.loads(str(z["policy"])))
    init = torch.from_numpy(z["init"])
    if ulp:
        init = torch.nextafter(init, torch.full_like(init, float("inf")))
    nets.load_flat(policy, init.numpy())
    policy = policy.to(DEV)
    rec = Recorder()
    algo = PPO(policy, DEV, rec, **kw)
    perms = [p.astype(np.int64) for p in z["perms"]]
    t = lambda k: torch.from_numpy(z[k]).to(DEV)
    r = DeviceRollout(DEV, t("next_episode_starts"), t("next_values"), t("obs"), t("actions"), t("rewards"),
                      t("episode_starts"), t("values"), t("logprobs"), None, kw["gamma"], kw["gae_lambda"],
                      perm_source=lambda n: torch.from_numpy(perms.pop(0)))
    np.testing.assert_array_equal(r.advantages.cpu().numpy(), z["advantages"])
    captured = []
    real_update = algo.update

    def update(rr):
        out = real_update(rr)
        captured.append(np.asarray(out[1], np.float64))
        return out

    algo.update = update

    class Gen:
        def rollout(self, gamma, gae_lambda):
            return r

    algo.learn_epoch(0, r.total_steps, Gen(), None)
    torch.cuda.synchronize()
    assert getattr(algo, "_we_ws", None) is not None, "the whole-epoch kernel path"
    assert not perms and algo.optimizer.step_count == len(z["grad_norms"]) == 2048
    return algo.flat.flat.detach().cpu().double().numpy(), captured[0]


def test_long_horizon_wide_epoch_matches_reference_learn_epoch(golden):
    """2,048 DEPENDENT optimizer steps of the C4-class whole-epoch kernel (rai_mlp_wide_epoch, C4's policy and
    hyperparameters) pinned to the reference itself (learn_epoch_long_wide.npz, tests/golden/make_golden_long.py:
    64 envs x 32 steps, batch 64, 64 epochs, the reference's rollout and permutations injected).  This
    trajectory is far more sensitive than C2's: at lr 2e-5 Adam moves every weight by ~lr per step
    whatever its gradient's size, so weights whose gradients are noise flip direction under a one-ulp
    change of the start (the reference's own ulp floor is 7.6e-2 of the update).  So: the first 64 steps'
    gradient norms to 1e-4 (before divergence compounds), and the final update (params - init) within
    4x the larger ulp floor (reference's, device's) of the reference's update."""
    z = golden("learn_epoch_long_wide.npz")
    init = z["init"].astype(np.float64)
    pd, nd = _long_wide_update(z)
    pu, nu = _long_wide_update(z, ulp=True)
    pr, pr_u = z["params"].astype(np.float64), z["params_ulp"].astype(np.float64)
    nr = z["grad_norms"]
    upd = lambda p: p - init
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(upd(b)))
    drift, floor_ref, floor_dev = rel(pd, pr), rel(pr_u, pr), rel(pu, pd)
    print(f"long horizon (wide epoch): |p_dev - p_ref| / |update| = {drift:.3e}, ulp floors ref {floor_ref:.3e} "
          f"dev {floor_dev:.3e}; first-64 grad-norm rel diff max {np.max(np.abs(nd[:64] - nr[:64]) / nr[:64]):.3e}")
    assert np.isfinite(pd).all()
    np.testing.assert_allclose(nd[:64], nr[:64], rtol=1e-4)
    assert drift <= 4 * max(floor_ref, floor_dev), (drift, floor_ref, floor_dev)


def test_a2c_step_matches_reference(golden):
    z = golden("a2c_step.npz")
    policy = nets.build("cartpole")
    nets.load_flat(policy, z["init"])
    policy = policy.to(DEV)
    algo = A2C(policy, DEV, None, learning_rate=7e-4, ent_coef=0.01)
    t = lambda k: torch.from_numpy(z[k]).to(DEV)
    b = Batch(t("obs"), None, t("actions"), None, None, t("values"), t("advantages"), t("returns"))
    r = FixedDeviceRollout([b])

    class Gen:
        def rollout(self, gamma, gae_lambda):
            return r

    algo.learn(r.total_steps, Gen())
    np.testing.assert_allclose(algo.flat.flat.cpu().numpy(), z["params"][-1], rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(algo.optimizer.state1.cpu().numpy(), z["opt_state1"], rtol=1e-3, atol=1e-12)


@pytest.mark.parametrize("kind", ["cartpole", "halfcheetah", "pong"])
def test_synthetic_training_end_to_end(kind, tmp_path):
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(1)
    N = {"cartpole": 64, "halfcheetah": 16, "pong": 8}[kind]
    env = SyntheticVecEnv(N, kind, seed=1)
    pkw = dict(activation_fn="relu") if kind == "pong" else {}
    if kind == "halfcheetah":
        pkw = dict(pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256], activation_fn="relu", log_std_init=-2,
                   init_layers_orthogonal=False)
    policy = ActorCritic(env, **pkw).to(DEV)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=16)
    rec = Recorder()
    algo = PPO(policy, DEV, rec, batch_size=64, n_epochs=2, learning_rate=1e-3, ent_coef=0.01)
    algo.learn(2 * 16 * N, gen)
    ts = algo.last_train_stats
    assert np.isfinite([ts.loss, ts.pi_loss, ts.entropy_loss, ts.approx_kl, ts.grad_norm]).all()
    assert rec.scalars["train/steps_per_second"] > 0
    assert (gen.actions >= (0 if kind != "halfcheetah" else -100)).all()
    # checkpoint round trip (model.pth + optimizer.pt in torch formats)
    policy.save(str(tmp_path))
    algo.save(str(tmp_path))
    sd = torch.load(tmp_path / "model.pth", weights_only=True)
    assert set(sd) == set(policy.state_dict())
    opt = torch.load(tmp_path / "optimizer.pt", weights_only=True)
    assert float(opt["state"][0]["step"]) == algo.optimizer.step_count


class _SpaceEnv:
    """Just the spaces ActorCritic reads (obs Box(d), Discrete(n))."""

    def __init__(self, d, n):
        from rl_algo_impls_amd.envs import Box, Discrete

        self.single_observation_space = Box(-1.0, 1.0, shape=(d,))
        self.single_action_space = Discrete(n)
        self.num_envs = 1


def _random_rollout(T, N, d, n, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    t = lambda x: x.to(DEV)
    obs = t(torch.randn(T, N, d, generator=g))
    act = t(torch.randint(0, n, (T, N), generator=g))
    rew = t(torch.randn(T, N, generator=g))
    starts = t((torch.rand(T, N, generator=g) < 0.05).to(torch.uint8))
    vals = t(torch.randn(T, N, generator=g))
    logp = t(torch.log(torch.full((T, N), 1.0 / n)) + 0.1 * torch.randn(T, N, generator=g))
    nstarts = t((torch.rand(N, generator=g) < 0.05).to(torch.uint8))
    nvals = t(torch.randn(N, generator=g))
    return obs, act, rew, starts, vals, logp, nstarts, nvals


@pytest.mark.parametrize("d,n,act,bs,T,N,layout", [
    (4, 2, "tanh", 256, 8, 96, "mc"),        # CartPole class, ragged last minibatch (768 % 256 = 0 -> 3 full)
    (4, 2, "tanh", 200, 9, 100, "mc"),       # B < 256, ragged tail (900 % 200 = 100)
    (4, 2, "relu", 64, 8, 64, "mc"),         # B = 64: CUs 4..15 see no rows
    (4, 2, "tanh", 40, 5, 50, "mc"),         # B = 40: CU 2's tile half-filled, ragged tail
    (4, 2, "tanh", 256, 8, 96, "mc8"),       # 8 CUs per network (two 16-row tiles per CU)
    (4, 2, "relu", 40, 5, 50, "mc8"),        # B = 40: CU 1's second tile half-filled
    (3, 1, "tanh", 96, 6, 50, "mc8"),
    (4, 2, "tanh", 256, 8, 96, "mc4"),       # 4-CU-per-network layout (the data-parallel grads kernel)
    (4, 2, "relu", 200, 9, 100, "mc4"),
    (2, 2, "tanh", 128, 5, 78, "mc"),        # in_dim 2 (padding columns), ragged tail (390 % 128 = 6)
    (3, 1, "tanh", 96, 6, 50, "mc"),         # one action
    (4, 2, "tanh", 256, 8, 96, "rows"),      # diagnostic one-CU row-tile layout
    (4, 2, "tanh", 256, 8, 96, "chunk"),     # chunked one-CU layout
    (6, 3, "tanh", 128, 8, 64, "chunk"),     # Acrobot-like: generic (8, 8) instantiation
    (8, 8, "relu", 256, 4, 200, "chunk"),    # maximum shape of the chunked kernel
])
def test_fused_epoch_matches_generic_path(d, n, act, bs, T, N, layout, monkeypatch):
    """One epoch of the fused kernel (given layout; "mc" = the default, 16 CUs per network) vs
    the per-minibatch PyTorch path, same
    rollout and permutation.  fp32 tolerances: different summation orders and the fused
    kernel's hardware sqrt/rcp Adam."""
    from rl_algo_impls_amd.policy import ActorCritic

    if (T * N) % bs == 1:
        pytest.skip("1-row minibatch has no unbiased std")
    if layout == "mc8":
        monkeypatch.setenv("RAI_MLP_CUS", "8")
    elif layout != "mc":
        monkeypatch.setenv("RAI_MLP_LAYOUT", layout)
    roll = _random_rollout(T, N, d, n, seed=d * 100 + n * 10 + bs)
    results = []
    for generic in (False, True):
        torch.manual_seed(5)
        policy = ActorCritic(_SpaceEnv(d, n), activation_fn=act).to(DEV)
        algo = PPO(policy, DEV, None, batch_size=bs, n_epochs=2, learning_rate=3e-3, ent_coef=0.01,
                   clip_range=0.2, gamma=0.98, gae_lambda=0.9)
        algo.force_generic = generic
        assert (algo.fused_mlp_spec() is None) == generic
        obs, a_, rew, starts, vals, logp, nstarts, nvals = roll
        perms = [torch.randperm(T * N, generator=torch.Generator().manual_seed(s)) for s in (1, 2)]
        r = DeviceRollout(DEV, nstarts, nvals, obs, a_, rew, starts, vals, logp, None, 0.98, 0.9,
                          perm_source=lambda k: perms.pop(0))
        stats, norms, _ = algo.update(r)
        results.append((algo.flat.flat.cpu().numpy(), stats, norms, algo.optimizer.state1.cpu().numpy()))
    (pf, sf, nf, mf), (pg, sg, ng, mg) = results
    np.testing.assert_allclose(nf, ng, rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(sf[:, :6], sg[:, :6], rtol=2e-3, atol=2e-6)
    np.testing.assert_allclose(pf, pg, rtol=1e-3, atol=2e-5)
    np.testing.assert_allclose(mf, mg, rtol=2e-2, atol=1e-6)


def _cartpole_best_return(seed):
    from rl_algo_impls_amd.envs import CartPoleVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(seed)
    env = CartPoleVecEnv(8, seed=seed)
    policy = ActorCritic(env).to(DEV)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=32, seed=seed)
    algo = PPO(policy, DEV, None, batch_size=256, n_epochs=20, learning_rate=1e-3, gamma=0.98, gae_lambda=0.8,
               clip_range=0.2, ent_coef=0.0)
    assert algo.fused_mlp_spec() is not None
    best = 0.0
    steps = 0
    while steps < 100_000:
        # the YAML's hyperparam_transitions: lr 1e-3 -> 0 and clip 0.2 -> 0, linear in progress
        # (rl_algo_impls/shared/callbacks/hyperparam_transitions.py:85-100, interpolate "linear")
        prog = steps / 100_000
        algo.learning_rate, algo.clip_range = 1e-3 * (1 - prog), 0.2 * (1 - prog)
        steps, _ = algo.learn_epoch(steps, 100_000, gen, None)
        if len(gen.episode_returns) >= 20:
            best = max(best, float(np.mean(gen.episode_returns)))
        if best > 475:
            break
    return best


def test_ppo_learns_cartpole_v1():
    """Return check on the real CartPole-v1 dynamics (envs.CartPoleVecEnv, gymnasium 0.29's
    public equations) with the reference's CartPole PPO hyperparameters
    (rl_algo_impls/hyperparams/ppo.yml:1-23: 8 envs x 32 steps, batch 256, 20 epochs, lr 1e-3,
    gamma 0.98, lambda 0.8, clip 0.2, and its linear lr/clip decay to 0 over the 100k steps).
    Statistical, not bit-level: the rolling mean of the last 100 episode returns must pass 475
    (the 500-step cap is CartPole-v1's maximum) within 100k steps, as the reference does, in at
    least 2 of 3 seeded runs (a single trajectory occasionally plateaus near 400-470, for any
    fp32 summation order: tools/learn_probe.py)."""
    bests = [_cartpole_best_return(seed) for seed in (1, 2, 3)]
    assert sum(b > 475 for b in bests) >= 2, f"best rolling mean returns per seed: {bests}"


def _policy_for(kind):
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    env = SyntheticVecEnv(4, kind, seed=3)
    pkw = dict(activation_fn="relu") if kind == "pong" else {}
    if kind == "halfcheetah":
        pkw = dict(pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256], activation_fn="relu", log_std_init=-2,
                   init_layers_orthogonal=False)
    return env, ActorCritic(env, **pkw)


@pytest.mark.parametrize("kind,T,N,bs,extra", [
    ("cartpole", 16, 40, 64, {}),                              # 640 rows: 10 full minibatches
    ("cartpole", 9, 50, 64, dict(clip_range_vf=0.1)),          # 450 rows: ragged tail of 2
    ("halfcheetah", 16, 24, 64, dict(ent_coef=0.01)),          # Gaussian head, 384 rows
    ("pong", 8, 12, 32, dict(ent_coef=0.01)),                  # NatureCNN, 96 rows
    ("cartpole", 8, 32, 64, dict(gradient_accumulation=True)),  # optimizer step once per epoch (eager)
])
def test_graphed_update_matches_eager(kind, T, N, bs, extra):
    """The hipGraph-replayed minibatch step (graphs.py) runs the same kernels on the same
    minibatches as the eager loop: parameters, optimizer state and stats agree over two updates
    (capture on the first, pure replay on the second)."""
    # MIOpen's default convolution-backward solvers are not run-to-run reproducible (split-K
    # accumulation order); the NatureCNN case asks for its deterministic solvers
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = kind == "pong"
    try:
        _graphed_vs_eager(kind, T, N, bs, extra)
    finally:
        torch.backends.cudnn.deterministic = det


def _graphed_vs_eager(kind, T, N, bs, extra):
    results = []
    for graphs in (False, True):
        torch.manual_seed(7)
        env, policy = _policy_for(kind)
        policy = policy.to(DEV)
        algo = PPO(policy, DEV, None, batch_size=bs, n_epochs=3, learning_rate=3e-4, **extra)
        algo.force_generic = True
        algo.use_graphs = graphs
        g = torch.Generator(device="cpu").manual_seed(11)
        shp = env.single_observation_space.shape
        obs = (torch.randint(0, 256, (T, N) + shp, generator=g, dtype=torch.uint8) if kind == "pong"
               else torch.randn((T, N) + shp, generator=g))
        if kind == "halfcheetah":
            act = torch.randn(T, N, 6, generator=g).clamp(-1, 1)
        else:
            act = torch.randint(0, env.single_action_space.n, (T, N), generator=g)
        t = lambda x: x.to(DEV)
        rew, vals = torch.randn(T, N, generator=g), torch.randn(T, N, generator=g)
        starts = (torch.rand(T, N, generator=g) < 0.05).to(torch.uint8)
        logp = -1.0 + 0.1 * torch.randn(T, N, generator=g)
        perm_g = torch.Generator(device="cpu").manual_seed(5)
        r = DeviceRollout(DEV, t(torch.zeros(N, dtype=torch.uint8)), t(torch.randn(N, generator=g)), t(obs), t(act),
                          t(rew), t(starts), t(vals), t(logp), None, 0.99, 0.95,
                          perm_source=lambda n: torch.randperm(n, generator=perm_g))
        out = []
        for _ in range(2):
            stats, norms, _ = algo.update(r)
            out.append((stats.copy(), norms.copy()))
        torch.cuda.synchronize()
        results.append((algo.flat.flat.cpu().numpy(), algo.optimizer.state1.cpu().numpy(), out,
                        algo.optimizer.step_count, algo._graphed))
    (p0, m0, o0, c0, _), (p1, m1, o1, c1, gu) = results
    assert c0 == c1
    if not extra.get("gradient_accumulation"):
        assert gu is not None and any(gr.graph is not None for gr in gu.graphs.values()), "no graph was captured"
    # NatureCNN: fp32 tolerance on top of the deterministic solvers (the graph and eager runs may
    # still pick different solvers); the MLP cases run identical kernels and agree to the last bits
    atol = 2e-5 if kind == "pong" else 1e-7
    np.testing.assert_allclose(p1, p0, rtol=1e-3 if kind == "pong" else 1e-6, atol=atol)
    # Adam's first moment of a near-zero gradient entry carries the conv backward's rounding: for
    # NatureCNN the bound is absolute (|m| entries ~1e-5 differ in the last bits)
    np.testing.assert_allclose(m1, m0, rtol=1e-3 if kind == "pong" else 1e-5, atol=1e-7 if kind == "pong" else 1e-9)
    for (s0, n0), (s1, n1) in zip(o0, o1):
        np.testing.assert_allclose(s1, s0, rtol=1e-4 if kind == "pong" else 1e-5, atol=1e-7)
        np.testing.assert_allclose(n1, n0, rtol=1e-4 if kind == "pong" else 1e-5)


def test_wide_epoch_full_c4_horizon_drift(monkeypatch):
    """Config C4's update at its per-GPU shape (256 envs x 512 steps = 131,072 rows; the YAML's batch 64
    x 20 epochs = 2,048 dependent optimizer steps per rai_mlp_wide_epoch launch, 40,960 per update;
    rl_algo_impls/hyperparams/ppo.yml:337-359) through the whole-epoch kernel vs the per-minibatch
    kernels (RAI_WIDE_EPOCH=0: graph-replayed wide-MLP forward/backward + rai_ppo_loss +
    rai_clip_optim_step), identical rollout and permutations.  The whole-epoch kernel reuses its
    per-step publish / drain slots thousands of times per launch; this is the horizon at which a slot
    reuse or drift bug would show.  Bound as test_fused_epoch_full_c2_horizon_drift: the per-minibatch
    path re-run from weights perturbed by one ulp sets the noise floor."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(3)
    env = SyntheticVecEnv(256, "halfcheetah", seed=5)
    policy = ActorCritic(env, pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256], activation_fn="relu",
                         log_std_init=-2, init_layers_orthogonal=False).to(DEV)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=512, seed=11)
    r = gen.rollout(gamma=0.98, gae_lambda=0.92)
    p0 = torch.nn.utils.parameters_to_vector(policy.parameters()).detach().clone()
    runs = {}
    for name, epoch, perturb in (("epoch", "1", 0), ("minibatch", "0", 0), ("minibatch_ulp", "0", 1),
                                 ("minibatch_ulp_down", "0", -1)):
        monkeypatch.setenv("RAI_WIDE_EPOCH", epoch)
        start = p0.clone()
        if perturb:
            start = torch.nextafter(start, torch.full_like(start, perturb * float("inf")))
        torch.nn.utils.vector_to_parameters(start, policy.parameters())
        algo = PPO(policy, DEV, None, batch_size=64, n_epochs=20, gamma=0.98, gae_lambda=0.92,
                   ent_coef=0.000401762, max_grad_norm=0.8, vf_coef=0.58096, learning_rate=2.0633e-05,
                   clip_range=0.1)
        g = torch.Generator(device=DEV)
        g.manual_seed(123)
        r._perm_source = lambda n: torch.randperm(n, device=DEV, generator=g)
        stats, norms, _ = algo.update(r)
        torch.cuda.synchronize()
        assert algo.optimizer.step_count == 40960
        assert (getattr(algo, "_we_ws", None) is not None) == (epoch == "1"), "whole-epoch kernel use"
        runs[name] = (algo.flat.flat.detach().cpu().double().numpy(), stats.astype(np.float64), norms)
    pe, se, ne = runs["epoch"]
    pm, sm, nm = runs["minibatch"]
    ulps = [runs["minibatch_ulp"], runs["minibatch_ulp_down"]]
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))
    drift, floor = rel(pe, pm), max(rel(pu, pm) for pu, _, _ in ulps)
    last = slice(-2048, None)
    stat_drift = np.abs(se[last, :6].mean(0) - sm[last, :6].mean(0))
    stat_floor = np.max([np.abs(su[last, :6].mean(0) - sm[last, :6].mean(0)) for _, su, _ in ulps], axis=0)
    norm_floor = max(rel(nu, nm) for _, _, nu in ulps)
    print(f"C4 horizon: |p_epoch - p_minibatch|/|p| = {drift:.3e}, ulp floor {floor:.3e}; max abs param diff "
          f"{np.abs(pe - pm).max():.3e}; last-epoch mean stats diff {stat_drift} floor {stat_floor}; "
          f"grad norms rel {rel(ne, nm):.3e} floor {norm_floor:.3e}")
    assert np.isfinite(pe).all() and np.isfinite(se).all() and np.isfinite(ne).all()
    assert drift <= max(4 * floor, 1e-5), (drift, floor)
    assert rel(ne, nm) <= max(4 * norm_floor, 1e-4)
    # clipped_frac (column 4) is a mean of 131,072 per-sample indicators: once the trajectories have
    # decorrelated to the ulp floor, its difference is sampling noise, 3 binomial standard deviations
    p_clip = float(sm[last, 4].mean())
    tol = np.maximum(4 * stat_floor, 1e-4 * (1 + np.abs(sm[last, :6].mean(0))))
    tol[4] = max(tol[4], 3 * np.sqrt(p_clip * (1 - p_clip) / (2048 * 64)))
    assert (stat_drift <= tol).all(), (stat_drift, tol)


@pytest.mark.parametrize("kind,hidden,act,extra", [
    ("halfcheetah", 256, "relu", dict(ent_coef=0.01)),                     # the C4 policy
    ("halfcheetah", 128, "tanh", dict(clip_range_vf=0.2)),
    ("cartpole", 256, "tanh", dict(ent_coef=0.01)),                        # Categorical head, 256 wide
    ("halfcheetah", 64, "relu", dict(gradient_accumulation=True)),         # accumulate mode
    ("halfcheetah", 192, "relu", dict(N=25, clip_range_vf=0.1)),           # 400 rows: ragged tail of 16
    ("halfcheetah", 128, "relu", dict(bs=50)),  # B IN = 850: 4-B observation staging; ragged tail of 34
])
@pytest.mark.parametrize("epoch", ["1", "0"], ids=["whole_epoch_kernel", "per_minibatch_kernels"])
def test_wide_mlp_kernels_match_pytorch_path(kind, hidden, act, extra, epoch, monkeypatch):
    """Fused wide-MLP path vs the PyTorch network + autograd (eager) on the same minibatches: two
    updates x 3 epochs, fp32 tolerance (different reduction order).  whole_epoch_kernel: one
    rai_mlp_wide_epoch launch per epoch (where its scope covers the options; gradient accumulation
    keeps the per-minibatch kernels); per_minibatch_kernels (RAI_WIDE_EPOCH=0): the graph-replayed
    wide-MLP kernels + rai_ppo_loss + rai_clip_optim_step."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    monkeypatch.setenv("RAI_WIDE_EPOCH", epoch)

    extra = dict(extra)
    T, N, bs = 16, extra.pop("N", 24), extra.pop("bs", 64)  # 384 rows: 6 minibatches of 64
    res = []
    for wide in (True, False):
        torch.manual_seed(7)
        env = SyntheticVecEnv(4, kind, seed=3)
        pkw = dict(pi_hidden_sizes=[hidden, hidden], v_hidden_sizes=[hidden, hidden], activation_fn=act)
        if kind == "halfcheetah":
            pkw.update(log_std_init=-1.0, init_layers_orthogonal=False)
        policy = ActorCritic(env, **pkw).to(DEV)
        algo = PPO(policy, DEV, None, batch_size=bs, n_epochs=3, learning_rate=3e-4, **extra)
        algo.use_wide = wide
        algo.use_graphs = wide
        g = torch.Generator(device="cpu").manual_seed(11)
        shp = env.single_observation_space.shape
        obs = torch.randn((T, N) + shp, generator=g)
        act_t = (torch.randn(T, N, 6, generator=g).clamp(-1, 1) if kind == "halfcheetah"
                 else torch.randint(0, 2, (T, N), generator=g))
        t = lambda x: x.to(DEV)
        perm_g = torch.Generator(device="cpu").manual_seed(5)
        r = DeviceRollout(DEV, t(torch.zeros(N, dtype=torch.uint8)), t(torch.randn(N, generator=g)), t(obs), t(act_t),
                          t(torch.randn(T, N, generator=g)), t((torch.rand(T, N, generator=g) < 0.05).to(torch.uint8)),
                          t(torch.randn(T, N, generator=g)), t(-1.0 + 0.1 * torch.randn(T, N, generator=g)), None,
                          0.99, 0.95, perm_source=lambda n: torch.randperm(n, generator=perm_g))
        out = [algo.update(r)[:2] for _ in range(2)]
        torch.cuda.synchronize()
        res.append((algo.flat.flat.cpu().numpy(), out, algo._wide, getattr(algo, "_we_ws", None) is not None))
    (p_w, o_w, w, we), (p_t, o_t, _, _) = res
    assert w not in (None, False), "wide path not taken"
    assert we == (epoch == "1" and not extra.get("gradient_accumulation")), "whole-epoch kernel use"
    np.testing.assert_allclose(p_w, p_t, rtol=1e-4, atol=2e-6)
    for (s_w, n_w), (s_t, n_t) in zip(o_w, o_t):
        np.testing.assert_allclose(s_w[:, :6], s_t[:, :6], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(n_w, n_t, rtol=1e-4)


def test_wide_epoch_ragged_tail_reads_nothing_past_the_records():
    """rai_mlp_wide_epoch's record prefetch on a ragged last minibatch (400 rows, B = 64: a tail of 16)
    with the workspace allocated at EXACTLY rai_mlp_wide_epoch_workspace_bytes and the bytes after it
    filled with NaN (0xFF): the per-row records are the workspace's last region, so a load past the
    rollout's last row would pull NaN into the tail rows' staging and, through 0 * NaN, into the
    gradient.  The update must be bitwise equal to the same update with a zeroed tail."""
    from rl_algo_impls_amd import _lib
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    T, N, bs, H = 16, 25, 64, 192
    res = []
    for poison in (0, 0xFF):
        torch.manual_seed(7)
        env = SyntheticVecEnv(4, "halfcheetah", seed=3)
        policy = ActorCritic(env, pi_hidden_sizes=[H, H], v_hidden_sizes=[H, H], activation_fn="relu",
                             log_std_init=-1.0, init_layers_orthogonal=False).to(DEV)
        algo = PPO(policy, DEV, None, batch_size=bs, n_epochs=2, learning_rate=3e-4, clip_range_vf=0.1)
        algo.use_wide = True
        in_dim = env.single_observation_space.shape[0]
        ws_bytes = int(_lib.lib().rai_mlp_wide_epoch_workspace_bytes(H, in_dim, T * N))
        assert ws_bytes > 0
        backing = torch.full((ws_bytes + (1 << 20),), poison, dtype=torch.uint8, device=DEV)
        backing[:ws_bytes].zero_()
        algo._we_ws = backing[:ws_bytes]  # exactly the required size; the update reuses it (numel >= need)
        g = torch.Generator(device="cpu").manual_seed(11)
        obs = torch.randn((T, N, in_dim), generator=g)
        act_t = torch.randn(T, N, 6, generator=g).clamp(-1, 1)
        t = lambda x: x.to(DEV)
        perm_g = torch.Generator(device="cpu").manual_seed(5)
        r = DeviceRollout(DEV, t(torch.zeros(N, dtype=torch.uint8)), t(torch.randn(N, generator=g)), t(obs), t(act_t),
                          t(torch.randn(T, N, generator=g)), t((torch.rand(T, N, generator=g) < 0.05).to(torch.uint8)),
                          t(torch.randn(T, N, generator=g)), t(-1.0 + 0.1 * torch.randn(T, N, generator=g)), None,
                          0.99, 0.95, perm_source=lambda n: torch.randperm(n, generator=perm_g))
        stats, norms, _ = algo.update(r)
        torch.cuda.synchronize()
        assert algo._we_ws.data_ptr() == backing.data_ptr(), "the whole-epoch kernel used the exact workspace"
        if poison:
            assert bool((backing[ws_bytes:] == poison).all()), "nothing written past the workspace"
        res.append((algo.flat.flat.cpu().numpy(), stats, norms))
    (p0, s0, n0), (p1, s1, n1) = res
    assert np.isfinite(p1).all() and np.isfinite(n1).all()
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(n1, n0)
    np.testing.assert_array_equal(s1[:, :6], s0[:, :6])


@pytest.mark.parametrize("kind,N", [("halfcheetah", 64), ("cartpole", 64), ("halfcheetah", 200)])
def test_wide_rollout_forward_matches_module(kind, N, monkeypatch):
    """The rollout's policy forward through rai_mlp_wide_dist_params (3 launches, graph-replayed)
    against the PyTorch module forward (RAI_ROLLOUT_WIDE=0): same seeded sampler, so the sampled
    actions, log-probs and values of 16 env steps agree to fp32 tolerance (the Gaussian action is
    mu + std * noise: it inherits mu's rounding)."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    res = []
    for wide in ("1", "0"):
        monkeypatch.setenv("RAI_ROLLOUT_WIDE", wide)
        torch.manual_seed(3)
        env = SyntheticVecEnv(N, kind, seed=5)  # N = 200: four 64-row chunks (grid.z), the last ragged
        pkw = dict(pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256], activation_fn="relu")
        if kind == "halfcheetah":
            pkw.update(log_std_init=-1.0, init_layers_orthogonal=False)
        policy = ActorCritic(env, **pkw).to(DEV)
        gen = SyncStepRolloutGenerator(policy, env, n_steps=16, seed=9)
        assert (gen._wide_fwd is not None) == (wide == "1")
        r = gen.rollout(gamma=0.99, gae_lambda=0.95)
        torch.cuda.synchronize()
        res.append((gen.actions.cpu().numpy().copy(), gen.logprobs.cpu().numpy().copy(),
                    gen.values.cpu().numpy().copy(), r.next_values.cpu().numpy().copy()))
    (a1, l1, v1, n1), (a0, l0, v0, n0) = res
    if kind == "cartpole":
        assert (a1 == a0).mean() > 0.99  # a logit within rounding of a sampling threshold may flip
    else:
        np.testing.assert_allclose(a1, a0, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(v1, v0, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(n1, n0, rtol=1e-4, atol=1e-5)
    same = (a1 == a0) if kind == "cartpole" else np.ones(l1.shape, dtype=bool)
    np.testing.assert_allclose(l1[same], l0[same], rtol=1e-4, atol=1e-5)


def test_fused_rollout_direct_slot_staging_is_identical(monkeypatch):
    """The CartPole-class rollout stages each step's next observations and episode starts straight into
    slot s + 1 (RAI_ROLLOUT_DIRECT, default on) instead of through next_obs_dev / next_episode_starts
    and a device copy: two seeded rollouts (two updates' worth, so the second starts from the first's
    carried-over state), one each way, give bit-identical buffers and bootstrap values."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    out = []
    for direct, native, mapped in (("1", "1", "1"), ("1", "1", "0"), ("1", "0", "0"), ("0", "0", "0")):
        monkeypatch.setenv("RAI_ROLLOUT_DIRECT", direct)
        monkeypatch.setenv("RAI_ROLLOUT_NATIVE", native)  # the native staging loop (default) vs torch copies
        monkeypatch.setenv("RAI_ROLLOUT_MAPPED", mapped)  # host-mapped hand-off in the policy-step kernel
        torch.manual_seed(3)
        env = SyntheticVecEnv(96, "cartpole", seed=5)
        policy = ActorCritic(env).to(DEV)
        gen = SyncStepRolloutGenerator(policy, env, n_steps=16, seed=9)
        assert gen.fused_step is not None
        res = []
        for _ in range(2):
            r = gen.rollout(gamma=0.98, gae_lambda=0.8)
            torch.cuda.synchronize()
            res.append([t.detach().cpu().numpy().copy() for t in (gen.obs, gen.actions, gen.rewards, gen.episode_starts,
                                                                   gen.values, gen.logprobs, r.next_values,
                                                                   r.next_episode_starts, r.advantages)])
        out.append(res)
    for other in out[1:]:
        for a, b in zip(out[0], other):
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
