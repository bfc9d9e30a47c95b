"""SURVEY 8(d) batch policy (b), "scaled" (batch_size = n_steps * num_envs / 4): the large-minibatch HIP
path of the CartPole-class MLP (csrc/mlp_large.hip, reached through rai_mlp_ppo_epoch / rai_mlp_ppo_grads
when batch_size > 256) against the reference's own PPO.learn_epoch (learn_epoch_scaled.npz, made by
tests/golden/make_golden_scaled.py), against the PyTorch network path on the same permutations, and at
the full C2 scaled shape (4096 x 128, batch 131,072) through size-independent properties."""
import json

import numpy as np
import pytest
import torch

from rl_algo_impls_amd import _lib
from rl_algo_impls_amd.ppo import PPO
from rl_algo_impls_amd.rollout import DeviceRollout, SyncStepRolloutGenerator
import make_golden_networks as nets

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class Recorder:
    def __init__(self):
        self.scalars = {}

    def add_scalar(self, tag, value, global_step=None):
        self.scalars[tag] = float(value)


def _run_fixture(z, case, generic):
    p = case + "/"
    kw = json.loads(str(z[p + "kw"]))
    policy = nets.build("cartpole")
    nets.load_flat(policy, z[p + "init"])
    policy = policy.to(DEV)
    rec = Recorder()
    algo = PPO(policy, DEV, rec, **kw)
    algo.force_generic = generic
    assert (algo.fused_mlp_spec() is None) == generic
    assert algo.batch_size > _lib.RAI_MLP_EPOCH_MAX_B
    perms = list(z[p + "perms"])
    t = lambda k: torch.from_numpy(z[p + k]).to(DEV)
    r = DeviceRollout(DEV, t("next_episode_starts"), t("next_values"), t("obs"), t("actions"), t("rewards"),
                      t("episode_starts"), t("values"), t("logprobs"), None, kw["gamma"], kw["gae_lambda"],
                      perm_source=lambda n: torch.from_numpy(perms.pop(0)))
    np.testing.assert_array_equal(r.advantages.cpu().numpy(), z[p + "advantages"])

    class Gen:
        def rollout(self, gamma, gae_lambda):
            return r

    algo.learn_epoch(0, r.total_steps, Gen(), None)
    assert not perms
    return algo, rec


@pytest.mark.parametrize("case", ["scaled", "ragged_vclip"])
@pytest.mark.parametrize("generic", [False, True], ids=["large_minibatch_kernels", "generic_path"])
def test_scaled_learn_epoch_matches_reference(golden, case, generic):
    z = golden("learn_epoch_scaled.npz")
    algo, rec = _run_fixture(z, case, generic)
    np.testing.assert_allclose(algo.flat.flat.cpu().numpy(), z[case + "/params"], rtol=2e-4, atol=5e-6)
    names = ("loss", "pi_loss", "v_loss", "entropy_loss", "approx_kl", "clipped_frac", "explained_var", "grad_norm")
    got = np.array([rec.scalars[f"losses/{k}"] for k in names])
    np.testing.assert_allclose(got, z[case + "/losses"], rtol=2e-4, atol=2e-6)
    assert algo.optimizer.step_count == len(z[case + "/grad_norms"])


def _c2_rollout(n_envs, n_steps, seed=5):
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(3)
    env = SyntheticVecEnv(n_envs, "cartpole", seed=seed)
    policy = ActorCritic(env).to(DEV)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=n_steps, seed=11)
    r = gen.rollout(gamma=0.98, gae_lambda=0.8)
    return policy, r


def _update(policy, r, start, batch, n_epochs, generic, seed=123, **kw):
    torch.nn.utils.vector_to_parameters(start, policy.parameters())
    algo = PPO(policy, DEV, None, batch_size=batch, n_epochs=n_epochs, learning_rate=1e-3, gamma=0.98,
               gae_lambda=0.8, clip_range=0.2, **kw)
    algo.force_generic = generic
    assert (algo.fused_mlp_spec() is None) == generic
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    r._perm_source = lambda n: torch.randperm(n, device=DEV, generator=g)
    stats, norms, _ = algo.update(r)
    torch.cuda.synchronize()
    return algo.flat.flat.detach().cpu().double().numpy(), stats.astype(np.float64), np.asarray(norms, np.float64)


def test_large_minibatch_matches_generic_one_epoch():
    """4096 envs x 16 steps, batch 16,384 (4 minibatches), one epoch: the large-minibatch kernels vs the
    PyTorch network + autograd path on identical permutations (fp32 summation orders differ)."""
    policy, r = _c2_rollout(4096, 16)
    p0 = torch.nn.utils.parameters_to_vector(policy.parameters()).detach().clone()
    pf, sf, nf = _update(policy, r, p0, 16384, 1, generic=False, ent_coef=0.01, clip_range_vf=0.2)
    pg, sg, ng = _update(policy, r, p0, 16384, 1, generic=True, ent_coef=0.01, clip_range_vf=0.2)
    np.testing.assert_allclose(nf, ng, rtol=1e-4)
    np.testing.assert_allclose(sf[:, :6], sg[:, :6], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(sf[:, 5 + _lib.RAI_MAX_K], sg[:, 5 + _lib.RAI_MAX_K], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(pf, pg, rtol=1e-4, atol=2e-6)


def test_large_minibatch_deterministic():
    """The fixed tile -> wave assignment and workgroup-order reductions make the update bitwise
    reproducible."""
    policy, r = _c2_rollout(4096, 8)
    p0 = torch.nn.utils.parameters_to_vector(policy.parameters()).detach().clone()
    a = _update(policy, r, p0, 8192, 2, generic=False)
    b = _update(policy, r, p0, 8192, 2, generic=False)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_full_c2_scaled_update_vs_generic():
    """Config C2 at batch policy (b): 4096 envs x 128 steps, batch 131,072 = T*N/4, 20 epochs = 80
    optimizer steps, large-minibatch kernels vs the PyTorch path from the same weights and permutations.
    The drift is bounded relative to the generic path re-run from weights one ulp away (the trajectory's
    own sensitivity over 80 Adam steps)."""
    policy, r = _c2_rollout(4096, 128)
    p0 = torch.nn.utils.parameters_to_vector(policy.parameters()).detach().clone()
    pf, sf, nf = _update(policy, r, p0, 131072, 20, generic=False)
    pg, sg, ng = _update(policy, r, p0, 131072, 20, generic=True)
    pu, su, nu = _update(policy, r, torch.nextafter(p0, torch.full_like(p0, float("inf"))), 131072, 20,
                         generic=True)
    assert len(nf) == 80
    rel = lambda x, y: float(np.linalg.norm(x - y) / np.linalg.norm(y))
    drift, floor = rel(pf, pg), rel(pu, pg)
    print(f"C2 scaled: param drift {drift:.3e} vs ulp floor {floor:.3e}; first-step norm "
          f"{nf[0]:.6f} vs {ng[0]:.6f}")
    np.testing.assert_allclose(nf[:4], ng[:4], rtol=1e-4)
    assert drift <= max(10 * floor, 1e-5), (drift, floor)
    np.testing.assert_allclose(sf[-4:, :6].mean(0), sg[-4:, :6].mean(0), rtol=2e-3, atol=1e-5)
