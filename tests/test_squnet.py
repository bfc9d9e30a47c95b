"""Squeeze-U-Net GridNet actor-critic (BASELINE config C5) against the reference
network run in this container (tests/golden/squnet_cases.npz, tests/golden/make_golden_squnet.py):

  * CPU: the full-width C5 network's state_dict keys, shapes and parameter count (5,458,513);
    seeded initialisation identical to the reference's (same module construction order): bit-exact
    for the default-initialised layers, 1e-5 of max|w| for orthogonal_ ones (host LAPACK QR);
    the critic values (torch CPU both sides, rtol 1e-5);
  * GPU: forward (backbone on MIOpen, GridNet log-prob/entropy on the fused HIP kernel) and the
    parameter gradients of sum(wl*logp + we*entropy + wv.v) against the reference's CPU autograd.
    Tolerance (fp32 convolutions on different engines, 20+ layers deep): logp / entropy sums over
    256 cells x 7 planes rtol 1e-4 atol 2e-3; values rtol 1e-4 atol 1e-5; gradients
    atol 2e-4 + rtol 2e-3 of each tensor's max |grad|.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

NVEC = np.array([6, 4, 4, 4, 4, 7, 49])
SUB = {0: {1: 1, 2: 2, 3: 3, 4: 4, 5: 4, 6: 5}}
C5_KW = dict(strides_per_level=[[2, 2], [2, 2]], deconv_strides_per_level=[[2, 2], [2, 2]],
             encoder_residual_blocks_per_level=[3, 2, 4], decoder_residual_blocks_per_level=[2, 3],
             increment_kernel_size_on_down_conv=True, additional_critic_activation_functions=["tanh", "identity"],
             subaction_mask=SUB, init_layers_orthogonal=True)


@pytest.fixture(scope="module")
def cases():
    return np.load(GOLDEN / "squnet_cases.npz", allow_pickle=False)


def _net(width, critic_channels=64, seed=None):
    from rl_algo_impls_amd.backbone import SqueezeUnetActorCriticNetwork
    from rl_algo_impls_amd.envs import Box, MultiDiscrete

    obs = Box(0.0, 1.0, (74, 16, 16), np.float32)
    if seed is not None:
        torch.manual_seed(seed)
    return SqueezeUnetActorCriticNetwork(obs, MultiDiscrete(np.tile(NVEC, 256)), MultiDiscrete(NVEC),
                                         channels_per_level=[width] * 3, critic_channels=critic_channels, **C5_KW)


def test_c5_state_dict_keys_shapes(cases):
    net = _net(128)
    sd = net.state_dict()
    assert list(sd.keys()) == [str(k) for k in cases["c5_keys"]]
    assert [",".join(map(str, v.shape)) for v in sd.values()] == [str(s) for s in cases["c5_shapes"]]
    assert sum(v.numel() for v in sd.values()) == int(cases["c5_num_params"]) == 5458513


@pytest.mark.parametrize("i", [0, 1])
def test_seeded_init_bit_identical(cases, i):
    seed, width, _ = (int(x) for x in cases[f"c{i}_meta"])
    net = _net(width, critic_channels=16, seed=seed)
    for k, v in net.state_dict().items():
        ref = cases[f"c{i}_init/{k}"]
        if k.startswith("backbone.") or k.endswith(".bias"):  # default init: RNG draws only
            np.testing.assert_array_equal(v.numpy(), ref, err_msg=k)
        else:  # orthogonal_: QR through the host LAPACK, whose last bits vary by machine
            np.testing.assert_allclose(v.numpy(), ref, rtol=0, atol=1e-5 * float(np.abs(ref).max()), err_msg=k)


@pytest.mark.parametrize("i", [0, 1])
def test_values_cpu(cases, i):
    seed, width, _ = (int(x) for x in cases[f"c{i}_meta"])
    net = _net(width, critic_channels=16, seed=seed)
    with torch.no_grad():
        v = net.value(torch.tensor(cases[f"c{i}_obs"]))
    np.testing.assert_allclose(v.numpy(), cases[f"c{i}_value"], rtol=1e-5, atol=1e-6)


def test_actor_critic_builds_squeeze_unet_policy():
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic

    env = SyntheticVecEnv(2, kind="microrts", obs_pool=2)
    pol = ActorCritic(env, actor_head_style="squeeze_unet", channels_per_level=[16, 16, 16], **{
        k: v for k, v in C5_KW.items() if k != "init_layers_orthogonal"})
    assert pol.action_shape == (256, 7) and pol.value_shape == (3,) and not pol.is_discrete
    assert any(k.startswith("network.backbone.encoders.0.0.") for k in pol.state_dict())


@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 1])
def test_forward_backward_vs_reference(cases, i):
    dev = torch.device("cuda", 0)
    seed, width, _ = (int(x) for x in cases[f"c{i}_meta"])
    net = _net(width, critic_channels=16, seed=seed).to(dev)
    obs = torch.tensor(cases[f"c{i}_obs"], device=dev)
    acts = torch.tensor(cases[f"c{i}_actions"], device=dev)
    masks = torch.tensor(cases[f"c{i}_masks"], device=dev)
    logp, ent, v = net(obs, acts, action_masks=masks)
    np.testing.assert_allclose(logp.detach().cpu().numpy(), cases[f"c{i}_logp"], rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(ent.detach().cpu().numpy(), cases[f"c{i}_entropy"], rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(v.detach().cpu().numpy(), cases[f"c{i}_v"], rtol=1e-4, atol=1e-5)
    t = lambda k: torch.tensor(cases[f"c{i}_{k}"], device=dev)
    ((t("wl") * logp).sum() + (t("we") * ent).sum() + (t("wv") * v).sum()).backward()
    for k, p in net.named_parameters():
        ref = cases[f"c{i}_grad/{k}"]
        tol = 2e-4 + 2e-3 * float(np.abs(ref).max())
        np.testing.assert_allclose(p.grad.cpu().numpy(), ref, rtol=0, atol=tol, err_msg=k)


class _FixedRollout:
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


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sq_c5_gradacc", "sq_steps_vclip"])
def test_ppo_update_matches_reference(name):
    """The C5 update path (squeeze-U-Net on MIOpen, fused GridNet head, rai_ppo_loss with K=3 critics
    and multi_reward_weights, clip + Adam) against the reference's PPO.learn_epoch on the same
    minibatches (tests/golden/squnet_ppo_steps.npz).  Tolerance: stats rtol 5e-4 atol 5e-5; parameters
    atol 0.05 * lr (Adam's first steps move every parameter by ~lr * g / |g|, so a conv-gradient
    entry near zero may differ in sign between the CPU reference and MIOpen); grad norms rtol 5e-4."""
    import json

    from make_golden_networks import load_flat
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import Batch

    dev = torch.device("cuda", 0)
    z = np.load(GOLDEN / "squnet_ppo_steps.npz", allow_pickle=False)
    meta = json.loads(str(z["index"]))[name]
    env = SyntheticVecEnv(1, kind="microrts", obs_pool=2)
    pol = ActorCritic(env, actor_head_style="squeeze_unet", channels_per_level=[meta["width"]] * 3,
                      critic_channels=16, **{k: v for k, v in C5_KW.items() if k != "init_layers_orthogonal"})
    load_flat(pol, z[f"{name}/init"])
    pol = pol.to(dev)
    kw = dict(meta["kw"])
    algo = PPO(pol, dev, None, **kw)
    bs = []
    for i in range(meta["n"]):
        t = lambda k: torch.from_numpy(z[f"{name}/b{i}_{k}"]).to(dev)
        bs.append(Batch(t("obs"), t("logprobs"), t("actions"), t("action_masks"), None, t("values"),
                        t("advantages"), t("returns")))
    stats, norms, K = algo.update(_FixedRollout(bs))
    assert K == 3
    ref = z[f"{name}/stats"]
    # per-sample logp is a sum over 256 cells x 7 planes (~ -2e3, fp32 ulp ~2e-4): pi_loss and
    # approx_kl inherit ~1e-5 absolute differences from it on either side
    np.testing.assert_allclose(stats[:, :5], ref[:, :5], rtol=5e-4, atol=5e-5)
    np.testing.assert_allclose(stats[:, 5:8], ref[:, 5:8], rtol=5e-4, atol=2e-6)
    np.testing.assert_allclose(norms, z[f"{name}/norms"], rtol=5e-4)
    np.testing.assert_allclose(algo.flat.flat.cpu().numpy(), z[f"{name}/params"][-1], rtol=0,
                               atol=0.05 * float(kw["learning_rate"]))
    assert float(algo.optimizer.state_dict()["state"][0]["step"]) == meta["opt_step"]


@pytest.mark.gpu
def test_microrts_training_end_to_end(tmp_path):
    """Rollout (per-position GridNet sampling under all-true masks, K=3 rewards and values) + GAE
    with vector gamma + the C5 update with gradient accumulation; checkpoint round trip."""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator

    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    env = SyntheticVecEnv(4, kind="microrts", seed=1, obs_pool=2)
    pol = ActorCritic(env, actor_head_style="squeeze_unet", channels_per_level=[16, 16, 16],
                      **{k: v for k, v in C5_KW.items() if k != "init_layers_orthogonal"}).to(dev)
    gen = SyncStepRolloutGenerator(pol, env, n_steps=8)
    algo = PPO(pol, dev, None, batch_size=8, n_epochs=2, gamma=[0.99, 0.999, 0.999], gae_lambda=[0.95, 0.99, 0.99],
               clip_range=0.1, clip_range_vf=None, ppo2_vf_coef_halving=True, gradient_accumulation=True,
               multi_reward_weights=[0.8, 0.01, 0.19], vf_coef=[0.5, 0.1, 0.2], ent_coef=0.01, learning_rate=1e-4)
    algo.learn(2 * 8 * 4, gen)
    ts = algo.last_train_stats
    assert np.isfinite([ts.loss, ts.pi_loss, ts.entropy_loss, ts.approx_kl, ts.grad_norm]).all()
    assert gen.actions.shape == (8, 4, 256, 7) and gen.values.shape == (8, 4, 3)
    nvec = torch.tensor(NVEC, device=dev)
    assert bool((gen.actions >= 0).all()) and bool((gen.actions < nvec).all())
    assert bool(torch.isfinite(gen.logprobs).all())
    pol.save(str(tmp_path))
    sd = torch.load(tmp_path / "model.pth", weights_only=True)
    assert set(sd) == set(pol.state_dict())


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,H", [(3, 16, 16), (2, 128, 4), (5, 128, 1), (4, 32, 8)])
def test_se_residual_epilogue_vs_pytorch(B, C, H):
    """rai_se_residual_fwd / _bwd (csrc/se_block.hip) against the PyTorch composition
    gelu(x + r * s) and its autograd, NHWC fp32.  Tolerance: rtol 1e-5 / atol 1e-6 (erf / exp in
    fp32 on both sides; ds is a sum over H*W)."""
    from rl_algo_impls_amd.backbone import _SEResidualEpilogue

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(B * 100 + C + H)
    mk = lambda *s: torch.randn(*s, generator=g).to(dev)
    x = mk(B, C, H, H).contiguous(memory_format=torch.channels_last).requires_grad_()
    r = mk(B, C, H, H).contiguous(memory_format=torch.channels_last).requires_grad_()
    s = torch.sigmoid(mk(B, C)).requires_grad_()
    dout = mk(B, C, H, H).contiguous(memory_format=torch.channels_last)
    out = _SEResidualEpilogue.apply(x, r, s)
    dx, dr, ds = torch.autograd.grad(out, (x, r, s), dout)
    ref = torch.nn.functional.gelu(x + r * s.view(B, C, 1, 1))
    rx, rr, rs = torch.autograd.grad(ref, (x, r, s), dout)
    for a, b_ in ((out, ref), (dx, rx), (dr, rr), (ds, rs)):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b_.detach().cpu().numpy(), rtol=1e-5, atol=1e-6)
    assert out.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.gpu
@pytest.mark.parametrize("transpose", [False, True])
def test_conv_bias_gelu_vs_pytorch(transpose):
    """conv_gelu (bias-free MIOpen conv + rai_bias_gelu_fwd/_bwd) against GELU(conv(x)) with the
    module's own bias, NHWC fp32: outputs and the gradients of input, weight and bias (rtol 1e-4 /
    atol 1e-5: the same convolution, the bias added in another pass)."""
    from rl_algo_impls_amd.backbone import conv_gelu

    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    conv = (torch.nn.ConvTranspose2d(32, 64, 2, stride=2) if transpose else torch.nn.Conv2d(32, 64, 3, padding=1)).to(dev)
    x = torch.randn(5, 32, 8, 8, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    dy = torch.randn_like(conv(x)).contiguous(memory_format=torch.channels_last)
    out = conv_gelu(conv, x)
    got = torch.autograd.grad(out, (x, conv.weight, conv.bias), dy)
    ref_out = torch.nn.functional.gelu(conv(x))
    ref = torch.autograd.grad(ref_out, (x, conv.weight, conv.bias), dy)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref_out.detach().cpu().numpy(), rtol=1e-4, atol=1e-5)
    for a, b_ in zip(got, ref):
        np.testing.assert_allclose(a.cpu().numpy(), b_.cpu().numpy(), rtol=1e-4, atol=1e-5)


@pytest.fixture(scope="module")
def case128():
    return np.load(GOLDEN / "squnet128_case.npz", allow_pickle=False)


def test_c5_width128_seeded_init(case128):
    """The C5 network at its own width (channels_per_level [128]*3, critic_channels 64) initialises
    like the reference from the same seed: per-tensor sum and sum of squares (float64 over the fp32
    values) equal for the default-initialised layers, within 1e-6 relative for orthogonal_ ones (the
    reference's own values at width 128 are in tests/golden/squnet128_case.npz)."""
    seed, width, _ = (int(x) for x in case128["meta"])
    net = _net(width, critic_channels=64, seed=seed)
    sd = net.state_dict()
    assert list(sd.keys()) == [str(k) for k in case128["keys"]]
    assert sum(v.numel() for v in sd.values()) == 5458513
    for (k, v), ref in zip(sd.items(), case128["init_moments"]):
        got = np.array([v.double().sum().item(), (v.double() ** 2).sum().item()])
        if k.startswith("backbone.") or k.endswith(".bias"):
            np.testing.assert_array_equal(got, ref, err_msg=k)
        else:
            np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6 * np.sqrt(ref[1]), err_msg=k)


@pytest.mark.gpu
def test_c5_width128_forward_backward_vs_reference(case128):
    """Forward (MIOpen channels_last backbone at 128 channels, fused GridNet head) and the autograd
    gradients of sum(wl*logp + we*entropy + wv.v) at B=2 against the reference's CPU run of the
    same seeded C5 network.  The fixture keeps per-tensor gradient moments, so the bounds are the
    ones the width-16/32 element-wise tolerance (atol 2e-4 + 2e-3 max|g|) implies for them: the
    norm within sqrt(n) times it and 1 % relative, the sum within n times it."""
    dev = torch.device("cuda", 0)
    seed, width, _ = (int(x) for x in case128["meta"])
    net = _net(width, critic_channels=64, seed=seed).to(dev)
    t = lambda k: torch.tensor(case128[k], device=dev)
    logp, ent, v = net(t("obs"), t("actions"), action_masks=t("masks"))
    np.testing.assert_allclose(logp.detach().cpu().numpy(), case128["logp"], rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(ent.detach().cpu().numpy(), case128["entropy"], rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(v.detach().cpu().numpy(), case128["v"], rtol=1e-4, atol=1e-5)
    ((t("wl") * logp).sum() + (t("we") * ent).sum() + (t("wv") * v).sum()).backward()
    names = [str(n) for n in case128["grad_names"]]
    params = dict(net.named_parameters())
    assert list(params) == names
    for n, (rsum, rsq, rmax) in zip(names, case128["grad_moments"]):
        g = params[n].grad.double()
        el = 2e-4 + 2e-3 * rmax
        norm, rnorm = float(g.norm()), float(np.sqrt(rsq))
        assert abs(norm - rnorm) <= min(np.sqrt(g.numel()) * el, 1e-2 * rnorm + 1e-6), (n, norm, rnorm)
        assert abs(float(g.sum()) - rsum) <= g.numel() * el, (n, float(g.sum()), rsum)


@pytest.mark.gpu
def test_c5_full_width_update():
    """C5 at its own width on the product path: the squnet-d16-128 policy (5,458,513 parameters,
    channels_last MIOpen backbone, fused GridNet head and SE epilogues), a 64-env x 24-step rollout
    through the GridNet sampler (C5's 64 envs per GPU), then one update at the per-GPU minibatch
    B = 768 (6,144 / 8 ranks) with the C5 hyperparameters (ppo-Microrts.yml:511-565, first schedule
    phase): gradient accumulation, K = 3 critics, multi_reward_weights, per-critic vf_coef, vf
    halving, 2 epochs.  Checks: finite stats and grad norms; Adam's per-step bound (|dp| <= ~lr per
    optimizer step); most parameters move; and, under MIOpen's deterministic solvers, the update is
    bitwise reproducible from the same weights, rollout and permutations.  (Gradient accumulation
    runs the minibatches eagerly: there is no graph-replayed variant of this update to compare.)"""
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator

    dev = torch.device("cuda", 0)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        torch.manual_seed(1)
        env = SyntheticVecEnv(64, kind="microrts", seed=1, obs_pool=2)
        pol = ActorCritic(env, actor_head_style="squeeze_unet", channels_per_level=[128, 128, 128],
                          **{k: v for k, v in C5_KW.items() if k != "init_layers_orthogonal"}).to(dev)
        assert sum(p.numel() for p in pol.parameters()) == 5458513
        kw = dict(batch_size=768, n_epochs=2, gamma=[0.99, 0.999, 0.999], gae_lambda=[0.95, 0.99, 0.99],
                  clip_range=0.1, clip_range_vf=None, ppo2_vf_coef_halving=True, max_grad_norm=0.5,
                  gradient_accumulation=True, multi_reward_weights=[0.8, 0.01, 0.19], vf_coef=[0.5, 0.1, 0.2],
                  ent_coef=0.01, learning_rate=1e-4)
        gen = SyncStepRolloutGenerator(pol, env, n_steps=24, seed=1)
        r = gen.rollout(gamma=np.array(kw["gamma"]), gae_lambda=np.array(kw["gae_lambda"]))
        assert tuple(r.values.shape) == (24, 64, 3) and bool(torch.isfinite(r.advantages).all())
        p0 = torch.nn.utils.parameters_to_vector(pol.parameters()).detach().clone()
        runs = []
        for _ in range(2):
            torch.nn.utils.vector_to_parameters(p0, pol.parameters())
            algo = PPO(pol, dev, None, **kw)
            g = torch.Generator(device="cpu").manual_seed(5)
            r._perm_source = lambda n: torch.randperm(n, generator=g)
            stats, norms, K = algo.update(r)
            torch.cuda.synchronize()
            runs.append((algo.flat.vector().detach().cpu().numpy().copy(), stats.copy(), norms.copy(),
                         algo.optimizer.step_count, K))
        (pa, sa, na, ca, K), (pb, sb, nb, cb, _) = runs
        assert K == 3 and ca == cb == 2  # one optimizer step per epoch under gradient accumulation
        assert np.isfinite(sa).all() and np.isfinite(na).all() and (na > 0).all()
        dp = np.abs(pa - p0.cpu().numpy())
        assert dp.max() <= 1.01 * kw["learning_rate"] * ca * 3.2
        # nearly every parameter tensor moves.  Exactly zero gradients do occur at this seed: a
        # squeeze-excitation block whose 8 ReLU units are all inactive on the pooled input passes no
        # gradient to its two fc weights (network.backbone.*.residual.3.fc.*, 1,024 elements each)
        off, still = 0, []
        for name_, p_ in pol.named_parameters():
            n_ = p_.numel()
            if dp[off:off + n_].max() == 0:
                still.append(name_)
            off += n_
        n_t = sum(1 for _ in pol.parameters())
        assert len(still) <= 0.1 * n_t and all(".fc." in n for n in still), still
        assert (dp > 0).mean() > 0.5
        np.testing.assert_array_equal(pa, pb)
        np.testing.assert_array_equal(na, nb)
        np.testing.assert_array_equal(sa, sb)
    finally:
        torch.backends.cudnn.deterministic = det
