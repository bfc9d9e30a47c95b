"""Config C3 (PongNoFrameskip-v4, NatureCNN, 1024 envs x 128 steps) on the GPU.

1. Parity with the REFERENCE: three PPO minibatch steps of the reference's own
   PPO.learn_epoch on its NatureCNN actor-critic (tests/golden/pong_steps.npz, made by
   tests/golden/make_golden_pong.py), replayed through the product path — uint8 frames
   gathered from the HBM rollout, the `/range_size` prescale (rl_algo_impls/shared/encoder/
   cnn.py:24-27), the NatureCNN convolutions on MIOpen (NHWC by default, NCHW as the
   alternative), the Categorical head through the fused GridNet operator, the fused PPO loss
   kernel, autograd, and the fused clip_grad_norm_ + Adam, with and without hipGraph replay.
2. The full C3 shape: one rollout of 1024 envs x 128 steps and one update with the
   `_atari` hyperparameters; GAE bit-exact against the C oracle at full size, finite stats,
   Adam's per-step bound on every parameter, and graph replay == eager loop for one epoch.
"""
import json
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from rl_algo_impls_amd import _lib
from rl_algo_impls_amd import policy as policy_mod
from rl_algo_impls_amd.ppo import PPO
from rl_algo_impls_amd.rollout import DeviceRollout, SyncStepRolloutGenerator
import make_golden_networks as nets

sys.path.insert(0, str(GOLDEN))
from make_golden_pong import pong_init  # noqa: E402  (numpy-only recipe, no reference import)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class Recorder:
    def __init__(self):
        self.scalars = {}

    def add_scalar(self, tag, value, global_step=None):
        self.scalars[tag] = float(value)


def _pong_policy(shapes=None):
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(7)
    pol = ActorCritic(nets.pong_env(), activation_fn="relu")
    got = [list(p.shape) for p in pol.parameters()]
    if shapes is not None:
        assert got == shapes, "NatureCNN module tree differs from the reference's"
    return pol


def _fixture_rollout(z, meta):
    """The fixture's minibatches, in order, as one HBM rollout (T=1, N=n*B) whose advantages
    and returns are the fixture's and whose permutation is the identity: the product path's
    gather then hands the kernels exactly the reference's minibatches."""
    n = meta["n"]
    cat = lambda f: np.concatenate([z[f"b{i}_{f}"] for i in range(n)])[None]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    obs, act, lp, val = t(cat("obs")), t(cat("actions")), t(cat("logprobs")), t(cat("values"))
    N = obs.shape[1]
    r = DeviceRollout(DEV, t(np.zeros(N, np.bool_)), t(np.zeros(N, np.float32)), obs, act,
                      t(np.zeros((1, N), np.float32)), t(np.zeros((1, N), np.bool_)), val, lp, None, 0.99, 0.95,
                      perm_source=lambda k: torch.arange(k))
    r.advantages.copy_(t(cat("advantages")))
    r.returns.copy_(t(cat("returns")))
    return r


@pytest.mark.parametrize("graphs", [True, False], ids=["graph_replay", "eager"])
@pytest.mark.parametrize("layout", ["nhwc_fused", "nhwc_fused_f32", "nhwc_fused_unfolded", "nhwc_fused_overlap", "nhwc",
                                    "nchw"])
def test_pong_minibatch_steps_match_reference(layout, graphs, monkeypatch):
    """nhwc_fused (the default): frames gathered as uint8 channels_last and read by conv1 itself
    (x = u8 / 255 in-kernel, cnn_ops RAI_CONV_U8) and the cnn_ops bias + ReLU epilogues with in-place
    gradient accumulation; nhwc_fused_f32: the same with the gather's uint8 -> float / 255 transform;
    nhwc_fused_unfolded: the fc ReLU backward as its own pass instead of folded into the heads' backward
    (RAI_FC_HEADS_FOLD=0); nhwc_fused_overlap: the weight-gradient partials on a side stream
    (RAI_WGRAD_OVERLAP=1, an option); nhwc: the modules' own kernels on channels_last; nchw: plain NCHW."""
    from rl_algo_impls_amd import cnn_ops

    z = np.load(GOLDEN / "pong_steps.npz", allow_pickle=False)
    meta = json.loads(str(z["index"]))
    monkeypatch.setattr(policy_mod, "_CHANNELS_LAST", layout != "nchw")
    monkeypatch.setattr(policy_mod, "_FUSED_EPILOGUES", layout.startswith("nhwc_fused"))
    monkeypatch.setattr(cnn_ops, "_CONV_U8", layout in ("nhwc_fused", "nhwc_fused_unfolded", "nhwc_fused_overlap"))
    monkeypatch.setattr(cnn_ops, "_FC_HEADS_FOLD", layout != "nhwc_fused_unfolded")
    monkeypatch.setattr(cnn_ops, "_WGRAD_OVERLAP", layout == "nhwc_fused_overlap")
    pol = _pong_policy(meta["shapes"])
    nets.load_flat(pol, pong_init([tuple(s) for s in meta["shapes"]], meta["init_seed"]))
    pol = pol.to(DEV)
    kw = dict(meta["kw"])
    algo = PPO(pol, DEV, Recorder(), n_epochs=1, **kw)
    algo.use_graphs = graphs
    assert algo.fused_mlp_spec() is None
    r = _fixture_rollout(z, meta)
    stats, norms, K = algo.update(r)
    torch.cuda.synchronize()
    if graphs:
        assert algo._graphed is not None and any(g.graph is not None for g in algo._graphed.graphs.values())
        fused_gather = any(g.xforms is not None for g in algo._graphed.graphs.values())
        assert fused_gather == layout.startswith("nhwc_fused")
        if fused_gather:
            kinds = {x.kind for g in algo._graphed.graphs.values() if g.xforms for x in g.xforms if x is not None}
            assert kinds == {_lib.RAI_XFORM_U8_CHW_TO_F32_HWC if layout == "nhwc_fused_f32"
                             else _lib.RAI_XFORM_U8_CHW_TO_U8_HWC}
    lr = float(kw["learning_rate"])
    # pre-clip gradient norms (each step clips to 0.5): fp32, different conv summation order
    np.testing.assert_allclose(norms, z["norms"], rtol=2e-4)
    ref = z["stats"]
    np.testing.assert_allclose(stats[:, :5], ref[:, :5], rtol=2e-4, atol=2e-6)  # loss, pi, entropy, kl, clipfrac
    np.testing.assert_allclose(stats[:, 5], ref[:, 5], rtol=2e-4)  # v_loss
    got = algo.flat.vector().cpu().numpy()  # parameters() order (conv weights are stored channels_last)
    # Adam's first steps move each weight by ~lr * g/|g|; a weight whose gradient is within
    # rounding of zero moves by a rounding-sized fraction of lr: the bound is absolute in lr
    np.testing.assert_allclose(got, z["params"], rtol=1e-4, atol=0.02 * lr)
    init = pong_init([tuple(s) for s in meta["shapes"]], meta["init_seed"])
    moved = np.abs(got - init) > 0.5 * lr
    ref_moved = np.abs(z["params"] - init) > 0.5 * lr
    assert (moved == ref_moved).mean() > 0.999
    sd = algo.optimizer.state_dict()
    assert float(sd["state"][0]["step"]) == meta["opt_step"]
    m = [np.linalg.norm(s["exp_avg"].double().cpu().numpy()) for s in sd["state"].values()]
    np.testing.assert_allclose(m, z["opt_state1_norms"], rtol=2e-3)


def test_pong_full_shape_update():
    """C3 at its BASELINE shape: 1024 envs x 128 steps, batch 256, the `_atari` hyperparameters."""
    import oracle
    from rl_algo_impls_amd.envs import SyntheticVecEnv

    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True  # graph vs eager below compares two runs
    try:
        N, T = 1024, 128
        env = SyntheticVecEnv(N, "pong", seed=1)
        torch.manual_seed(1)
        from rl_algo_impls_amd.policy import ActorCritic

        pol = ActorCritic(env, activation_fn="relu").to(DEV)
        gen = SyncStepRolloutGenerator(pol, env, n_steps=T, seed=1)
        r = gen.rollout(gamma=0.99, gae_lambda=0.95)
        assert r.obs.dtype == torch.uint8 and tuple(r.obs.shape) == (T, N, 4, 84, 84)
        adv_ref, ret_ref = oracle.gae_c(r.rewards.cpu().numpy(), r.values.cpu().numpy(),
                                        r.episode_starts.cpu().numpy(), r.next_episode_starts.cpu().numpy(),
                                        r.next_values.cpu().numpy(), 0.99, 0.95)
        np.testing.assert_array_equal(r.advantages.cpu().numpy(), adv_ref)
        np.testing.assert_array_equal(r.returns.cpu().numpy(), ret_ref)
        acts = r.actions.cpu().numpy()
        assert acts.min() >= 0 and acts.max() < 6
        lp = r.logprobs.cpu().numpy()
        assert np.isfinite(lp).all() and (lp <= 0).all()

        kw = dict(batch_size=256, learning_rate=2.5e-4, clip_range=0.1, vf_coef=0.5, ent_coef=0.01)
        p0 = torch.nn.utils.parameters_to_vector(pol.parameters()).detach().clone()
        results = []
        for graphs in (True, False):
            torch.nn.utils.vector_to_parameters(p0, pol.parameters())
            algo = PPO(pol, DEV, None, n_epochs=1, **kw)
            algo.use_graphs = graphs
            g = torch.Generator(device="cpu").manual_seed(5)
            r._perm_source = lambda n: torch.randperm(n, generator=g)
            stats, norms, _ = algo.update(r)
            torch.cuda.synchronize()
            results.append((algo.flat.vector().detach().cpu().numpy().copy(), stats.copy(), norms.copy(),
                            algo.optimizer.step_count))
        (pg, sg, ng, cg), (pe, se, ne, ce) = results
        nmb = (N * T) // 256
        assert cg == ce == nmb
        assert np.isfinite(sg[:, :6]).all() and np.isfinite(ng).all() and (ng > 0).all()
        # Adam moves a parameter by at most ~lr per step (bias-corrected m/sqrt(v) <= ~1)
        dp = np.abs(pg - p0.cpu().numpy())
        assert dp.max() <= 1.01 * kw["learning_rate"] * nmb * 3.2
        assert (dp > 0).mean() > 0.9
        # the graph-replayed epoch and the eager loop run the same kernels on the same minibatches
        np.testing.assert_allclose(ng, ne, rtol=1e-3)
        np.testing.assert_allclose(sg[:, :6], se[:, :6], rtol=1e-3, atol=1e-6)
        np.testing.assert_allclose(pg, pe, rtol=1e-3, atol=2e-5)
    finally:
        torch.backends.cudnn.deterministic = det


@pytest.mark.parametrize("deterministic", [True, False], ids=["deterministic", "default"])
def test_c3_update_reproducibility(deterministic, tmp_path, monkeypatch):
    """The reference runs with torch.use_deterministic_algorithms(True) by default
    (rl_algo_impls/runner/running_utils.py:161-166).  Under running_utils.set_device_optimizations
    the same C3 update from the same weights, rollout and permutations is bitwise reproducible
    (HIP kernels: fixed reduction orders; MIOpen / hipBLASLt: deterministic solvers).  Without it
    the two runs agree within fp32 summation tolerance (MIOpen may pick split-K atomics).
    Each mode runs in a process of its own with its own MIOpen user database: MIOpen's recorded
    solver choices outlive a process, and the deterministic ones are ~100x slower at these shapes."""
    import multiprocessing as mp
    import queue
    import time

    import dp_worker

    monkeypatch.setenv("MIOPEN_USER_DB_PATH", str(tmp_path))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=dp_worker.c3_repro_worker, args=(q, deterministic))
    p.start()
    deadline = time.time() + 240
    while True:
        try:
            (pa, na), (pb, nb) = q.get(timeout=2)
            break
        except queue.Empty:
            assert p.exitcode in (None, 0), f"worker exited with {p.exitcode}"
            assert time.time() < deadline, "worker did not report in time"
    p.join(timeout=60)
    assert p.exitcode == 0
    if deterministic:
        np.testing.assert_array_equal(pa, pb)
        np.testing.assert_array_equal(na, nb)
    else:
        # MIOpen's split-K atomics reorder fp32 sums run to run: the first step's gradient norm
        # agrees to rounding; afterwards Adam's early, sign-like steps (|step| <= ~lr) can move a
        # near-zero-gradient weight either way, so parameters only agree within lr per step
        np.testing.assert_allclose(na[0], nb[0], rtol=1e-4)
        assert np.abs(pa - pb).max() <= 2 * 2.5e-4 * len(na)
