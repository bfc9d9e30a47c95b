"""Parity of the gfx950 kernels against the oracle and the reference's golden vectors.
Every test calls through the C ABI (librai_amd.so)."""
import json

import numpy as np
import pytest
import torch

import oracle
from rl_algo_impls_amd import _lib
from rl_algo_impls_amd.gae import EXACT, FAST, compute_advantages, compute_advantages_device
from rl_algo_impls_amd.pg_common import DeviceBlocks, launch_loss, make_hparams
from rl_algo_impls_amd.rollout import feistel_permutation, gather_rows

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


# ---------------------------------------------------------------- GAE ----------------
def test_gae_golden_bit_exact_numpy_dropin(gae_cases):
    for c in gae_cases:
        adv = compute_advantages(c["rewards"], c["values"], c["episode_starts"], c["next_episode_starts"],
                                 c["next_values"], c["gamma"], c["lam"])
        assert adv.dtype == np.float32
        np.testing.assert_array_equal(adv, c["adv"], err_msg=f"case {c['idx']}")


def test_gae_golden_returns_fused(gae_cases):
    for c in gae_cases:
        adv, ret = compute_advantages_device(dev(c["rewards"]), dev(c["values"]), dev(c["episode_starts"]),
                                             dev(c["next_episode_starts"]), dev(c["next_values"]),
                                             c["gamma"], c["lam"], want_returns=True)
        np.testing.assert_array_equal(adv.cpu().numpy(), c["adv"])
        np.testing.assert_array_equal(ret.cpu().numpy(), c["returns"])


@pytest.mark.parametrize("T,N,K,dens", [(128, 4096, 1, 0.005), (512, 2048, 1, 0.001), (37, 999, 3, 0.05),
                                        (128, 65536, 1, 0.005),
                                        # the 4-columns-per-lane streaming kernel (C >= 2^18, C % 4 == 0):
                                        # K = 1 (start bytes read 4 at a time), K = 3 vector gamma, and T
                                        # not a multiple of its 8-row chunks
                                        (19, 1 << 18, 1, 0.02), (13, 87384, 3, 0.05), (8, 262148, 1, 1.0)])
def test_gae_full_size_exact_vs_c_oracle(T, N, K, dens):
    rng = np.random.default_rng(T * N + K)
    shp = (T, N) if K == 1 else (T, N, K)
    r = rng.standard_normal(shp, dtype=np.float32)
    v = rng.standard_normal(shp, dtype=np.float32) * 5
    es = rng.random((T, N)) < dens
    nes = rng.random(N) < dens
    nv = rng.standard_normal(shp[1:], dtype=np.float32)
    gamma = 0.99 if K == 1 else np.array([0.99, 0.995, 0.9][:K])
    adv_ref, ret_ref = oracle.gae_c(r, v, es, nes, nv, gamma, 0.95)
    adv, ret = compute_advantages_device(dev(r), dev(v), dev(es), dev(nes), dev(nv), gamma, 0.95,
                                         want_returns=True)
    np.testing.assert_array_equal(adv.cpu().numpy(), adv_ref)
    np.testing.assert_array_equal(ret.cpu().numpy(), ret_ref)


@pytest.mark.parametrize("D,NT,NTM", [("8", "256", "0"), ("4", "256", "0"), ("8", "512", "0"), ("4", "1024", "0"),
                                      ("4", "1024", "1"), ("8", "default", "1")])
def test_gae_stream_kernel_rows_in_flight_variants(D, NT, NTM, monkeypatch):
    """Both chunk depths of the streaming GAE kernel (RAI_GAE_STREAM_D) and the tiled kernel forced on
    the same large input (RAI_GAE_STREAM=0) give the C oracle's bits."""
    rng = np.random.default_rng(41)
    T, N = 21, 1 << 18
    r = rng.standard_normal((T, N), dtype=np.float32)
    v = rng.standard_normal((T, N), dtype=np.float32)
    es = rng.random((T, N)) < 0.03
    nes = rng.random(N) < 0.03
    nv = rng.standard_normal(N, dtype=np.float32)
    adv_ref, ret_ref = oracle.gae_c(r, v, es, nes, nv, 0.98, 0.8)
    for stream in ("1", "0"):
        monkeypatch.setenv("RAI_GAE_STREAM_D", D)
        monkeypatch.setenv("RAI_GAE_STREAM_NT", NT)
        monkeypatch.setenv("RAI_GAE_NT", NTM)  # nontemporal loads / stores
        monkeypatch.setenv("RAI_GAE_STREAM", stream)
        adv, ret = compute_advantages_device(dev(r), dev(v), dev(es), dev(nes), dev(nv), 0.98, 0.8, want_returns=True)
        np.testing.assert_array_equal(adv.cpu().numpy(), adv_ref)
        np.testing.assert_array_equal(ret.cpu().numpy(), ret_ref)
    fast, _ = compute_advantages_device(dev(r), dev(v), dev(es), dev(nes), dev(nv), 0.98, 0.8, mode=FAST)
    np.testing.assert_allclose(fast.cpu().numpy(), adv_ref, rtol=1e-5, atol=1e-5)


def test_gae_fast_mode_tolerance():
    rng = np.random.default_rng(3)
    T, N = 256, 1000
    r = rng.standard_normal((T, N), dtype=np.float32)
    v = rng.standard_normal((T, N), dtype=np.float32)
    es = rng.random((T, N)) < 0.01
    nes = rng.random(N) < 0.01
    nv = rng.standard_normal(N, dtype=np.float32)
    ref, _ = oracle.gae_c(r, v, es, nes, nv, 0.99, 0.95)
    adv, _ = compute_advantages_device(dev(r), dev(v), dev(es), dev(nes), dev(nv), 0.99, 0.95, mode=FAST)
    np.testing.assert_allclose(adv.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("T,N,K", [(1, 1, 1), (5, 7, 1), (128, 4096, 1), (33, 200, 1), (1024, 100, 1),
                                   (1025, 100, 1), (128, 700, 3), (64, 20000, 1), (200, 9000, 1)])
def test_gae_fast_mode_affine_scan(T, N, K, monkeypatch):
    """Fast mode's chunked affine scan (gae_scan_kernel: segments of <= 32 rows, 16 / 32 / 64 columns per
    block; T = 1025 at 100 columns falls back to the serial fp32 chain) against the exact C oracle and
    against the serial fp32 chain (RAI_GAE_SCAN=0), at fast mode's tolerance; episode starts dense enough
    to cut every segment, and none in some columns (long carries)."""
    rng = np.random.default_rng(T * 7 + N + K)
    shp = (T, N) if K == 1 else (T, N, K)
    r = rng.standard_normal(shp, dtype=np.float32)
    v = rng.standard_normal(shp, dtype=np.float32)
    es = rng.random((T, N)) < 0.05
    es[:, : N // 3] = False
    nes = rng.random(N) < 0.05
    nv = rng.standard_normal(shp[1:], dtype=np.float32)
    g = 0.99 if K == 1 else np.array([0.99, 0.995, 0.999])
    lam = 0.95 if K == 1 else np.array([0.95, 0.9, 0.99])
    adv_ref, ret_ref = oracle.gae_c(r, v, es, nes, nv, g, lam)
    tol = dict(rtol=1e-5, atol=1e-5 * max(1.0, float(np.abs(adv_ref).max())))
    fast, fret = compute_advantages_device(dev(r), dev(v), dev(es), dev(nes), dev(nv), g, lam, mode=FAST,
                                           want_returns=True)
    np.testing.assert_allclose(fast.cpu().numpy(), adv_ref, **tol)
    np.testing.assert_allclose(fret.cpu().numpy(), ret_ref, **tol)
    monkeypatch.setenv("RAI_GAE_SCAN", "0")
    serial, _ = compute_advantages_device(dev(r), dev(v), dev(es), dev(nes), dev(nv), g, lam, mode=FAST)
    np.testing.assert_allclose(fast.cpu().numpy(), serial.cpu().numpy(), **tol)


def test_gae_edge_cases():
    # T=1, N=1; all starts; no starts; ragged column count (not a multiple of 64)
    for T, N in [(1, 1), (1, 65), (33, 63), (64, 129)]:
        for dens in (0.0, 1.0):
            rng = np.random.default_rng(T + N)
            r = rng.standard_normal((T, N), dtype=np.float32)
            v = rng.standard_normal((T, N), dtype=np.float32)
            es = np.full((T, N), dens > 0)
            nes = np.full(N, dens > 0)
            nv = rng.standard_normal(N, dtype=np.float32)
            ref = oracle.compute_advantages(r, v, es, nes, nv, 0.98, 0.8)
            np.testing.assert_array_equal(compute_advantages(r, v, es, nes, nv, 0.98, 0.8), ref)


def test_gae_shape_errors_match_reference():
    r = np.zeros((4, 3), np.float32)
    with pytest.raises(AssertionError):
        compute_advantages(r, r, np.zeros((4, 3), bool), np.zeros(2, bool), np.zeros(3, np.float32), 0.9, 0.9)


def test_gae_linearity_property_full_size():
    """Size-independent property at the BASELINE size: GAE is linear in (r, V) for fixed
    episode boundaries, so adv(r1+r2) ~= adv(r1) + adv(r2) (fp tolerance)."""
    T, N = 128, 4096
    rng = np.random.default_rng(9)
    es = dev(rng.random((T, N)) < 0.005)
    nes = dev(rng.random(N) < 0.005)
    z = torch.zeros((T, N), device=DEV)
    zn = torch.zeros(N, device=DEV)
    r1 = torch.randn((T, N), device=DEV)
    r2 = torch.randn((T, N), device=DEV)
    a1, _ = compute_advantages_device(r1, z, es, nes, zn, 0.99, 0.95)
    a2, _ = compute_advantages_device(r2, z, es, nes, zn, 0.99, 0.95)
    a12, _ = compute_advantages_device(r1 + r2, z, es, nes, zn, 0.99, 0.95)
    torch.testing.assert_close(a12, a1 + a2, rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------- loss ---------------
def _golden_loss_inputs(z, name, meta, i=0):
    import make_golden_networks as nets

    policy = nets.build(meta["policy"])
    nets.load_flat(policy, z[f"{name}/init"])
    p = f"{name}/b{i}_"
    with torch.no_grad():
        lp, ent, v = policy(torch.from_numpy(z[p + "obs"]), torch.from_numpy(z[p + "actions"]))
    return lp.numpy(), ent.numpy(), v.numpy(), z[p + "logprobs"], z[p + "values"], z[p + "advantages"], z[p + "returns"]


def _kw_to_hparams(kw, K, algo="ppo", grad_scale=1.0):
    return make_hparams(
        loss_kind=0 if algo == "ppo" else 1, K=K, clip_range=kw.get("clip_range", 0.2),
        clip_range_vf=kw.get("clip_range_vf"), ent_coef=kw.get("ent_coef", 0.0), vf_coef=kw.get("vf_coef", 0.5),
        vf_weights=kw.get("vf_weights"), multi_reward_weights=kw.get("multi_reward_weights"),
        normalize_advantage=kw.get("normalize_advantage", True),
        standardize_advantage=kw.get("standardize_advantage", False),
        normalize_after_scaling=kw.get("normalize_advantages_after_scaling", False),
        ppo2_vf_coef_halving=kw.get("ppo2_vf_coef_halving", False), kl_cutoff=kw.get("kl_cutoff"),
        vf_loss_fn=kw.get("vf_loss_fn", "mse_loss"), grad_scale=grad_scale)


def test_loss_kernel_matches_oracle_on_golden_batches(golden):
    z = golden("ppo_steps.npz")
    index = json.loads(str(z["index"]))
    for name, meta in index.items():
        lp, ent, v, olp, ov, adv, ret = _golden_loss_inputs(z, name, meta)
        K = meta["K"]
        gs = 1.0 / meta["n"] if meta["kw"].get("gradient_accumulation") else 1.0
        blocks = DeviceBlocks(DEV)
        blocks.ensure_tables(4, 4)
        blocks.upload(_kw_to_hparams(meta["kw"], K, grad_scale=gs), 0)
        d_lp, d_ent, d_v = launch_loss(blocks, dev(lp), dev(ent), dev(v), dev(olp), dev(ov), dev(adv), dev(ret), K)
        hp = dict(meta["kw"], algo="ppo", grad_scale=gs)
        r_lp, r_ent, r_v, st = oracle.pg_loss_grads(lp, ent, v, olp, ov, adv, ret, hp)
        np.testing.assert_allclose(d_lp.cpu().numpy(), r_lp, rtol=2e-5, atol=1e-8, err_msg=name)
        np.testing.assert_allclose(d_ent.cpu().numpy(), r_ent, rtol=1e-6, atol=0, err_msg=name)
        np.testing.assert_allclose(d_v.cpu().numpy(), r_v, rtol=2e-5, atol=1e-8, err_msg=name)
        row = blocks.stats[0].cpu().numpy()
        np.testing.assert_allclose(row[0], st["loss"], rtol=2e-5, atol=1e-7, err_msg=name)
        np.testing.assert_allclose(row[1], st["pi_loss"], rtol=2e-5, atol=1e-7, err_msg=name)
        np.testing.assert_allclose(row[2], st["entropy_loss"], rtol=2e-5, atol=1e-7, err_msg=name)
        np.testing.assert_allclose(row[3], st["approx_kl"], rtol=1e-4, atol=1e-8, err_msg=name)
        np.testing.assert_allclose(row[4], st["clipped_frac"], rtol=1e-6, err_msg=name)
        # reference step stats (PPO.learn_epoch's TrainStepStats) agree as well
        ref_row = z[f"{name}/stats"][0]
        np.testing.assert_allclose(row[:5], ref_row[:5], rtol=1e-4, atol=1e-6, err_msg=name)


def test_loss_kernel_a2c_and_large_batch():
    rng = np.random.default_rng(4)
    for B in (1000, 70000):
        lp = rng.standard_normal(B, dtype=np.float32)
        ent = rng.random(B, dtype=np.float32)
        v = rng.standard_normal(B, dtype=np.float32)
        adv = rng.standard_normal(B, dtype=np.float32) * 3
        ret = rng.standard_normal(B, dtype=np.float32)
        for algo in ("ppo", "a2c"):
            kw = dict(ent_coef=0.01, normalize_advantage=(algo == "ppo"))
            blocks = DeviceBlocks(DEV)
            blocks.upload(_kw_to_hparams(kw, 1, algo=algo), 0)
            olp = lp + rng.standard_normal(B, dtype=np.float32) * 0.1
            d_lp, d_ent, d_v = launch_loss(blocks, dev(lp), dev(ent), dev(v), dev(olp), dev(v), dev(adv),
                                           dev(ret), 1)
            r_lp, r_ent, r_v, st = oracle.pg_loss_grads(lp, ent, v, olp, v, adv, ret, dict(kw, algo=algo, clip_range=0.2))
            np.testing.assert_allclose(d_lp.cpu().numpy(), r_lp, rtol=3e-5, atol=1e-10)
            np.testing.assert_allclose(d_v.cpu().numpy(), r_v, rtol=3e-5, atol=1e-10)
            np.testing.assert_allclose(d_ent.cpu().numpy(), r_ent, rtol=1e-6)


def test_loss_kernel_tie_semantics():
    """ratio exactly 1 (ties in min) and ratio on the clip boundary follow autograd."""
    B = 8
    lp = np.zeros(B, np.float32)
    adv = np.array([1, -1, 2, -2, 0.5, -0.5, 3, -3], np.float32)
    kw = dict(normalize_advantage=False)
    blocks = DeviceBlocks(DEV)
    blocks.upload(_kw_to_hparams(kw, 1), 0)
    zeros = np.zeros(B, np.float32)
    d_lp, _, _ = launch_loss(blocks, dev(lp), dev(zeros), dev(zeros), dev(lp), dev(zeros), dev(adv), dev(zeros), 1)
    # autograd reference
    t = torch.zeros(B, requires_grad=True)
    ratio = torch.exp(t - torch.from_numpy(lp))
    A = torch.from_numpy(adv)
    loss = -torch.min(ratio * A, torch.clamp(ratio, 0.8, 1.2) * A).mean()
    loss.backward()
    np.testing.assert_allclose(d_lp.cpu().numpy(), t.grad.numpy(), rtol=1e-6)


# ---------------------------------------------------------------- optimizer -----------
def test_clip_adam_matches_torch_over_steps():
    from rl_algo_impls_amd.optim import FlatOptimizer, FlatParams

    torch.manual_seed(0)
    for P_sizes in ([9155 - 130, 130], [3, 5, 7], [1 << 20, 37]):
        ref_params = [torch.nn.Parameter(torch.randn(n, dtype=torch.float64)) for n in P_sizes]
        mod = torch.nn.ParameterList([torch.nn.Parameter(p.detach().float().clone()) for p in ref_params]).to(DEV)
        flat = FlatParams(mod, DEV)
        opt = FlatOptimizer(flat, FlatOptimizer.ADAM, lr=1e-3, eps=1e-7, max_grad_norm=0.5)
        blocks = DeviceBlocks(DEV)
        blocks.ensure_tables(1, 8)
        blocks.upload(make_hparams(loss_kind=0, K=1), 0)
        p64 = [p.detach().double().clone() for p in ref_params]
        m = [torch.zeros_like(p) for p in p64]
        v = [torch.zeros_like(p) for p in p64]
        for step in range(1, 6):
            grads = [torch.randn(n, dtype=torch.float64) * (0.01 if step % 2 else 3) for n in P_sizes]
            for pp, g in zip(mod, grads):
                pp.grad.copy_(g.float())
            opt.step(blocks.state, blocks.norms)
            tot = torch.sqrt(sum((g.double() ** 2).sum() for g in grads))
            coef = min(0.5 / (tot + 1e-6), 1.0)
            for i, g in enumerate(grads):
                g = g * coef
                m[i] = m[i] + 0.1 * (g - m[i])
                v[i] = v[i] * 0.999 + 0.001 * g * g
                bc1, bc2 = 1 - 0.9 ** step, 1 - 0.999 ** step
                p64[i] = p64[i] - (1e-3 / bc1) * m[i] / (torch.sqrt(v[i]) / np.sqrt(bc2) + 1e-7)
            norms = blocks.norms[:step].cpu().numpy()
            np.testing.assert_allclose(norms[-1], float(tot), rtol=1e-5)
            for pp, ref in zip(mod, p64):
                np.testing.assert_allclose(pp.detach().cpu().numpy(), ref.numpy(), rtol=1e-4, atol=2e-6)
            assert float(flat.grad.abs().max()) == 0.0  # zero_grad
        sd = opt.state_dict()
        assert sd["state"][0]["step"].item() == 5.0


@pytest.mark.parametrize("P", [9155, 143_367, 1_690_003, 3_000_001])
@pytest.mark.parametrize("kind", [0, 1])
def test_clip_optim_matches_torch_at_config_sizes(P, kind):
    """clip_grad_norm_ + Adam(eps=1e-7) / RMSprop(alpha=0.99, eps=1e-5) over six steps of alternating
    large and small gradients (clipping on and off) against torch.optim on the same device, at the
    C2, C4 and C3 parameter counts and one past them (float4 body + scalar tail): parameters, both
    moments and the pre-clip norms within fp32 tolerance (rl_algo_impls/ppo/ppo.py:441-447,
    rl_algo_impls/a2c/a2c.py:45-50,202-205), and the flat gradient zeroed."""
    from rl_algo_impls_amd.optim import FlatOptimizer, FlatParams

    torch.manual_seed(1)
    init = torch.randn(P)
    mod = torch.nn.ParameterList([torch.nn.Parameter(init.clone())]).to(DEV)
    flat = FlatParams(mod, DEV)
    eps = 1e-7 if kind == 0 else 1e-5
    opt = FlatOptimizer(flat, kind, lr=1e-3, eps=eps, max_grad_norm=0.5)
    ref_p = torch.nn.Parameter(init.clone().to(DEV))
    ref = (torch.optim.Adam([ref_p], lr=1e-3, eps=eps) if kind == 0 else
           torch.optim.RMSprop([ref_p], lr=1e-3, alpha=0.99, eps=eps))
    blocks = DeviceBlocks(DEV)
    blocks.ensure_tables(1, 8)
    blocks.upload(make_hparams(loss_kind=0, K=1), 0)
    g = torch.Generator().manual_seed(7)
    ref_norms = []
    for step in range(6):
        grad = (torch.randn(P, generator=g) * (0.01 if step % 2 else 3)).to(DEV)
        flat.grad.copy_(grad)
        opt.step(blocks.state, blocks.norms)
        ref_p.grad = grad.clone()
        ref_norms.append(float(torch.nn.utils.clip_grad_norm_([ref_p], 0.5)))
        ref.step()
    torch.cuda.synchronize()
    assert int(blocks.state.cpu()[0:8].view(torch.int64)[0]) == 6
    np.testing.assert_allclose(blocks.norms[:6].cpu().numpy(), ref_norms, rtol=1e-5)
    np.testing.assert_allclose(flat.flat.cpu().numpy(), ref_p.detach().cpu().numpy(), rtol=1e-4, atol=2e-6)
    st = ref.state[ref_p]
    np.testing.assert_allclose(opt.state1.cpu().numpy(),
                               (st["exp_avg"] if kind == 0 else st["square_avg"]).cpu().numpy(),
                               rtol=1e-4, atol=1e-9)
    if kind == 0:
        np.testing.assert_allclose(opt.state2.cpu().numpy(), st["exp_avg_sq"].cpu().numpy(), rtol=1e-4, atol=1e-12)
    assert float(flat.grad.abs().max()) == 0.0


def test_optimizer_state_dict_loads_into_torch_adam():
    from rl_algo_impls_amd.optim import FlatOptimizer, FlatParams

    mod = torch.nn.Linear(5, 3).to(DEV)
    flat = FlatParams(mod, DEV)
    opt = FlatOptimizer(flat, FlatOptimizer.ADAM, lr=3e-4, eps=1e-7)
    blocks = DeviceBlocks(DEV)
    blocks.upload(make_hparams(loss_kind=0, K=1), 0)
    flat.grad.normal_()
    opt.step(blocks.state, None)
    sd = opt.state_dict()
    t = torch.optim.Adam(mod.parameters(), lr=3e-4, eps=1e-7)
    t.load_state_dict(sd)
    assert t.state_dict()["state"][1]["exp_avg"].shape == (3,)
    opt2 = FlatOptimizer(flat, FlatOptimizer.ADAM, lr=1.0, eps=1e-7)
    opt2.load_state_dict(t.state_dict())
    torch.testing.assert_close(opt2.state1, opt.state1)
    assert opt2.step_count == 1 and opt2.lr == 3e-4


# ---------------------------------------------------------------- gather / sample -----
def test_gather_rows_multi_field():
    rng = np.random.default_rng(0)
    n = 5000
    fields = [rng.integers(0, 255, (n, 4, 84, 84), dtype=np.uint8)[:, :, :, :1],  # 336-B rows
              rng.standard_normal((n, 4), dtype=np.float32),
              rng.integers(0, 6, n).astype(np.int64),
              rng.standard_normal((n, 17), dtype=np.float32),  # 68-B rows
              rng.integers(0, 2, (n, 3)).astype(np.bool_)]   # 3-B rows
    srcs = [dev(np.ascontiguousarray(f)) for f in fields]
    idx = rng.permutation(n)[:3000]
    dsts = [torch.empty((3000,) + tuple(s.shape[1:]), dtype=s.dtype, device=DEV) for s in srcs]
    gather_rows(srcs, dsts, dev(idx))
    for f, d in zip(fields, dsts):
        np.testing.assert_array_equal(d.cpu().numpy(), np.ascontiguousarray(f)[idx])


@pytest.mark.parametrize("n", [1, 2, 3, 64, 1000, 4097, 524288, (1 << 20) + 7])
def test_feistel_permutation_matches_spec_and_is_bijection(n):
    """rai_feistel_permutation (the epoch shuffle) equals oracle.feistel_permutation bit for bit, is a
    bijection of [0, n) (sortedness of the sorted output) and depends on the key."""
    for key in (0, 0x1234567890ABCDEF, 2**64 - 1):
        got = feistel_permutation(n, DEV, key=key).cpu().numpy()
        np.testing.assert_array_equal(got, oracle.feistel_permutation(n, key))
        np.testing.assert_array_equal(np.sort(got), np.arange(n))
    if n >= 64:
        a = feistel_permutation(n, DEV, key=1).cpu().numpy()
        b = feistel_permutation(n, DEV, key=2).cpu().numpy()
        assert (a != b).mean() > 0.9
        assert 0.3 < np.abs(a - np.arange(n)).mean() / n < 0.37  # E|p(i) - i| = n/3 for a uniform shuffle


def test_feistel_permutation_edge_cases():
    assert _lib.lib().rai_feistel_permutation(0, 5, None, None) == 0
    assert _lib.lib().rai_feistel_permutation(-1, 5, None, None) != 0
    assert _lib.lib().rai_feistel_permutation(4, 5, None, None) != 0


def test_categorical_sample_distribution_and_logp():
    L = _lib.lib()
    N, A = 200000, 6
    logits = torch.randn(8, A, device=DEV).repeat(N // 8, 1).contiguous()
    acts = torch.empty(N, dtype=torch.int64, device=DEV)
    logp = torch.empty(N, dtype=torch.float32, device=DEV)
    v = torch.randn(N, device=DEV)
    vo = torch.empty(N, device=DEV)
    rc = L.rai_categorical_sample(logits.data_ptr(), None, N, A, 1234, 7, acts.data_ptr(), logp.data_ptr(),
                                  v.data_ptr(), vo.data_ptr(), 1, _lib.stream_handle())
    _lib.check(rc, "sample")
    a = acts.cpu().numpy()
    assert a.min() >= 0 and a.max() < A
    np.testing.assert_allclose(logp.cpu().numpy(), oracle.categorical_logp(logits.cpu().numpy(), a), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(vo, v)
    probs = torch.softmax(logits[:8], -1).cpu().numpy()
    for row in range(8):
        freq = np.bincount(a[row::8], minlength=A) / (N // 8)
        np.testing.assert_allclose(freq, probs[row], atol=0.015)
    # masked: never picks a masked action
    mask = torch.zeros(N, A, dtype=torch.uint8, device=DEV)
    mask[:, 2] = 1
    mask[::2, 4] = 1
    rc = L.rai_categorical_sample(logits.data_ptr(), mask.data_ptr(), N, A, 99, 0, acts.data_ptr(), logp.data_ptr(),
                                  None, None, 0, _lib.stream_handle())
    _lib.check(rc, "sample")
    a = acts.cpu().numpy()
    assert set(np.unique(a)) <= {2, 4}
    assert (a[1::2] == 2).all()


def test_gaussian_sample_moments_logp_clamp():
    L = _lib.lib()
    N, A = 100000, 6
    mu = (torch.arange(A, device=DEV, dtype=torch.float32) * 0.3 - 0.8).repeat(N, 1).contiguous()
    log_std = torch.full((A,), -0.5, device=DEV)
    low = torch.full((A,), -1.0, device=DEV)
    high = torch.full((A,), 1.0, device=DEV)
    acts = torch.empty(N, A, device=DEV)
    cl = torch.empty(N, A, device=DEV)
    lp = torch.empty(N, device=DEV)
    rc = L.rai_gaussian_sample(mu.data_ptr(), log_std.data_ptr(), N, A, low.data_ptr(), high.data_ptr(), 5, 0,
                               acts.data_ptr(), cl.data_ptr(), lp.data_ptr(), None, None, 0, _lib.stream_handle())
    _lib.check(rc, "gaussian")
    a = acts.cpu().numpy()
    np.testing.assert_allclose(a.mean(0), mu[0].cpu().numpy(), atol=0.01)
    np.testing.assert_allclose(a.std(0), np.exp(-0.5), rtol=0.01)
    np.testing.assert_allclose(lp.cpu().numpy(), oracle.gaussian_logp(a, mu.cpu().numpy(), log_std.cpu().numpy()),
                               rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(cl.cpu().numpy(), np.clip(a, -1, 1))


@pytest.mark.parametrize("d,n,act", [(4, 2, "tanh"), (4, 2, "relu"), (6, 3, "tanh"), (8, 8, "relu")])
def test_fused_policy_step_matches_torch_forward_and_sampler(d, n, act):
    """rai_mlp_policy_step (both MLP forwards + categorical sample + slot writes) vs the PyTorch
    forward followed by rai_categorical_sample with the same seed/offset: values and log-probs
    within fp32 tolerance; actions identical except where the uniform draw falls within the
    forward's rounding of a CDF boundary."""
    import ctypes as C

    from rl_algo_impls_amd.envs import Box, Discrete
    from rl_algo_impls_amd.policy import ActorCritic, mlp_actor_critic_spec

    class E:
        single_observation_space = Box(-1.0, 1.0, shape=(d,))
        single_action_space = Discrete(n)
        num_envs = 1

    torch.manual_seed(3)
    pol = ActorCritic(E(), activation_fn=act).to(DEV)
    spec = mlp_actor_critic_spec(pol)
    assert spec is not None
    N = 5000
    obs = torch.randn(N, d, device=DEV) * 2
    ps = [p.detach() for p in pol.parameters()]
    arr = lambda xs: (C.c_void_p * 6)(*[x.data_ptr() for x in xs])
    a1 = torch.empty(N, dtype=torch.int64, device=DEV)
    l1 = torch.empty(N, device=DEV)
    v1 = torch.empty(N, device=DEV)
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    _lib.check(L.rai_mlp_policy_step(arr(ps[:6]), arr(ps[6:]), obs.data_ptr(), N, d, 64, n, spec["activation"], 77, 5,
                                     a1.data_ptr(), l1.data_ptr(), v1.data_ptr(), st), "policy_step")
    with torch.no_grad():
        logits, v = pol.network.dist_params_and_value(obs)
    logits = logits.contiguous().float()
    v = v.contiguous().float()
    a2 = torch.empty(N, dtype=torch.int64, device=DEV)
    l2 = torch.empty(N, device=DEV)
    v2 = torch.empty(N, device=DEV)
    _lib.check(L.rai_categorical_sample(logits.data_ptr(), None, N, n, 77, 5, a2.data_ptr(), l2.data_ptr(),
                                        v.data_ptr(), v2.data_ptr(), 1, st), "categorical_sample")
    torch.cuda.synchronize()
    np.testing.assert_allclose(v1.cpu().numpy(), v2.cpu().numpy(), rtol=1e-4, atol=1e-5)
    same = (a1 == a2).cpu().numpy()
    assert same.mean() > 0.999, same.mean()
    np.testing.assert_allclose(l1.cpu().numpy()[same], l2.cpu().numpy()[same], rtol=1e-4, atol=1e-5)
    # value-only call (bootstrap): same values
    v3 = torch.empty(N, device=DEV)
    _lib.check(L.rai_mlp_policy_step(None, arr(ps[6:]), obs.data_ptr(), N, d, 64, n, spec["activation"], 0, 0,
                                     None, None, v3.data_ptr(), st), "policy_step values")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(v3.cpu().numpy(), v1.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("n,B,shuffle", [(1000, 256, True), (300, 64, True), (77, 32, False), (4096, 1000, True)])
def test_gather_minibatch_next_all_field_granularities(n, B, shuffle):
    """rai_gather_minibatch_next (csrc/rollout.hip) on fields of 16-, 4- and 1-byte units (f32 image
    rows, i64 actions, f32 scalars, u8 masks, odd-width u8 rows), a ragged last minibatch and the
    on-device minibatch advance: every minibatch equals the index-gathered rows, bit for bit, and
    desc->mb / desc->arrivals end at (number of minibatches, 0)."""
    import ctypes as C

    from rl_algo_impls_amd import _lib
    from rl_algo_impls_amd.graphs import GraphedUpdate

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(n + B)
    fields = [torch.randn(n, 4, 9, 7, generator=g).to(dev),                       # 1008 B rows (16-B units)
              torch.randint(0, 9, (n, 3), generator=g).to(dev),                   # 24 B rows (4-B units)
              torch.randn(n, generator=g).to(dev),                                # 4 B rows
              (torch.rand(n, 5, 7, generator=g) < 0.5).to(dev),                   # 35 B rows (1-B units)
              torch.randint(0, 255, (n, 48), generator=g, dtype=torch.uint8).to(dev)]  # 48 B rows
    gu = GraphedUpdate(dev)
    gu.set_rollout(fields, B, shuffle)
    perm = torch.randperm(n, generator=g).to(dev) if shuffle else None
    gu.start_epoch(perm)
    idx = perm if shuffle else torch.arange(n, device=dev)
    row_bytes = [int(f[0].numel() * f.element_size()) for f in fields]
    nmb = (n + B - 1) // B
    for mb in range(nmb):
        rows = min(B, n - mb * B)
        out = [torch.full((B,) + tuple(f.shape[1:]), 7, dtype=f.dtype, device=dev) for f in fields]
        dst = (C.c_void_p * len(out))(*[o.data_ptr() for o in out])
        rb = (C.c_int64 * len(out))(*row_bytes)
        rc = _lib.lib().rai_gather_minibatch_next(gu.desc.data_ptr(), len(out), C.cast(dst, C.c_void_p),
                                                  C.cast(rb, C.c_void_p), B, _lib.stream_handle(dev))
        assert rc == 0
        sel = idx[mb * B: mb * B + rows]
        for f, o in zip(fields, out):
            assert torch.equal(o[:rows], f[sel])
            if rows < B:  # rows past the ragged tail are left untouched
                assert torch.equal(o[rows:], torch.full_like(o[rows:], 7))
    torch.cuda.synchronize()
    d = _lib.MinibatchDesc.from_buffer_copy(bytes(gu.desc.cpu().numpy()))
    assert d.mb == nmb and d.arrivals == 0


@pytest.mark.parametrize("C,H,W,n,B", [(4, 84, 84, 700, 256), (1, 12, 10, 300, 64), (3, 8, 8, 130, 64),
                                       (2, 84, 84, 50, 32)])
def test_gather_minibatch_frame_transform(C, H, W, n, B):
    """rai_gather_minibatch_x with RAI_XFORM_U8_CHW_TO_F32_HWC on a uint8 frame field (the NatureCNN
    prescale obs.float() / range_size of rl_algo_impls/shared/encoder/cnn.py:24-27 fused with the
    channels_last conversion) next to copied fields: every minibatch's frames equal the CPU
    reference's true division bit for bit, in channels_last layout; the copied fields equal the
    index-gathered rows; the ragged tail and the device advance as for the plain gather."""
    from rl_algo_impls_amd.graphs import GraphedUpdate, gather_next, static_buffers

    g = torch.Generator(device="cpu").manual_seed(C * 1000 + n)
    frames = torch.randint(0, 256, (n, C, H, W), generator=g, dtype=torch.uint8)
    fields = [frames.to(DEV), torch.randint(0, 6, (n,), generator=g).to(DEV), torch.randn(n, generator=g).to(DEV)]
    xf = _lib.GatherXform(kind=_lib.RAI_XFORM_U8_CHW_TO_F32_HWC, channels=C, hw=H * W, divisor=255.0)
    xforms = [xf, None, None]
    gu = GraphedUpdate(DEV)
    gu.set_rollout(fields, B, True)
    perm = torch.randperm(n, generator=g)
    gu.start_epoch(perm.to(DEV))
    row_bytes = [int(f[0].numel() * f.element_size()) for f in fields]
    ref = frames.float() / 255.0  # the reference's CPU path: IEEE division
    for mb in range((n + B - 1) // B):
        rows = min(B, n - mb * B)
        bufs = static_buffers(fields, B, DEV, xforms)
        assert bufs[0].dtype == torch.float32 and bufs[0].is_contiguous(memory_format=torch.channels_last)
        bufs[0].fill_(-1.0)
        gather_next(DEV, gu.desc, bufs, row_bytes, xforms)
        sel = perm[mb * B: mb * B + rows]
        got = bufs[0][:rows].cpu()
        assert torch.equal(got, ref[sel]), "frame transform differs from obs.float() / 255"
        assert torch.equal(bufs[1][:rows].cpu(), fields[1][sel.to(DEV)].cpu())
        assert torch.equal(bufs[2][:rows].cpu(), fields[2][sel.to(DEV)].cpu())
        if rows < B:
            assert (bufs[0][rows:] == -1.0).all()
    torch.cuda.synchronize()
    d = _lib.MinibatchDesc.from_buffer_copy(bytes(gu.desc.cpu().numpy()))
    assert d.mb == (n + B - 1) // B and d.arrivals == 0
    assert all(v == 0 for v in d.group_arrivals)  # the two-level arrival's group counters, re-armed


def test_gather_minibatch_transform_rejects_bad_shapes():
    import ctypes as C

    from rl_algo_impls_amd.graphs import GraphedUpdate

    fields = [torch.zeros(8, 5, 3, 3, dtype=torch.uint8, device=DEV)]  # 5 planes, hw = 9 (not % 4)
    gu = GraphedUpdate(DEV)
    gu.set_rollout(fields, 4, False)
    gu.start_epoch(None)
    out = torch.empty(4, 5, 3, 3, device=DEV)
    dst = (C.c_void_p * 1)(out.data_ptr())
    rb = (C.c_int64 * 1)(45)
    for x in (_lib.GatherXform(kind=1, channels=5, hw=9, divisor=255.0),
              _lib.GatherXform(kind=1, channels=4, hw=9, divisor=255.0), _lib.GatherXform(kind=7)):
        arr = (_lib.GatherXform * 1)(x)
        rc = _lib.lib().rai_gather_minibatch_x(gu.desc.data_ptr(), 1, C.cast(dst, C.c_void_p), C.cast(rb, C.c_void_p),
                                               C.cast(arr, C.c_void_p), 4, 1, _lib.stream_handle(DEV))
        assert rc in (-2, -3)


@pytest.mark.parametrize("rows,C", [(256 * 400, 32), (256 * 81, 64), (256 * 49, 64), (256, 512), (3, 8), (1000, 1024)])
def test_bias_relu_fwd_bwd_match_torch(rows, C):
    """rai_bias_relu_fwd / _bwd (csrc/se_block.hip) against torch fp32: relu(x + b) and
    threshold_backward bit for bit; the bias gradient (one fixed-order reduction) within fp32
    summation tolerance of torch's column sum, written or accumulated, and identical run to run."""
    g = torch.Generator(device="cpu").manual_seed(rows + C)
    x = torch.randn(rows, C, generator=g).to(DEV)
    b = torch.randn(C, generator=g).to(DEV)
    dy = torch.randn(rows, C, generator=g).to(DEV)
    x[0, :4] = float("nan")
    L, st = _lib.lib(), _lib.stream_handle(DEV)
    y = torch.empty_like(x)
    _lib.check(L.rai_bias_relu_fwd(x.data_ptr(), b.data_ptr(), rows, C, y.data_ptr(), st), "fwd")
    ref = torch.relu(x + b)
    assert torch.equal(y.isnan(), ref.isnan())
    assert torch.equal(torch.nan_to_num(y), torch.nan_to_num(ref))
    y = torch.nan_to_num(y)
    ws = torch.zeros(int(L.rai_bias_relu_workspace_bytes(C)), dtype=torch.uint8, device=DEV)
    dbs = []
    for acc in (0, 1, 0):
        dx = torch.empty_like(x)
        db = torch.full((C,), 0.5, device=DEV)
        _lib.check(L.rai_bias_relu_bwd(dy.data_ptr(), y.data_ptr(), rows, C, dx.data_ptr(), db.data_ptr(), acc,
                                       ws.data_ptr(), ws.numel(), st), "bwd")
        dx_ref = torch.ops.aten.threshold_backward(dy, y, 0.0)
        assert torch.equal(dx, dx_ref)
        db_ref = dx_ref.double().sum(0)
        np.testing.assert_allclose(db.double().cpu().numpy(), (db_ref + (0.5 if acc else 0.0)).cpu().numpy(),
                                   rtol=1e-5, atol=2e-6 * rows ** 0.5)
        dbs.append(db - (0.5 if acc else 0.0))
    assert torch.equal(dbs[0], dbs[2])  # deterministic
    assert bool((ws[-576:].view(torch.int32) == 0).all())  # the arrival counters, re-armed


@pytest.mark.parametrize("B,H,W,C", [(256, 7, 7, 64), (1024, 7, 7, 64), (5, 3, 3, 8), (700, 2, 5, 32), (2, 7, 7, 128)])
def test_bias_relu_nchw_pair_matches_torch_flatten(B, H, W, C):
    """rai_bias_relu_fwd_nchw / _bwd_nchw (csrc/se_block.hip, NatureCNN conv3 -> Flatten): the forward
    equals torch.flatten(relu(z + b), 1) of the channels_last conv output bit for bit; the backward
    takes the flattened gradient, returns threshold_backward in NHWC bit for bit and the bias gradient
    within fp32 summation tolerance (written, accumulated, deterministic, counters re-armed).
    B = 700 / 1024 > 512 workgroups: several samples per workgroup."""
    g = torch.Generator(device="cpu").manual_seed(B * 7 + C)
    z = torch.randn(B, C, H, W, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    b = torch.randn(C, generator=g).to(DEV)
    L, st = _lib.lib(), _lib.stream_handle(DEV)
    y = torch.empty(B, C * H * W, device=DEV)
    _lib.check(L.rai_bias_relu_fwd_nchw(z.data_ptr(), b.data_ptr(), B, H * W, C, y.data_ptr(), st), "fwd_nchw")
    ref = torch.flatten(torch.relu(z + b.view(1, C, 1, 1)), 1)
    assert torch.equal(y, ref)
    dy = torch.randn(B, C * H * W, generator=g).to(DEV)
    ws = torch.zeros(int(L.rai_bias_relu_workspace_bytes(C)), dtype=torch.uint8, device=DEV)
    dx_ref = torch.ops.aten.threshold_backward(dy, y, 0.0).view(B, C, H, W)
    dbs = []
    for acc in (0, 1, 0):
        dx = torch.empty(B, C, H, W, device=DEV, memory_format=torch.channels_last)
        db = torch.full((C,), 0.5, device=DEV)
        _lib.check(L.rai_bias_relu_bwd_nchw(dy.data_ptr(), y.data_ptr(), B, H * W, C, dx.data_ptr(), db.data_ptr(),
                                            acc, ws.data_ptr(), ws.numel(), st), "bwd_nchw")
        assert torch.equal(dx, dx_ref)
        db_ref = dx_ref.double().sum((0, 2, 3))
        np.testing.assert_allclose(db.double().cpu().numpy(), (db_ref + (0.5 if acc else 0.0)).cpu().numpy(),
                                   rtol=1e-5, atol=2e-6 * (B * H * W) ** 0.5)
        dbs.append(db - (0.5 if acc else 0.0))
    assert torch.equal(dbs[0], dbs[2])
    assert bool((ws[-576:].view(torch.int32) == 0).all())
    # the scalar form (RAI_BRT_VEC=0; also taken for misaligned dy / y) gives the same bits as the float4 form
    import os
    os.environ["RAI_BRT_VEC"] = "0"
    try:
        dx = torch.empty(B, C, H, W, device=DEV, memory_format=torch.channels_last)
        db = torch.empty(C, device=DEV)
        _lib.check(L.rai_bias_relu_bwd_nchw(dy.data_ptr(), y.data_ptr(), B, H * W, C, dx.data_ptr(), db.data_ptr(),
                                            0, ws.data_ptr(), ws.numel(), st), "bwd_nchw scalar")
    finally:
        del os.environ["RAI_BRT_VEC"]
    assert torch.equal(dx, dx_ref)
    assert torch.equal(db, dbs[0])
    # shapes the pair does not take: C not a multiple of 4, (C + 1) * HW over the LDS plane
    assert L.rai_bias_relu_fwd_nchw(z.data_ptr(), b.data_ptr(), B, H * W, 6, y.data_ptr(), st) == -2
    assert L.rai_bias_relu_fwd_nchw(z.data_ptr(), b.data_ptr(), 1, 4096, 64, y.data_ptr(), st) == -2
