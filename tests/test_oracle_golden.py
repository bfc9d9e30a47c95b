"""Pin the oracle (oracle/oracle.py, oracle/gae_ref.c) against golden vectors produced
by running the reference itself (tests/golden/make_golden.py).  CPU only."""
import json

import numpy as np
import pytest
import torch

import oracle


def test_gae_numpy_oracle_bit_exact(gae_cases):
    for c in gae_cases:
        adv = oracle.compute_advantages(c["rewards"], c["values"], c["episode_starts"],
                                        c["next_episode_starts"], c["next_values"], c["gamma"], c["lam"])
        assert adv.dtype == np.float32
        np.testing.assert_array_equal(adv, c["adv"], err_msg=f"case {c['idx']}")


def test_gae_c_oracle_bit_exact(gae_cases):
    for c in gae_cases:
        adv, ret = oracle.gae_c(c["rewards"], c["values"], c["episode_starts"],
                                c["next_episode_starts"], c["next_values"], c["gamma"], c["lam"])
        np.testing.assert_array_equal(adv, c["adv"], err_msg=f"case {c['idx']}")
        np.testing.assert_array_equal(ret, c["returns"], err_msg=f"case {c['idx']}")


def test_gae_pure_fp32_is_not_exact(gae_cases):
    """Documents why the exact mode exists: an fp32 carry differs from the reference."""
    diffs = []
    for c in gae_cases:
        if c["values"].ndim > 2 or isinstance(c["gamma"], np.ndarray) or c["rewards"].shape[0] < 32:
            continue
        r, v = c["rewards"], c["values"]
        nes = c["next_episode_starts"]
        last = np.zeros_like(v[0])
        out = np.zeros_like(v)
        g, l = np.float32(c["gamma"]), np.float32(c["lam"])
        for t in reversed(range(r.shape[0])):
            nn = (1 - (nes if t == r.shape[0] - 1 else c["episode_starts"][t + 1])).astype(np.float32)
            nv = c["next_values"] if t == r.shape[0] - 1 else v[t + 1]
            last = r[t] + g * nv * nn - v[t] + g * l * nn * last
            out[t] = last
        diffs.append(np.abs(out - c["adv"]).max())
    assert max(diffs) > 0


def _loss_case(z, index, name, i):
    p = f"{name}/b{i}_"
    return {k: z[p + k] for k in ("obs", "logprobs", "actions", "values", "advantages", "returns")}


def test_loss_oracle_matches_reference_grads(golden):
    """Reproduce the reference's first-step parameter gradients: torch CPU network
    forward -> oracle loss grads -> torch backward from (d_logp, d_entropy, d_v)."""
    import make_golden_networks as nets

    z = golden("ppo_steps.npz")
    index = json.loads(str(z["index"]))
    for name, meta in index.items():
        policy = nets.build(meta["policy"])
        nets.load_flat(policy, z[f"{name}/init"])
        hp = dict(meta["kw"], algo="ppo")
        acc = bool(hp.get("gradient_accumulation"))
        if acc:
            hp["grad_scale"] = 1.0 / meta["n"]
        for i in range(meta["n"] if acc else 1):
            b = _loss_case(z, index, name, i)
            logp, ent, v = policy(torch.from_numpy(b["obs"]), torch.from_numpy(b["actions"]))
            d_logp, d_ent, d_v, st = oracle.pg_loss_grads(
                logp.detach().numpy(), ent.detach().numpy(), v.detach().numpy(), b["logprobs"], b["values"],
                b["advantages"], b["returns"], hp)
            torch.autograd.backward([logp, ent, v], [torch.from_numpy(d_logp), torch.from_numpy(d_ent),
                                                     torch.from_numpy(d_v)])
            if i == 0:
                st0 = st
        st = st0
        g = torch.cat([p.grad.reshape(-1) for p in policy.parameters()]).numpy()
        ref = z[f"{name}/grads"]
        np.testing.assert_allclose(g, ref, rtol=2e-4, atol=2e-6, err_msg=name)
        stats = z[f"{name}/stats"][0]
        np.testing.assert_allclose(st["loss"], stats[0], rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(st["pi_loss"], stats[1], rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(st["entropy_loss"], stats[2], rtol=1e-5, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(st["approx_kl"], stats[3], rtol=1e-4, atol=1e-7, err_msg=name)


def test_clip_adam_oracle_matches_reference(golden):
    """Apply oracle clip+Adam to the reference's own first-step grads -> its params."""
    z = golden("ppo_steps.npz")
    index = json.loads(str(z["index"]))
    for name, meta in index.items():
        if meta["kw"].get("gradient_accumulation"):
            continue
        kw = meta["kw"]
        g, norm = oracle.clip_grad_norm(z[f"{name}/grads"], kw.get("max_grad_norm", 0.5))
        np.testing.assert_allclose(norm, z[f"{name}/norms"][0], rtol=1e-5, err_msg=name)
        p0 = z[f"{name}/init"]
        p1, m, v = oracle.adam_step(p0, g, np.zeros_like(p0), np.zeros_like(p0), 1, kw["learning_rate"])
        np.testing.assert_allclose(p1, z[f"{name}/params"][0], rtol=1e-5, atol=1e-7, err_msg=name)


def test_rmsprop_oracle_matches_reference(golden):
    z = golden("a2c_step.npz")
    g, _ = oracle.clip_grad_norm(z["grads"][0], 0.5)
    p1, sq = oracle.rmsprop_step(z["init"], g, np.zeros_like(z["init"]), 7e-4)
    np.testing.assert_allclose(p1, z["params"][0], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(sq, z["opt_state1"], rtol=1e-5, atol=1e-12)


def test_learn_epoch_gae_matches(golden):
    z = golden("learn_epoch_cartpole.npz")
    adv = oracle.compute_advantages(z["rewards"], z["values"], z["episode_starts"], z["next_episode_starts"],
                                    z["next_values"], 0.98, 0.8)
    np.testing.assert_array_equal(adv, z["advantages"])
    a2, r2 = oracle.gae_c(z["rewards"], z["values"], z["episode_starts"], z["next_episode_starts"],
                          z["next_values"], 0.98, 0.8)
    np.testing.assert_array_equal(a2, z["advantages"])
    np.testing.assert_array_equal(r2, z["returns"])


def test_feistel_permutation_spec_is_a_bijection():
    """The epoch-shuffle specification (oracle.feistel_permutation, which the device kernel must match):
    a bijection for every size including the non-power-of-two and tiny ones, key-dependent."""
    for n in (1, 2, 3, 5, 63, 64, 65, 1000, 131072, 131073):
        for key in (0, 7, 2**64 - 1):
            p = oracle.feistel_permutation(n, key)
            np.testing.assert_array_equal(np.sort(p), np.arange(n))
    assert (oracle.feistel_permutation(1000, 1) != oracle.feistel_permutation(1000, 2)).mean() > 0.9
