"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every
symbol include/rai_amd.h declares; the policy module tree is state_dict-compatible
with the reference and initialises bit-identically from the same seed."""
import json
import re

import numpy as np
import pytest
import torch

from conftest import ROOT

from rl_algo_impls_amd import _lib
from rl_algo_impls_amd.policy import ActorCritic
import make_golden_networks as nets


def declared_symbols():
    hdr = (ROOT / "include" / "rai_amd.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(rai_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    assert "rai_gae" in syms and "rai_ppo_loss" in syms and "rai_clip_optim_step" in syms
    assert set(syms) == set(_lib.EXPORTED), (set(syms) ^ set(_lib.EXPORTED))


def test_library_loads_and_exports_all_symbols():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert L.rai_abi_version() == 1
    assert L.rai_strerror(-2) == b"invalid shape argument"
    # only the HIP runtime torch mapped is present (SONAME-deduplicated)
    assert len(_lib.hip_runtimes_mapped()) <= 1


def test_argument_errors_are_reported_without_a_device():
    L = _lib.lib()
    import ctypes as C
    g = (C.c_double * 1)(0.99)
    assert L.rai_gae(None, None, None, None, None, 4, 4, 99, g, g, 0, 0, None, None, None) == -4
    assert L.rai_gae(None, None, None, None, None, 4, 4, 1, g, g, 0, 7, None, None, None) == -3
    assert L.rai_gae(None, None, None, None, None, 4, 4, 1, g, g, 0, 0, None, None, None) == -1
    assert L.rai_gae(None, None, None, None, None, 0, 4, 1, g, g, 0, 0, None, None, None) == 0
    assert L.rai_ppo_loss(None, None, 1, *([None] * 5), 0, 1, *([None] * 6), 0, None, 0, None) == -2
    with pytest.raises(RuntimeError, match="invalid shape"):
        _lib.check(-2, "x")


@pytest.mark.parametrize("name", ["cartpole", "halfcheetah", "pong"])
def test_policy_state_dict_keys_and_init_match_reference(name, golden):
    meta = json.loads((ROOT / "tests" / "golden" / "policy_init.json").read_text())[name]
    env = {"cartpole": nets.cartpole_env, "halfcheetah": nets.halfcheetah_env, "pong": nets.pong_env}[name]()
    torch.manual_seed(1)
    policy = ActorCritic(env, **meta["kwargs"])
    sd = policy.state_dict()
    assert [k for k, *_ in meta["keys"]] == list(sd.keys())
    for k, shape, s, s2, head in meta["keys"]:
        t = sd[k]
        assert list(t.shape) == shape, k
        np.testing.assert_allclose(float(t.double().sum()), s, rtol=1e-9, atol=1e-9, err_msg=k)
        np.testing.assert_allclose(float((t.double() ** 2).sum()), s2, rtol=1e-9, err_msg=k)
        np.testing.assert_array_equal(t.reshape(-1)[:4].numpy(), np.array(head, np.float32), err_msg=k)
    z = golden("policy_forward.npz")
    with torch.no_grad():
        lp, ent, v = policy(torch.from_numpy(z[f"{name}_obs"]), torch.from_numpy(z[f"{name}_act"]))
    np.testing.assert_allclose(lp.numpy(), z[f"{name}_logp"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ent.numpy(), z[f"{name}_entropy"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(v.numpy(), z[f"{name}_v"], rtol=1e-5, atol=1e-6)


def test_registries_use_reference_names():
    from rl_algo_impls_amd import registry

    # the reference's on-policy algorithms over the rollout hot path (running_utils.py:38-55)
    assert set(registry.ALGOS) == {"ppo", "a2c", "acbc"}
    for k in registry.ALGOS:
        assert registry.DEFAULT_ROLLOUT_GENERATORS[k].__name__ == "SyncStepRolloutGenerator"
    assert registry.POLICIES["ppo"] is ActorCritic


def test_clamp_actions_reference_vectors():
    """The reference's only unit test (tests/shared/policy/test_actor_critic.py:8-17)."""
    from rl_algo_impls_amd.envs import Box
    from rl_algo_impls_amd.policy import clamp_actions

    space = Box(low=-1, high=1, shape=(1,))
    np.testing.assert_array_equal(clamp_actions(np.array([-1.5, 0, 1.5]), space, False), np.array([-1, 0, 1]))
    space = Box(low=-3, high=2, shape=(1,))
    np.testing.assert_array_equal(clamp_actions(np.array([-1, 0, 1]), space, True), np.array([-3, -0.5, 2]))


def test_bias_relu_workspaces_are_freed_with_their_layer():
    """cnn_ops keys the bias + ReLU backward workspaces weakly on the layer module: one workspace per
    (layer, channels, device), reused on every call, dropped when the layer is collected (so a later
    layer can never alias a dead layer's workspace, as an id() key could)."""
    import gc

    from rl_algo_impls_amd import cnn_ops

    ws = cnn_ops._Workspaces()
    a, b = torch.nn.Linear(4, 8), torch.nn.Linear(4, 8)
    wa = ws.get(a, 8, torch.device("cpu"))
    assert ws.get(a, 8, torch.device("cpu")) is wa
    assert ws.get(b, 8, torch.device("cpu")) is not wa
    assert int(wa.numel()) == int(_lib.lib().rai_bias_relu_workspace_bytes(8)) and not wa.any()
    del a
    gc.collect()
    assert len(ws._ws) == 1


def test_ctypes_signatures_match_header_arity():
    """Every ctypes binding (_lib._SIGNATURES) passes exactly as many arguments as the C declaration
    in include/rai_amd.h takes (a short list silently shifts every later argument)."""
    hdr = (ROOT / "include" / "rai_amd.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    decls = {m.group(1): m.group(2) for m in re.finditer(r"\b(rai_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", hdr, flags=re.S)}
    for name, (_, args) in _lib._SIGNATURES.items():
        params = decls[name].strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert len(args) == n, (name, len(args), n)


def test_error_code_constants_match_header():
    """_lib's RAI_E_* constants are the header's enum values (cnn_ops' MIOpen fallback keys on
    RAI_E_UNSUPPORTED: a renumbered enum must fail here, not turn the fallback into a hard error)."""
    hdr = (ROOT / "include" / "rai_amd.h").read_text()
    codes = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(RAI_E_[A-Z_]+)\s*=\s*(-?\d+)", hdr)}
    assert codes and "RAI_E_UNSUPPORTED" in codes
    for name, v in codes.items():
        assert getattr(_lib, name) == v, name
