"""rai_categorical_critic_heads_fwd / _bwd (csrc/heads.hip, cnn_ops.CategoricalCriticHeads) against
the modules' own path: CategoricalActorHead Linear(D, A) + torch.distributions.Categorical
(rl_algo_impls/shared/actor/categorical.py:57-87) and CriticHead Linear(D, 1)
(rl_algo_impls/shared/policy/critic.py:11-41): log-prob, entropy, value and every gradient (the input,
both weights and biases), returned to autograd or accumulated in place into the flat gradient views."""
import numpy as np
import pytest
import torch

from rl_algo_impls_amd import cnn_ops
from rl_algo_impls_amd.policy import CategoricalActorHead, CriticHead

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("B,D,A", [(256, 512, 6), (37, 512, 2), (64, 96, 12), (1, 512, 3)])
def test_heads_match_module_path(B, D, A):
    torch.manual_seed(B + A)
    pi = CategoricalActorHead(A, D, (), torch.nn.ReLU).to(DEV)
    v = CriticHead(D, (), torch.nn.ReLU).to(DEV)
    with torch.no_grad():  # non-trivial logits (the reference's head init is gain 0.01)
        pi._fc[0].weight.mul_(30.0)
    enc = torch.randn(B, D, device=DEV)
    act = torch.randint(0, A, (B,), device=DEV)
    up = [torch.randn(B, device=DEV) for _ in range(3)]
    params = [pi._fc[0].weight, pi._fc[0].bias, v._fc[0][0].weight, v._fc[0][0].bias]

    # reference: the modules with torch.distributions.Categorical
    e1 = enc.clone().requires_grad_(True)
    d = torch.distributions.Categorical(logits=pi._fc(e1))
    ref = (d.log_prob(act), d.entropy(), v(e1))
    gref = torch.autograd.grad(ref, [e1] + params, up)

    e2 = enc.clone().requires_grad_(True)
    out = cnn_ops.CategoricalCriticHeads.apply(e2, params[0], params[1], params[2], params[3], act)
    for o, r in zip(out, ref):
        np.testing.assert_allclose(o.detach().cpu().numpy(), r.detach().cpu().numpy(), rtol=2e-5, atol=2e-5)
    g = torch.autograd.grad(out, [e2] + params, up)
    for name, a, b in zip(("enc", "wpi", "bpi", "wv", "bv"), g, gref):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=2e-4, atol=2e-5 * float(b.abs().max()),
                                   err_msg=name)

    # in place: gradients added to existing .grad views (the trainer's flat buffer)
    for p in params:
        p.grad = torch.full_like(p, 0.25)
    e3 = enc.clone().requires_grad_(True)
    with cnn_ops.direct_grads():
        out = cnn_ops.CategoricalCriticHeads.apply(e3, params[0], params[1], params[2], params[3], act)
    torch.autograd.backward(out, up)
    np.testing.assert_allclose(e3.grad.cpu().numpy(), gref[0].cpu().numpy(), rtol=2e-4,
                               atol=2e-5 * float(gref[0].abs().max()))
    for p, b in zip(params, gref[1:]):
        np.testing.assert_allclose((p.grad - 0.25).cpu().numpy(), b.reshape(p.shape).cpu().numpy(), rtol=2e-4,
                                   atol=2e-5 * float(b.abs().max()) + 1e-6)
