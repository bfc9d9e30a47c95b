"""Host side of the wide-MLP fused minibatch step (csrc/mlp_wide.hip).

For ActorCritics whose network is ConnectedTrio with a Flatten encoder and separate
[in -> H -> H -> out] actor / critic MLPs (H in {64, 128, 192, 256}; the HalfCheetah-class
policies of rl_algo_impls/hyperparams/ppo.yml), the minibatch forward + backward of
rl_algo_impls/ppo/ppo.py:290-377 runs as rai_mlp_wide_forward_loss (forward + head + loss) ->
rai_mlp_wide_backward (5 launches) instead of the PyTorch module forward and autograd.
The descriptor holds the parameter and flat-gradient pointers (stable for the trainer's life:
FlatParams never reallocates), so the launches can be captured into the replayed minibatch graph.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import torch

from . import _lib
from .policy import ActorCritic, CategoricalActorHead, GaussianActorHead


def _linears(seq) -> list:
    return [m for m in seq.modules() if isinstance(m, torch.nn.Linear)]


def wide_mlp_spec(pol) -> Optional[dict]:
    """The structure rai_mlp_wide_* implements, or None."""
    if not isinstance(pol, ActorCritic):
        return None
    net = pol.network
    if getattr(net, "_feature_extractor", None) is None or net._feature_extractor.kind != "flat":
        return None
    if net.activation_fn not in ("tanh", "relu"):
        return None
    if len(net.pi_hidden_sizes) != 2 or net.pi_hidden_sizes != net.v_hidden_sizes:
        return None
    H = net.pi_hidden_sizes[0]
    if net.pi_hidden_sizes[1] != H or H % 64 or not (64 <= H <= _lib.RAI_WIDE_MAX_H):
        return None
    if isinstance(net._pi, GaussianActorHead):
        head, pi_seq = 1, net._pi.mu_net
    elif isinstance(net._pi, CategoricalActorHead):
        head, pi_seq = 0, net._pi._fc
    else:
        return None
    in_dim, out = net._feature_extractor.out_dim, net._pi.act_dim
    if not (1 <= in_dim <= _lib.RAI_WIDE_MAX_IN and 1 <= out <= _lib.RAI_WIDE_MAX_OUT):
        return None
    pi_l, v_l = _linears(pi_seq), _linears(net._v)
    want = lambda o: [(H, in_dim), (H, H), (o, H)]
    if [tuple(l.weight.shape) for l in pi_l] != want(out) or [tuple(l.weight.shape) for l in v_l] != want(1):
        return None
    return dict(hidden=H, in_dim=in_dim, out=out, head=head, activation=0 if net.activation_fn == "tanh" else 1,
                pi=pi_l, v=v_l, log_std=getattr(net._pi, "log_std", None))


class WideStep:
    """Descriptor + workspace; forward()/backward() enqueue on the current stream (capturable)."""

    def __init__(self, policy, device: torch.device, accumulate: bool = False):
        spec = wide_mlp_spec(policy)
        if spec is None:
            raise ValueError("policy does not have the wide-MLP structure")
        self.spec = spec
        self.device = device
        d = _lib.MlpWideDesc()
        for n, layers in enumerate((spec["pi"], spec["v"])):
            ts = []
            for l in layers:
                ts += [l.weight, l.bias]
            for i, p in enumerate(ts):
                if p.grad is None or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("wide-MLP step needs the flat parameter/gradient views")
                d.w[n][i] = p.data_ptr()
                d.g[n][i] = p.grad.data_ptr()
        ls = spec["log_std"]
        if spec["head"] == 1:
            d.log_std, d.g_log_std = ls.data_ptr(), ls.grad.data_ptr()
        d.in_dim, d.hidden, d.out_pi = spec["in_dim"], spec["hidden"], spec["out"]
        d.head, d.activation, d.accumulate = spec["head"], spec["activation"], int(accumulate)
        self.desc = d
        self._ws: Dict[int, torch.Tensor] = {}
        self._params = [p for l in spec["pi"] + spec["v"] for p in (l.weight, l.bias)]
        if ls is not None:
            self._params.append(ls)
        self._ptrs = [(p.data_ptr(), p.grad.data_ptr()) for p in self._params]

    def check_pointers(self) -> None:
        assert [(p.data_ptr(), p.grad.data_ptr()) for p in self._params] == self._ptrs, \
            "parameter / gradient storage moved after the wide-MLP descriptor was built"

    def workspace(self, B: int) -> torch.Tensor:
        ws = self._ws.get(B)
        if ws is None:
            nbytes = int(_lib.lib().rai_mlp_wide_workspace_bytes(B, self.spec["hidden"]))
            ws = torch.empty(nbytes // 4, dtype=torch.float32, device=self.device)
            self._ws[B] = ws
        return ws

    def outputs(self, B: int):
        """Static (logp, entropy, v) buffers shaped like the PyTorch path's outputs."""
        ent_shape = (B, self.spec["out"]) if self.spec["head"] == 1 else (B,)
        z = lambda *s: torch.empty(s, dtype=torch.float32, device=self.device)
        return z(B), z(*ent_shape), z(B)

    def forward(self, obs: torch.Tensor, actions: torch.Tensor, logp, ent, v) -> None:
        B = int(obs.shape[0])
        if B > _lib.RAI_WIDE_MAX_B:
            raise ValueError(f"minibatch of {B} rows exceeds RAI_WIDE_MAX_B={_lib.RAI_WIDE_MAX_B}")
        obs = obs if obs.dtype == torch.float32 else obs.float()
        ws = self.workspace(B)
        rc = _lib.lib().rai_mlp_wide_forward(C.byref(self.desc), obs.contiguous().data_ptr(),
                                             actions.contiguous().data_ptr(), B, logp.data_ptr(), ent.data_ptr(),
                                             v.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                                             _lib.stream_handle(self.device))
        _lib.check(rc, "rai_mlp_wide_forward")

    def forward_loss(self, obs: torch.Tensor, actions: torch.Tensor, logp, ent, v, blocks, old_logp, old_values,
                     adv, ret):
        """forward() + rai_ppo_loss (K = 1) as rai_mlp_wide_forward_loss: the head and the loss share
        one launch.  Returns the loss gradients (d_logp, d_entropy, d_v) for backward()."""
        B = int(obs.shape[0])
        if B > _lib.RAI_WIDE_MAX_B:
            raise ValueError(f"minibatch of {B} rows exceeds RAI_WIDE_MAX_B={_lib.RAI_WIDE_MAX_B}")
        obs = obs if obs.dtype == torch.float32 else obs.float()
        ws = self.workspace(B)
        d_logp, d_ent, d_v = blocks.grad_buffers(logp, ent, v)
        p = lambda t: None if t is None else t.contiguous().data_ptr()
        rc = _lib.lib().rai_mlp_wide_forward_loss(
            C.byref(self.desc), obs.contiguous().data_ptr(), actions.contiguous().data_ptr(), B, logp.data_ptr(),
            ent.data_ptr(), v.data_ptr(), p(old_logp), p(old_values), p(adv), p(ret), blocks.hp.data_ptr(),
            blocks.state.data_ptr(), d_logp.data_ptr(), d_ent.data_ptr(), d_v.data_ptr(), blocks.stats.data_ptr(),
            int(blocks.stats.shape[0]), ws.data_ptr(), ws.numel() * 4, _lib.stream_handle(self.device))
        _lib.check(rc, "rai_mlp_wide_forward_loss")
        return d_logp, d_ent, d_v

    def backward(self, obs: torch.Tensor, actions: torch.Tensor, d_logp, d_ent, d_v) -> None:
        B = int(obs.shape[0])
        obs = obs if obs.dtype == torch.float32 else obs.float()
        ws = self.workspace(B)
        rc = _lib.lib().rai_mlp_wide_backward(C.byref(self.desc), obs.contiguous().data_ptr(),
                                              actions.contiguous().data_ptr(), B, d_logp.data_ptr(),
                                              d_ent.data_ptr(), d_v.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                                              _lib.stream_handle(self.device))
        _lib.check(rc, "rai_mlp_wide_backward")


class WideRolloutForward:
    """Rollout forward of a wide-MLP policy (rai_mlp_wide_dist_params): the actor's distribution
    parameters (Gaussian mean / Categorical logits) and the critic value for a fixed batch of B
    observations, into static buffers (capturable into the rollout's step graph).  Weight pointers
    only; the descriptor is rebuilt if a parameter's storage moved (FlatParams re-views them once,
    when the trainer is built)."""

    def __init__(self, policy, device: torch.device, B: int):
        spec = wide_mlp_spec(policy)
        if spec is None:
            raise ValueError("policy does not have the wide-MLP structure")
        if not 1 <= B <= _lib.RAI_WIDE_MAX_B:
            raise ValueError(f"rollout batch {B} outside 1..{_lib.RAI_WIDE_MAX_B}")
        self.spec, self.device, self.B = spec, device, B
        self._params = [p for l in spec["pi"] + spec["v"] for p in (l.weight, l.bias)]
        self._key = None
        nbytes = int(_lib.lib().rai_mlp_wide_workspace_bytes(B, spec["hidden"]))
        self.ws = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
        self.params_out = torch.empty((B, spec["out"]), dtype=torch.float32, device=device)
        self.v_out = torch.empty((B,), dtype=torch.float32, device=device)

    def _desc(self):
        key = tuple(p.data_ptr() for p in self._params)
        if key != self._key:
            for p in self._params:
                assert p.is_contiguous() and p.dtype == torch.float32
            d = _lib.MlpWideDesc()
            for n in range(2):
                for i in range(6):
                    d.w[n][i] = self._params[6 * n + i].data_ptr()
            d.in_dim, d.hidden, d.out_pi = self.spec["in_dim"], self.spec["hidden"], self.spec["out"]
            d.head, d.activation = self.spec["head"], self.spec["activation"]
            if self.spec["head"] == 1:
                d.log_std = self.spec["log_std"].data_ptr()
            self.desc, self._key = d, key
        return self.desc

    def __call__(self, obs: torch.Tensor):
        obs = obs if obs.dtype == torch.float32 else obs.float()
        rc = _lib.lib().rai_mlp_wide_dist_params(C.byref(self._desc()), obs.contiguous().data_ptr(), self.B,
                                                 self.params_out.data_ptr(), self.v_out.data_ptr(),
                                                 self.ws.data_ptr(), self.ws.numel() * 4,
                                                 _lib.stream_handle(self.device))
        _lib.check(rc, "rai_mlp_wide_dist_params")
        return self.params_out, self.v_out
