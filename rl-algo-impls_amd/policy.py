"""ActorCritic policy with the reference's module tree (state_dict-compatible).

Mirrors rl_algo_impls/shared/policy/actor_critic.py:110-340 for the configurations
on the hot path (share_features_extractor=True -> ConnectedTrio network,
rl_algo_impls/shared/policy/actor_critic_network/connected_trio.py:17-116):

  network._feature_extractor   Encoder: Flatten for 1-D Box obs
                               (shared/encoder/encoder.py:51-58) or NatureCnn for
                               3-D Box obs (shared/encoder/nature_cnn.py:10-53,
                               shared/encoder/cnn.py:24-72; /range_size prescale)
  network._pi                  CategoricalActorHead._fc (shared/actor/categorical.py:57-87)
                               or GaussianActorHead.{log_std, mu_net} (shared/actor/gaussian.py:19-61)
  network._v                   CriticHead._fc = Sequential(mlp) (shared/policy/critic.py:11-41)

Modules are constructed (and layer_init'ed, shared/module/utils.py:7-45) in the
reference's order, so the same torch seed yields bit-identical initial weights,
and model.pth checkpoints load in both directions.

The networks' forward/backward run on PyTorch-ROCm (rocBLAS/hipBLASLt GEMMs,
MIOpen convolutions -> MFMA on gfx950).  Distribution math is written out
(no torch.distributions validation, which forces host syncs) with the exact
formulas of torch.distributions.Categorical / Normal.
"""
from __future__ import annotations

import math
import os
from typing import NamedTuple, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from .envs import is_box, is_discrete

ACTIVATION = {"tanh": nn.Tanh, "relu": nn.ReLU, "identity": nn.Identity, "sigmoid": nn.Sigmoid}
MODEL_FILENAME = "model.pth"
NORMALIZE_OBSERVATION_FILENAME = "norm_obs.npz"
NORMALIZE_REWARD_FILENAME = "norm_reward.npz"
F32_MIN = torch.finfo(torch.float32).min
# NatureCNN activations NHWC on the GPU (RAI_CHANNELS_LAST=0: NCHW).  Pong A/B with the fused
# minibatch gather and Categorical head: 1.611 vs 1.667 s per update (MIOpen's NHWC solvers, no
# layout transposes, contiguous bias-gradient reductions).
_CHANNELS_LAST = os.environ.get("RAI_CHANNELS_LAST", "1") == "1"
# NatureCNN conv / Linear -> ReLU as bias-free contractions plus one-pass bias + ReLU epilogues
# (cnn_ops.py), and the uint8 -> float / range_size prescale fused into the minibatch gather
# (RAI_CNN_FUSED=0: the modules' own bias / ReLU kernels and the torch prescale)
_FUSED_EPILOGUES = os.environ.get("RAI_CNN_FUSED", "1") == "1"


class Step(NamedTuple):  # actor_critic.py:42-46
    a: np.ndarray
    v: np.ndarray
    logp_a: np.ndarray
    clamped_a: np.ndarray


class ACForward(NamedTuple):  # actor_critic.py:49-53
    logp_a: torch.Tensor
    entropy: torch.Tensor
    v: torch.Tensor


def layer_init(layer: nn.Module, init_layers_orthogonal: bool, std: float = np.sqrt(2)) -> nn.Module:
    if not init_layers_orthogonal:
        return layer
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, 0.0)
    return layer


def mlp(layer_sizes: Sequence[int], activation, output_activation=nn.Identity,
        init_layers_orthogonal: bool = False, final_layer_gain: float = np.sqrt(2),
        hidden_layer_gain: float = np.sqrt(2)) -> nn.Sequential:
    layers = []
    for i in range(len(layer_sizes) - 2):
        layers.append(layer_init(nn.Linear(layer_sizes[i], layer_sizes[i + 1]), init_layers_orthogonal,
                                 std=hidden_layer_gain))
        layers.append(activation())
    layers.append(layer_init(nn.Linear(layer_sizes[-2], layer_sizes[-1]), init_layers_orthogonal,
                             std=final_layer_gain))
    layers.append(output_activation())
    return nn.Sequential(*layers)


def default_hidden_sizes(obs_space) -> Sequence[int]:  # actor_critic_network/network.py:73-85
    if is_box(obs_space):
        if len(obs_space.shape) == 3:
            return []
        if len(obs_space.shape) == 1:
            return [64, 64]
        raise ValueError(f"Unsupported observation space: {obs_space}")
    if is_discrete(obs_space):
        return [64]
    raise ValueError(f"Unsupported observation space: {obs_space}")


class NatureCnnEncoder(nn.Module):
    """shared/encoder/nature_cnn.py + cnn.py FlattenedCnnEncoder (keys cnn.{0,2,4}, fc.1)."""

    def __init__(self, obs_space, activation, cnn_init_layers_orthogonal: Optional[bool],
                 linear_init_layers_orthogonal: bool, cnn_flatten_dim: int):
        super().__init__()
        if cnn_init_layers_orthogonal is None:
            cnn_init_layers_orthogonal = True
        self.range_size = float(np.max(obs_space.high) - np.min(obs_space.low))
        in_channels = obs_space.shape[0]
        self.cnn = nn.Sequential(
            layer_init(nn.Conv2d(in_channels, 32, kernel_size=8, stride=4), cnn_init_layers_orthogonal),
            activation(),
            layer_init(nn.Conv2d(32, 64, kernel_size=4, stride=2), cnn_init_layers_orthogonal),
            activation(),
            layer_init(nn.Conv2d(64, 64, kernel_size=3, stride=1), cnn_init_layers_orthogonal),
            activation(),
        )
        with torch.no_grad():
            dummy = torch.zeros((1,) + tuple(obs_space.shape))
            n_flat = torch.flatten(self.cnn(dummy), start_dim=1).shape[1]
        self.fc = nn.Sequential(
            nn.Flatten(),
            layer_init(nn.Linear(n_flat, cnn_flatten_dim), linear_init_layers_orthogonal),
            activation(),
        )
        self.out_dim = cnn_flatten_dim
        self._relu = activation is nn.ReLU
        # the divisor as a device scalar (non-persistent: not in the state_dict), see forward()
        self.register_buffer("_range", torch.tensor(self.range_size, dtype=torch.float32), persistent=False)

    def _u8_input(self, obs: torch.Tensor) -> bool:
        """conv1 reads the uint8 frames itself (cnn_ops RAI_CONV_U8): 4 channels, the fused ReLU path."""
        from . import cnn_ops

        return (cnn_ops._CONV_U8 and cnn_ops._CONV_MFMA and _CHANNELS_LAST and _FUSED_EPILOGUES and self._relu
                and obs.is_cuda and obs.dtype == torch.uint8 and int(obs.shape[-3]) == 4)

    def obs_transform(self, obs: torch.Tensor):
        """The rai_gather_xform that turns a gathered uint8 frame row into this encoder's input
        (obs.float() / range_size, channels_last; or, where conv1 reads uint8 itself, the uint8 frames
        in channels_last), or None when the fused path does not apply."""
        from . import _lib

        C, H, W = (int(d) for d in obs.shape[-3:])
        if not (_CHANNELS_LAST and _FUSED_EPILOGUES and obs.is_cuda and obs.dtype == torch.uint8 and C <= 4
                and (H * W) % 4 == 0):
            return None
        kind = _lib.RAI_XFORM_U8_CHW_TO_U8_HWC if self._u8_input(obs) else _lib.RAI_XFORM_U8_CHW_TO_F32_HWC
        return _lib.GatherXform(kind=kind, channels=C, hw=H * W, divisor=self.range_size)

    def forward(self, obs: torch.Tensor, prepared: bool = False) -> torch.Tensor:
        """prepared: obs is already the encoder's input in channels_last (the minibatch gather's output:
        obs.float() / range_size, or the uint8 frames when conv1 applies the prescale itself)."""
        if obs.dim() == 3:
            obs = obs.unsqueeze(0)
        if prepared:
            x = obs
        elif self._u8_input(obs):
            x = obs.contiguous(memory_format=torch.channels_last)  # uint8: conv1 divides in-kernel
        elif obs.is_cuda:
            # IEEE division, as the reference's CPU path and the fused gather: torch divides a CUDA
            # tensor by a Python scalar as a multiply by the rounded reciprocal
            x = obs.float() / self._range
        else:
            x = obs.float() / self.range_size
        if x.dtype == torch.uint8:  # prepared uint8 frames: only the fused path takes them
            return self._forward_fused(x.contiguous(memory_format=torch.channels_last))
        if _CHANNELS_LAST and x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
            if _FUSED_EPILOGUES and self._relu:
                return self._forward_fused(x)
        return self.fc(self.cnn(x))

    def _forward_fused(self, x: torch.Tensor) -> torch.Tensor:
        """Bias-free MIOpen convolutions / hipBLASLt GEMM with the bias + ReLU epilogues of
        cnn_ops (same modules, same parameters, same state_dict)."""
        return self.fc_relu(self._trunk_fused(x))

    def _trunk_fused(self, x: torch.Tensor) -> torch.Tensor:
        """The three conv -> ReLU layers; conv3's epilogue writes the flattened (NCHW-order) fc input
        itself: no layout copies."""
        from .cnn_ops import conv_relu

        x = conv_relu(self.cnn[0], x, x_div=self.range_size if x.dtype == torch.uint8 else None)
        x = conv_relu(self.cnn[2], x)
        return conv_relu(self.cnn[4], x, flatten=True)

    def fc_relu(self, flat: torch.Tensor) -> torch.Tensor:
        from .cnn_ops import linear_relu

        return linear_relu(self.fc[1], flat)

    def forward_trunk(self, obs: torch.Tensor, prepared: bool = False):
        """The flattened conv3 output (the fc layer's input) where the fused GPU path applies, else None
        (the caller then runs forward())."""
        if obs.dim() == 3:
            obs = obs.unsqueeze(0)
        if not (obs.is_cuda and _CHANNELS_LAST and _FUSED_EPILOGUES and self._relu):
            return None
        if prepared:
            x = obs
        elif self._u8_input(obs):
            x = obs
        else:
            x = obs.float() / self._range
        return self._trunk_fused(x.contiguous(memory_format=torch.channels_last))


class Encoder(nn.Module):  # shared/encoder/encoder.py:25-73
    def __init__(self, obs_space, activation, init_layers_orthogonal: bool = False,
                 cnn_flatten_dim: int = 512, cnn_style: str = "nature",
                 cnn_layers_init_orthogonal: Optional[bool] = None):
        super().__init__()
        if is_box(obs_space) and len(obs_space.shape) == 3:
            if cnn_style != "nature":
                raise NotImplementedError(f"cnn_style={cnn_style} is outside the hot-path scope")
            self.kind = "cnn"
            self.feature_extractor = NatureCnnEncoder(obs_space, activation, cnn_layers_init_orthogonal,
                                                      init_layers_orthogonal, cnn_flatten_dim)
            self.out_dim = self.feature_extractor.out_dim
        elif is_box(obs_space) and len(obs_space.shape) == 1:
            self.kind = "flat"
            self.feature_extractor = nn.Flatten()
            self.out_dim = int(np.prod(obs_space.shape))
        elif is_discrete(obs_space):
            self.kind = "onehot"
            self.n = obs_space.n
            self.feature_extractor = nn.Flatten()
            self.out_dim = obs_space.n
        else:
            raise NotImplementedError(f"Unsupported observation space: {obs_space}")

    def forward(self, obs: torch.Tensor, prepared: bool = False) -> torch.Tensor:
        if self.kind == "cnn":
            return self.feature_extractor(obs, prepared)
        if self.kind == "flat":
            if obs.dim() == 1:
                obs = obs.unsqueeze(0)
            obs = obs.float()
        elif self.kind == "onehot":
            obs = nn.functional.one_hot(obs, self.n).float()
        return self.feature_extractor(obs)


class CategoricalActorHead(nn.Module):
    def __init__(self, act_dim, in_dim, hidden_sizes=(32,), activation=nn.Tanh, init_layers_orthogonal=True):
        super().__init__()
        self.act_dim = act_dim
        self._fc = mlp((in_dim,) + tuple(hidden_sizes) + (act_dim,), activation,
                       init_layers_orthogonal=init_layers_orthogonal, final_layer_gain=0.01)

    def params(self, x):
        return self._fc(x)

    @staticmethod
    def logp_entropy(logits, actions, action_masks=None):
        """torch.distributions.Categorical (+ MaskedCategorical, categorical.py:12-54).  On the GPU:
        the fused GridNet operator with one cell and one plane (rai_gridnet_logp_entropy forward,
        rai_gridnet_backward backward: two launches instead of ~16 small torch kernels)."""
        if logits.is_cuda and logits.dtype == torch.float32 and logits.dim() == 2 and logits.shape[-1] <= 256:
            from .gridnet import GridnetLogpEntropy, categorical_spec

            B, A = int(logits.shape[0]), int(logits.shape[1])
            masks = (action_masks.reshape(B, 1, A) if action_masks is not None
                     else torch.ones((B, 1, A), dtype=torch.bool, device=logits.device))
            return GridnetLogpEntropy.apply(logits.reshape(B, 1, A), masks,
                                            actions.long().reshape(B, 1, 1), categorical_spec(A))
        if action_masks is not None:
            logits = torch.where(action_masks, logits, F32_MIN)
        norm = logits - logits.logsumexp(dim=-1, keepdim=True)
        probs = torch.softmax(norm, dim=-1)
        logp = norm.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        if action_masks is None:
            ent = -(torch.clamp(norm, min=F32_MIN) * probs).sum(-1)
        else:
            ent = -torch.where(action_masks, norm * probs, torch.zeros((), device=norm.device)).sum(-1)
        return logp, ent

    def mode(self, logits, action_masks=None):
        if action_masks is not None:
            logits = torch.where(action_masks, logits, F32_MIN)
        return logits.argmax(-1)

    @property
    def action_shape(self):
        return ()


class GaussianActorHead(nn.Module):
    def __init__(self, act_dim, in_dim, hidden_sizes=(32,), activation=nn.Tanh, init_layers_orthogonal=True,
                 log_std_init=-0.5):
        super().__init__()
        self.act_dim = act_dim
        self.mu_net = mlp((in_dim,) + tuple(hidden_sizes) + (act_dim,), activation,
                          init_layers_orthogonal=init_layers_orthogonal, final_layer_gain=0.01)
        self.log_std = nn.Parameter(torch.ones(act_dim, dtype=torch.float32) * log_std_init)

    def params(self, x):
        return self.mu_net(x)

    def logp_entropy(self, mu, actions, action_masks=None):
        """GaussianDistribution (gaussian.py:11-16): log_prob summed over action dims,
        entropy per dimension (B, act_dim) — the loss averages it (ppo.py:351)."""
        assert action_masks is None, "GaussianActorHead does not support action_masks"
        scale = torch.exp(self.log_std)
        var = scale ** 2
        log_scale = scale.log()
        lp = -((actions - mu) ** 2) / (2 * var) - log_scale - math.log(math.sqrt(2 * math.pi))
        ent = (0.5 + 0.5 * math.log(2 * math.pi) + torch.log(scale)).expand_as(mu)
        return lp.sum(dim=-1), ent

    def mode(self, mu, action_masks=None):
        return mu

    @property
    def action_shape(self):
        return (self.act_dim,)


class CriticHead(nn.Module):
    def __init__(self, in_dim, hidden_sizes=(), activation=nn.Tanh, init_layers_orthogonal=True):
        super().__init__()
        self._fc = nn.Sequential(mlp((in_dim,) + tuple(hidden_sizes) + (1,), activation,
                                     init_layers_orthogonal=init_layers_orthogonal, final_layer_gain=1.0))

    def forward(self, x):
        return self._fc(x).squeeze(-1)


class ConnectedTrioNetwork(nn.Module):
    def __init__(self, observation_space, action_space, pi_hidden_sizes=None, v_hidden_sizes=None,
                 init_layers_orthogonal=True, activation_fn="tanh", log_std_init=-0.5,
                 cnn_flatten_dim=512, cnn_style="nature", cnn_layers_init_orthogonal=None):
        super().__init__()
        pi_hidden_sizes = pi_hidden_sizes if pi_hidden_sizes is not None else default_hidden_sizes(observation_space)
        v_hidden_sizes = v_hidden_sizes if v_hidden_sizes is not None else default_hidden_sizes(observation_space)
        activation = ACTIVATION[activation_fn]
        self.activation_fn = activation_fn
        self._feature_extractor = Encoder(observation_space, activation, init_layers_orthogonal,
                                          cnn_flatten_dim, cnn_style, cnn_layers_init_orthogonal)
        in_dim = self._feature_extractor.out_dim
        if is_discrete(action_space):
            self._pi = CategoricalActorHead(action_space.n, in_dim, tuple(pi_hidden_sizes), activation,
                                            init_layers_orthogonal)
        elif is_box(action_space):
            self._pi = GaussianActorHead(action_space.shape[0], in_dim, tuple(pi_hidden_sizes), activation,
                                         init_layers_orthogonal, log_std_init)
        else:
            raise NotImplementedError(f"action space {action_space} is outside the hot-path scope")
        self._v = CriticHead(in_dim, v_hidden_sizes, activation, init_layers_orthogonal)
        self.pi_hidden_sizes = tuple(pi_hidden_sizes)
        self.v_hidden_sizes = tuple(v_hidden_sizes)

    def forward(self, obs, action, action_masks=None, obs_prepared: bool = False):
        if _FUSED_EPILOGUES and self._feature_extractor.kind == "cnn":
            fe = self._feature_extractor.feature_extractor
            trunk = fe.forward_trunk(obs, obs_prepared)  # conv3's flattened output, or None
            if trunk is not None:
                from .cnn_ops import fc_relu_heads, fc_relu_heads_fusable

                # the fc -> ReLU and both heads as one node: the ReLU backward folded into the heads' backward
                if fc_relu_heads_fusable(self, fe.fc[1], trunk, action_masks):
                    return fc_relu_heads(self, fe.fc[1], trunk, action)
                enc = fe.fc_relu(trunk)
            else:
                enc = self._feature_extractor(obs, obs_prepared)
        else:
            enc = self._feature_extractor(obs, obs_prepared)
        if _FUSED_EPILOGUES and self._feature_extractor.kind == "cnn":
            from .cnn_ops import categorical_critic_heads, heads_fusable

            if heads_fusable(self, enc, action_masks):  # one launch forward, two backward (csrc/heads.hip)
                return categorical_critic_heads(self, enc, action)
        logp, ent = self._pi.logp_entropy(self._pi.params(enc), action, action_masks)
        return logp, ent, self._v(enc)

    def dist_params_and_value(self, obs):
        enc = self._feature_extractor(obs)
        return self._pi.params(enc), self._v(enc)

    def value(self, obs):
        return self._v(self._feature_extractor(obs))


class ActorCritic(nn.Module):
    """Same constructor kwargs as the reference ActorCritic for the hot-path
    configurations; unsupported styles raise NotImplementedError loudly."""

    def __init__(self, env, pi_hidden_sizes=None, v_hidden_sizes=None, init_layers_orthogonal=True,
                 activation_fn="tanh", log_std_init=-0.5, use_sde=False, full_std=True, squash_output=False,
                 share_features_extractor=True, cnn_flatten_dim=512, cnn_style="nature",
                 cnn_layers_init_orthogonal=None, actor_head_style="single", critic_channels=64,
                 num_additional_critics=0, additional_critic_activation_functions=None, channels_per_level=None,
                 strides_per_level=None, deconv_strides_per_level=None, encoder_residual_blocks_per_level=None,
                 decoder_residual_blocks_per_level=None, increment_kernel_size_on_down_conv=False,
                 output_activation_fn="identity", subaction_mask=None, critic_shares_backbone=None,
                 save_critic_separate=None, shared_critic_head=None, normalization=None, **kwargs):
        super().__init__()
        if use_sde or squash_output:
            raise NotImplementedError("gSDE / squash_output are outside the hot-path scope")
        if not share_features_extractor:
            raise NotImplementedError("SeparateActorCriticNetwork is outside the hot-path scope")
        if actor_head_style not in ("single", "squeeze_unet"):
            raise NotImplementedError(f"actor_head_style={actor_head_style} is outside the hot-path scope")
        self.env = env
        self.action_space = env.single_action_space
        self.observation_space = env.single_observation_space
        self.squash_output = squash_output
        self.gridnet = actor_head_style == "squeeze_unet"
        if self.gridnet:  # actor_critic.py:200-229 (MicroRTS, config C5)
            from .backbone import SqueezeUnetActorCriticNetwork

            plane = getattr(env, "action_plane_space", None)
            assert plane is not None, "squeeze_unet needs the env's action_plane_space"
            self.network = SqueezeUnetActorCriticNetwork(
                env.single_observation_space, env.single_action_space, plane,
                init_layers_orthogonal=init_layers_orthogonal, cnn_layers_init_orthogonal=cnn_layers_init_orthogonal,
                num_additional_critics=num_additional_critics,
                additional_critic_activation_functions=additional_critic_activation_functions,
                critic_channels=critic_channels, channels_per_level=channels_per_level,
                strides_per_level=strides_per_level, deconv_strides_per_level=deconv_strides_per_level,
                encoder_residual_blocks_per_level=encoder_residual_blocks_per_level,
                decoder_residual_blocks_per_level=decoder_residual_blocks_per_level,
                increment_kernel_size_on_down_conv=increment_kernel_size_on_down_conv,
                output_activation_fn=output_activation_fn, subaction_mask=subaction_mask,
                critic_shares_backbone=critic_shares_backbone if critic_shares_backbone is not None else True,
                save_critic_separate=save_critic_separate if save_critic_separate is not None else False,
                shared_critic_head=shared_critic_head if shared_critic_head is not None else False,
                normalization=normalization)
        else:
            self.network = ConnectedTrioNetwork(env.single_observation_space, env.single_action_space,
                                                pi_hidden_sizes, v_hidden_sizes, init_layers_orthogonal,
                                                activation_fn, log_std_init, cnn_flatten_dim, cnn_style,
                                                cnn_layers_init_orthogonal)
        self._device: Optional[torch.device] = None
        # policy.py:31-36: the env's normalisation statistics travel with the checkpoint
        from .wrappers import NormalizeObservation, NormalizeReward, find_wrapper

        norm_obs = find_wrapper(env, NormalizeObservation)
        self.norm_observation_rms = norm_obs.rms if norm_obs else None
        norm_rew = find_wrapper(env, NormalizeReward)
        self.norm_reward_rms = norm_rew.rms if norm_rew else None
        self.load_path: Optional[str] = None

    # -- reference API ------------------------------------------------------------
    def to(self, device=None, *args, **kwargs):
        super().to(device, *args, **kwargs)
        if device is not None:
            self._device = torch.device(device)
        return self

    @property
    def device(self) -> torch.device:
        assert self._device is not None, "Expect device to be set"
        return self._device

    @property
    def action_shape(self) -> Tuple[int, ...]:
        return self.network.action_shape if self.gridnet else self.network._pi.action_shape

    @property
    def value_shape(self) -> Tuple[int, ...]:
        return self.network.value_shape if self.gridnet else ()

    @property
    def is_discrete(self) -> bool:
        return not self.gridnet and isinstance(self.network._pi, CategoricalActorHead)

    def forward(self, obs, action, action_masks=None, obs_prepared: bool = False) -> ACForward:
        """obs_prepared: obs came through the minibatch gather's transform (obs_transform())"""
        if obs_prepared:
            return ACForward(*self.network(obs, action, action_masks, obs_prepared=True))
        return ACForward(*self.network(obs, action, action_masks))

    def channels_last_params(self) -> list:
        """Parameters the flat buffer should store channels_last (optim.FlatParams): the NatureCNN
        convolution weights when the activations are NHWC on the GPU."""
        if self.gridnet or self.network._feature_extractor.kind != "cnn" or not _CHANNELS_LAST:
            return []
        cnn = self.network._feature_extractor.feature_extractor.cnn
        return [cnn[i].weight for i in (0, 2, 4)]

    def obs_transform(self, obs: torch.Tensor):
        """The gather transform (rai_gather_xform) that prepares rollout obs rows for forward(...,
        obs_prepared=True), or None (NatureCNN on uint8 frames only)."""
        if self.gridnet or self.network._feature_extractor.kind != "cnn":
            return None
        return self.network._feature_extractor.feature_extractor.obs_transform(obs)

    def _as_tensor(self, a):
        return torch.as_tensor(a).to(self.device)

    def value(self, obs: np.ndarray) -> np.ndarray:
        with torch.no_grad():
            return self.network.value(self._as_tensor(obs)).cpu().numpy()

    def step(self, obs: np.ndarray, action_masks=None) -> Step:
        """Numpy step for eval/enjoy parity (actor_critic.py:306-318); the trainer's
        rollout uses the HBM-resident path in rollout.py instead."""
        with torch.no_grad():
            o = self._as_tensor(obs)
            if self.gridnet:  # backbone_actor_critic.py:194-223 via actor_critic.py:306-318
                pi, v = self.network.distribution_and_value(o, self._as_tensor(action_masks))
                a = pi.sample()
                logp = pi.log_prob(a)
                a_np = a.cpu().numpy()
                return Step(a_np, v.cpu().numpy(), logp.cpu().numpy(), a_np)
            params, v = self.network.dist_params_and_value(o)
            if self.is_discrete:
                m = self._as_tensor(action_masks) if action_masks is not None else None
                if m is not None:
                    params = torch.where(m, params, F32_MIN)
                a = torch.multinomial(torch.softmax(params, -1), 1).squeeze(-1)
                logp, _ = self.network._pi.logp_entropy(params, a, m)
            else:
                a = params + torch.exp(self.network._pi.log_std) * torch.randn_like(params)
                logp, _ = self.network._pi.logp_entropy(params, a)
        a_np = a.cpu().numpy()
        return Step(a_np, v.cpu().numpy(), logp.cpu().numpy(), clamp_actions(a_np, self.action_space, False))

    def act(self, obs: np.ndarray, deterministic: bool = True, action_masks=None) -> np.ndarray:
        if not deterministic:
            return self.step(obs, action_masks=action_masks).clamped_a
        with torch.no_grad():
            o = self._as_tensor(obs)
            if self.gridnet:
                pi, _ = self.network.distribution_and_value(o, self._as_tensor(action_masks))
                return pi.mode.cpu().numpy()
            params, _ = self.network.dist_params_and_value(o)
            m = self._as_tensor(action_masks) if action_masks is not None else None
            a = self.network._pi.mode(params, m)
        return clamp_actions(a.cpu().numpy(), self.action_space, self.squash_output)

    def reset_noise(self, batch_size: Optional[int] = None) -> None:
        pass

    def save_weights(self, path: str) -> None:
        torch.save(self.state_dict(), os.path.join(path, MODEL_FILENAME))

    def load_weights(self, path: str) -> None:
        self.load_state_dict(torch.load(os.path.join(path, MODEL_FILENAME), map_location=self._device,
                                        weights_only=True))

    def save(self, path: str) -> None:  # policy.py:76-85
        os.makedirs(path, exist_ok=True)
        if self.norm_observation_rms:
            self.norm_observation_rms.save(os.path.join(path, NORMALIZE_OBSERVATION_FILENAME))
        if self.norm_reward_rms:
            self.norm_reward_rms.save(os.path.join(path, NORMALIZE_REWARD_FILENAME))
        self.save_weights(path)

    def load(self, path: str, load_norm_rms_count_override=None) -> None:  # policy.py:87-101
        self.load_path = path
        self.load_weights(path)
        if self.norm_observation_rms:
            self.norm_observation_rms.load(os.path.join(path, NORMALIZE_OBSERVATION_FILENAME),
                                           count_override=load_norm_rms_count_override)
        if self.norm_reward_rms:
            self.norm_reward_rms.load(os.path.join(path, NORMALIZE_REWARD_FILENAME),
                                      count_override=load_norm_rms_count_override)

    def sync_normalization(self, destination_env) -> None:  # policy.py:141-152
        from copy import deepcopy

        from .wrappers import NormalizeObservation, NormalizeReward

        current = destination_env
        while current is not current.unwrapped:
            if isinstance(current, NormalizeObservation):
                assert self.norm_observation_rms
                current.rms = deepcopy(self.norm_observation_rms)
            elif isinstance(current, NormalizeReward):
                assert self.norm_reward_rms
                current.rms = deepcopy(self.norm_reward_rms)
            current = getattr(current, "env", None)
            if current is None:
                raise AttributeError("wrapper chain without an env attribute")

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def freeze(self, freeze_policy_head: bool, freeze_value_head: bool, freeze_backbone: bool = True) -> None:
        if self.gridnet:  # backbone_actor_critic.py:254-265
            for mod, frz in ((self.network.actor_head, freeze_policy_head),
                             (self.network.critic_heads, freeze_value_head), (self.network.backbone, freeze_backbone)):
                for p in mod.parameters():
                    p.requires_grad = not frz
            return
        for p in self.network._pi.parameters():
            p.requires_grad = not freeze_policy_head
        for p in self.network._v.parameters():
            p.requires_grad = not freeze_value_head
        for p in self.network._feature_extractor.parameters():
            p.requires_grad = not freeze_backbone

    def unfreeze(self) -> None:
        self.freeze(False, False, False)


def clamp_actions(actions, action_space, squash_output: bool):
    """actor_critic.py:62-87 (Box: clip, or rescale when squash_output)."""
    if is_box(action_space):
        low, high = action_space.low, action_space.high
        if squash_output:
            return low + 0.5 * (actions + 1) * (high - low)
        return np.clip(actions, low, high)
    return actions


def mlp_actor_critic_spec(pol) -> Optional[dict]:
    """The CartPole-class structure the fused kernels implement (rai_mlp_ppo_epoch,
    rai_mlp_policy_step): an ActorCritic with a Flatten encoder, separate [in -> 64 -> 64 -> out]
    actor and critic MLPs (tanh or relu), a Categorical head, in_dim <= 8, n_actions <= 8,
    parameters() in the order actor W1,b1,W2,b2,W3,b3 then critic.  None otherwise."""
    if not isinstance(pol, ActorCritic) or pol.gridnet:
        return None
    net = pol.network
    if net._feature_extractor.kind != "flat" or not isinstance(net._pi, CategoricalActorHead):
        return None
    if net.pi_hidden_sizes != (64, 64) or net.v_hidden_sizes != (64, 64):
        return None
    if net.activation_fn not in ("tanh", "relu"):
        return None
    in_dim, n_act = net._feature_extractor.out_dim, net._pi.act_dim
    if not (1 <= in_dim <= 8 and 1 <= n_act <= 8):
        return None
    shapes = [tuple(p.shape) for p in pol.parameters()]
    want = []
    for out in (n_act, 1):
        want += [(64, in_dim), (64,), (64, 64), (64,), (out, 64), (out,)]
    if shapes != want:
        return None
    return dict(in_dim=in_dim, n_act=n_act, activation=0 if net.activation_fn == "tanh" else 1)
