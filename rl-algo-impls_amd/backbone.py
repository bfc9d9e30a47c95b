"""Squeeze-U-Net GridNet actor-critic (MicroRTS, BASELINE config C5) on PyTorch-ROCm.

Mirrors, for state_dict keys, parameter shapes and the seeded initialisation order:

  SqueezeExcitation / SEResidualBlock   rl_algo_impls/shared/policy/actor_critic_network/double_cone.py:18-86
  SqueezeUnetBackbone                    rl_algo_impls/shared/policy/actor_critic_network/squeeze_unet.py:20-195
  SqueezeUnetActorCriticNetwork          squeeze_unet.py:198-270
  BackboneActorCritic (actor head, critic heads, _preprocess, value)
                                         rl_algo_impls/shared/policy/actor_critic_network/backbone_actor_critic.py:31-232

The backbone's convolutions run on MIOpen / hipBLASLt (the north star keeps the CNN contractions on
PyTorch-ROCm).  The GridNet head's log-prob and entropy over every cell and sub-action is the fused
HIP operator of gridnet.py (one launch forward, one backward) instead of the reference's H*W*7
MaskedCategoricals.  Normalisation layers (`normalization=...`), the non-shared critic
(`critic_shares_backbone=False`, `save_critic_separate`), the shared critic head and the Lux
`pick_position` action space are outside the hot path and raise NotImplementedError.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch
import torch.nn as nn

from .gridnet import GridnetDistribution, ValueDependentMask

Strides = Sequence[Union[int, Sequence[int]]]
# NHWC activations on the GPU (RAI_SQUNET_NHWC=0 keeps NCHW): MIOpen's implicit-GEMM solvers take
# them without the NCHW<->NHWC transposes, and the fused SE epilogue below runs on them.  (The
# NatureCNN encoder has its own switch, RAI_CHANNELS_LAST, also on by default.)
_CHANNELS_LAST = os.environ.get("RAI_SQUNET_NHWC", "1") == "1"
if _CHANNELS_LAST:
    os.environ.setdefault("PYTORCH_MIOPEN_SUGGEST_NHWC", "1")


def _nhwc(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.float32 and t.dim() == 4 and t.is_contiguous(
        memory_format=torch.channels_last)


class _SEResidualEpilogue(torch.autograd.Function):
    """GELU(x + r * s) (double_cone.py:43-47,85-86) as one HIP pass forward and one backward
    (rai_se_residual_fwd / _bwd, csrc/se_block.hip); NHWC fp32 activations, s (B, C)."""

    @staticmethod
    def forward(ctx, x, r, s):
        from . import _lib

        B, C, H, W = (int(d) for d in x.shape)
        s = s.contiguous()
        out = torch.empty_like(x)
        _lib.check(_lib.lib().rai_se_residual_fwd(x.data_ptr(), r.data_ptr(), s.data_ptr(), B, C, H * W,
                                                  out.data_ptr(), _lib.stream_handle(x.device)),
                   "rai_se_residual_fwd")
        ctx.save_for_backward(x, r, s)
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import _lib

        x, r, s = ctx.saved_tensors
        B, C, H, W = (int(d) for d in x.shape)
        dout = dout.contiguous(memory_format=torch.channels_last)
        dx, dr, ds = torch.empty_like(x), torch.empty_like(r), torch.empty_like(s)
        _lib.check(_lib.lib().rai_se_residual_bwd(dout.data_ptr(), x.data_ptr(), r.data_ptr(), s.data_ptr(), B, C,
                                                  H * W, dx.data_ptr(), dr.data_ptr(), ds.data_ptr(),
                                                  _lib.stream_handle(x.device)), "rai_se_residual_bwd")
        return dx, dr, ds


class _BiasGelu(torch.autograd.Function):
    """GELU(x + b) over an NHWC conv output (rai_bias_gelu_fwd / _bwd): MIOpen's separate bias pass and
    the GELU kernel in one pass; the bias gradient is the rows-sum of dx."""

    @staticmethod
    def forward(ctx, x, b):
        from . import _lib

        C = int(x.shape[1])
        out = torch.empty_like(x)
        _lib.check(_lib.lib().rai_bias_gelu_fwd(x.data_ptr(), b.data_ptr(), x.numel() // C, C, out.data_ptr(),
                                                _lib.stream_handle(x.device)), "rai_bias_gelu_fwd")
        ctx.save_for_backward(x, b)
        return out

    @staticmethod
    def backward(ctx, dy):
        from . import _lib

        x, b = ctx.saved_tensors
        C = int(x.shape[1])
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        _lib.check(_lib.lib().rai_bias_gelu_bwd(dy.data_ptr(), x.data_ptr(), b.data_ptr(), x.numel() // C, C,
                                                dx.data_ptr(), _lib.stream_handle(x.device)), "rai_bias_gelu_bwd")
        # NHWC: dx viewed (rows, C) is contiguous; the bias gradient is its column sum
        db = dx.permute(0, 2, 3, 1).reshape(-1, C).sum(0)
        return dx, db


def conv_gelu(conv: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """GELU(conv(x)) for a Conv2d / ConvTranspose2d with bias: on NHWC fp32 GPU activations the
    convolution runs bias-free on MIOpen and bias + GELU is one HIP pass; else the modules' own path."""
    if _nhwc(x) and conv.bias is not None and conv.out_channels % 4 == 0:
        if isinstance(conv, nn.ConvTranspose2d):
            y = torch.nn.functional.conv_transpose2d(x, conv.weight, None, conv.stride, conv.padding,
                                                     conv.output_padding, conv.groups, conv.dilation)
        else:
            y = torch.nn.functional.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation,
                                           conv.groups)
        if _nhwc(y):
            return _BiasGelu.apply(y, conv.bias)
        return torch.nn.functional.gelu(y + conv.bias.view(1, -1, 1, 1))
    return torch.nn.functional.gelu(conv(x))


def run_sequential(seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """seq(x) with every (conv, GELU) pair through conv_gelu (same modules, same state_dict)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if (isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)) and i + 1 < len(mods)
                and isinstance(mods[i + 1], nn.GELU) and mods[i + 1].approximate == "none"):
            x = conv_gelu(m, x)
            i += 2
        else:
            x = m(x)
            i += 1
    return x


def se_residual_epilogue(x: torch.Tensor, r: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """GELU(x + r * s[..., None, None]); the fused HIP pass for NHWC fp32 GPU activations whose C
    the kernel tiles (C % 4 == 0, C / 4 divides 256), else the PyTorch composition."""
    C = int(x.shape[1]) if x.dim() == 4 else 0
    if (_nhwc(x) and _nhwc(r) and r.shape == x.shape and C % 4 == 0 and C >= 4 and 256 % (C // 4) == 0
            and s.is_cuda and s.dtype == torch.float32):
        return _SEResidualEpilogue.apply(x, r, s)
    return torch.nn.functional.gelu(x + r * s.view(s.shape[0], s.shape[1], 1, 1))


def _init(layer: nn.Module, orthogonal: bool, std: float = float(np.sqrt(2))) -> nn.Module:
    """shared/module/utils.py:36-45 (bias-free layers: orthogonal weight only)."""
    if orthogonal:
        nn.init.orthogonal_(layer.weight, std)
        if getattr(layer, "bias", None) is not None:
            nn.init.constant_(layer.bias, 0.0)
    return layer


def _as_list(s) -> List[int]:
    return list(s) if isinstance(s, (list, tuple)) else [int(s)]


class SqueezeExcitation(nn.Module):  # double_cone.py:18-47
    def __init__(self, in_channels: int, reduction_ratio: int = 16, init_layers_orthogonal: bool = False) -> None:
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        mid = in_channels // reduction_ratio
        self.fc = nn.Sequential(_init(nn.Linear(in_channels, mid, bias=False), init_layers_orthogonal), nn.GELU(),
                                _init(nn.Linear(mid, in_channels, bias=False), init_layers_orthogonal), nn.Sigmoid())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, c = x.shape[0], x.shape[1]
        return x * self.fc(self.avg_pool(x).view(b, c)).view(b, c, 1, 1)


class SEResidualBlock(nn.Module):  # double_cone.py:50-86 (normalization=None)
    def __init__(self, channels: int, init_layers_orthogonal: bool = False) -> None:
        super().__init__()
        conv = lambda: _init(nn.Conv2d(channels, channels, 3, padding=1), init_layers_orthogonal)
        c0 = conv()
        act = nn.GELU()
        c1 = conv()
        self.residual = nn.Sequential(c0, act, c1, SqueezeExcitation(channels,
                                                                     init_layers_orthogonal=init_layers_orthogonal))
        self.gelu = nn.GELU()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        conv0, act, conv1, se = self.residual
        r = conv1(conv_gelu(conv0, x))  # act = GELU
        b, c = r.shape[0], r.shape[1]
        s = se.fc(se.avg_pool(r).view(b, c))
        return se_residual_epilogue(x, r, s)  # == self.gelu(x + self.residual(x))


class SqueezeUnetBackbone(nn.Module):  # squeeze_unet.py:20-195
    """Encoder levels (3x3 head conv + SE blocks; then per level strided down-convs + SE blocks),
    decoder levels (transposed-conv up-sampling + SE blocks) with additive skips."""

    def __init__(self, in_channels: int, channels_per_level: List[int], strides_per_level: Strides,
                 encoder_residual_blocks_per_level: List[int], decoder_residual_blocks_per_level: List[int],
                 deconv_strides_per_level: Optional[Strides] = None, init_layers_orthogonal: bool = False,
                 increment_kernel_size_on_down_conv: bool = False, normalization: Optional[str] = None) -> None:
        super().__init__()
        if normalization:
            raise NotImplementedError("squeeze-U-Net normalization layers are outside the hot-path scope")
        orth = init_layers_orthogonal
        ch = list(channels_per_level)
        se = lambda c, n: [SEResidualBlock(c, init_layers_orthogonal=orth) for _ in range(n)]

        def down(cin: int, cout: int, stride) -> List[nn.Module]:
            mods: List[nn.Module] = []
            for i, s in enumerate(_as_list(stride)):
                k, pad = s, 0
                if increment_kernel_size_on_down_conv and s % 2 == 0:  # squeeze_unet.py:47-55
                    k, pad = s + 1, 1
                mods += [_init(nn.Conv2d(cin if i == 0 else cout, cout, kernel_size=k, stride=s, padding=pad), orth),
                         nn.GELU()]
            return mods

        def up(cin: int, cout: int, stride) -> List[nn.Module]:
            mods: List[nn.Module] = []
            for i, s in enumerate(_as_list(stride)):
                mods += [_init(nn.ConvTranspose2d(cin if i == 0 else cout, cout, kernel_size=s, stride=s), orth),
                         nn.GELU()]
            return mods

        head = [_init(nn.Conv2d(in_channels, ch[0], 3, padding=1), orth), nn.GELU()]
        self.encoders = nn.ModuleList([nn.Sequential(*(head + se(ch[0], encoder_residual_blocks_per_level[0])))])
        for lvl in range(1, len(ch)):
            self.encoders.append(nn.Sequential(*(down(ch[lvl - 1], ch[lvl], strides_per_level[lvl - 1])
                                                 + se(ch[lvl], encoder_residual_blocks_per_level[lvl]))))
        dstr = list(deconv_strides_per_level or strides_per_level)
        self.decoders = nn.ModuleList([nn.Sequential(*up(ch[-1], ch[-2], dstr[-1]))])
        # middle levels, deepest first: SE blocks at the level's width, then up-sample one level
        # (squeeze_unet.py:151-171 zips the reversed lists, so it stops at the shortest)
        mids = list(zip(reversed(ch[1:-1]), reversed(ch[:-2]), reversed(dstr[:-1]),
                        reversed(decoder_residual_blocks_per_level[:-1])))
        for c, cout, s, n in mids:
            self.decoders.append(nn.Sequential(*(se(c, n) + up(c, cout, s))))
        self.decoders.append(nn.Sequential(*se(ch[0], decoder_residual_blocks_per_level[0])))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        skips = []
        for enc in self.encoders:
            x = run_sequential(enc, x)
            skips.append(x)
        d = None
        for e, dec in zip(reversed(skips), self.decoders):
            d = run_sequential(dec, e if d is None else e + d)  # the reference adds zeros_like at the deepest level
        return d


class _Transpose(nn.Module):  # actor/gridnet_decoder.py:14-20
    def __init__(self, permutation) -> None:
        super().__init__()
        self.permutation = tuple(permutation)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x.permute(self.permutation)


class _HStack(nn.ModuleList):  # shared/module/stack.py
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.hstack([run_sequential(m, x) for m in self])


_OUT_ACT = {"tanh": nn.Tanh, "relu": nn.ReLU, "identity": nn.Identity, "sigmoid": nn.Sigmoid}


class SqueezeUnetActorCriticNetwork(nn.Module):
    """squeeze_unet.py:198-270 + backbone_actor_critic.py:31-232 (per-position GridNet actions)."""

    def __init__(self, observation_space, action_space, action_plane_space, init_layers_orthogonal: bool = True,
                 cnn_layers_init_orthogonal: Optional[bool] = None, channels_per_level: Optional[List[int]] = None,
                 strides_per_level: Optional[Strides] = None, deconv_strides_per_level: Optional[Strides] = None,
                 encoder_residual_blocks_per_level: Optional[List[int]] = None,
                 decoder_residual_blocks_per_level: Optional[List[int]] = None, num_additional_critics: int = 0,
                 additional_critic_activation_functions: Optional[List[str]] = None, critic_channels: int = 64,
                 increment_kernel_size_on_down_conv: bool = False, output_activation_fn: str = "identity",
                 subaction_mask: Optional[Dict[int, Dict[int, int]]] = None, critic_shares_backbone: bool = True,
                 save_critic_separate: bool = False, shared_critic_head: bool = False,
                 normalization: Optional[str] = None) -> None:
        super().__init__()
        if not critic_shares_backbone or save_critic_separate or shared_critic_head:
            raise NotImplementedError("non-shared / shared-head critics are outside the hot-path scope")
        cnn_orth = bool(cnn_layers_init_orthogonal) if cnn_layers_init_orthogonal is not None else False
        ch = list(channels_per_level or [64, 128, 256])
        strides = list(strides_per_level or [2] * (len(ch) - 1))
        enc_blocks = list(encoder_residual_blocks_per_level or [1] * len(ch))
        dec_blocks = list(decoder_residual_blocks_per_level or enc_blocks[:-1])
        assert len(strides) == len(ch) - 1 and len(enc_blocks) == len(ch) and len(dec_blocks) == len(ch) - 1
        if num_additional_critics and not additional_critic_activation_functions:
            additional_critic_activation_functions = ["identity"] * num_additional_critics
        # construction order = the reference's (backbone, actor head, critic heads): the seeded
        # default initialisation consumes the RNG identically
        self.backbone = SqueezeUnetBackbone(int(observation_space.shape[0]), ch, strides, enc_blocks, dec_blocks,
                                            deconv_strides_per_level=deconv_strides_per_level,
                                            init_layers_orthogonal=cnn_orth,
                                            increment_kernel_size_on_down_conv=increment_kernel_size_on_down_conv,
                                            normalization=normalization)
        self.range_size = float(np.max(observation_space.high) - np.min(observation_space.low))
        self.action_vec = np.asarray(action_plane_space.nvec)
        if isinstance(action_space, dict) or hasattr(action_space, "spaces"):
            raise NotImplementedError("pick_position (Lux) GridNet actions are outside the hot path")
        self.map_size = len(action_space.nvec) // len(self.action_vec)
        self.subaction_mask = subaction_mask
        self._sub = (ValueDependentMask.from_reference_index_to_index_to_value(subaction_mask)
                     if subaction_mask else None)
        self.actor_head = nn.Sequential(
            _init(nn.Conv2d(ch[0], int(self.action_vec.sum()), kernel_size=3, padding=1), init_layers_orthogonal,
                  std=0.01),
            _Transpose((0, 2, 3, 1)))
        flat_strides: List[int] = []
        for s in strides:
            flat_strides += _as_list(s)

        def critic(act: nn.Module) -> nn.Sequential:  # backbone_actor_critic.py:111-171
            mods: List[nn.Module] = []
            cin = ch[0]
            for s in flat_strides:
                k = max(3, s)
                mods += [_init(nn.Conv2d(cin, critic_channels, k, stride=s, padding=1 if k % 2 else 0), cnn_orth),
                         nn.GELU()]
                cin = critic_channels
            mods += [nn.AdaptiveAvgPool2d(1), nn.Flatten(),
                     _init(nn.Linear(critic_channels, critic_channels), init_layers_orthogonal), nn.GELU(),
                     _init(nn.Linear(critic_channels, 1), init_layers_orthogonal, std=1.0), act]
            return nn.Sequential(*mods)

        acts = [_OUT_ACT[n]() for n in [output_activation_fn] + list(additional_critic_activation_functions or [])]
        self._critic_features = len(acts)
        self.critic_heads = _HStack([critic(a) for a in acts])

    # -- backbone_actor_critic.py:189-232 ----------------------------------------------------
    def _preprocess(self, obs: torch.Tensor) -> torch.Tensor:
        if obs.dim() == 3:
            obs = obs.unsqueeze(0)
        x = obs.float() / self.range_size
        if _CHANNELS_LAST and x.is_cuda:  # NHWC activations for MIOpen's implicit-GEMM solvers
            x = x.contiguous(memory_format=torch.channels_last)
        return x

    def _values(self, x: torch.Tensor) -> torch.Tensor:
        v = self.critic_heads(x)
        return v.squeeze(-1) if v.shape[-1] == 1 else v

    def distribution_and_value(self, obs: torch.Tensor, action_masks: torch.Tensor):
        if action_masks is None:
            raise AssertionError("No mask case unhandled in SqueezeUnetActorCriticNetwork")
        o = self._preprocess(obs)
        x = self.backbone(o)
        pi = GridnetDistribution(int(np.prod(o.shape[-2:])), self.action_vec, self.actor_head(x), action_masks,
                                 subaction_mask=self._sub)
        return pi, self._values(x)

    def logits_and_value(self, obs: torch.Tensor):
        """(actor-head logits (B, H, W, sum(nvec)), values) — the graph-captured rollout forward."""
        x = self.backbone(self._preprocess(obs))
        return self.actor_head(x), self._values(x)

    def distribution(self, logits: torch.Tensor, action_masks: torch.Tensor) -> GridnetDistribution:
        return GridnetDistribution(int(np.prod(logits.shape[1:3])), self.action_vec, logits, action_masks,
                                   subaction_mask=self._sub)

    def forward(self, obs, action, action_masks=None):
        pi, v = self.distribution_and_value(obs, action_masks)
        logp = pi.log_prob(action)
        return logp, pi.entropy(), v

    def value(self, obs: torch.Tensor) -> torch.Tensor:
        return self._values(self.backbone(self._preprocess(obs)))

    @property
    def action_shape(self):
        return (self.map_size, len(self.action_vec))

    @property
    def value_shape(self):
        return (self._critic_features,) if self._critic_features > 1 else ()
