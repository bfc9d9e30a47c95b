"""GAE / returns operator backed by the gfx950 reverse-scan kernel.

Drop-in for rl_algo_impls/shared/gae.py:97-124 (`compute_advantages`), same
signature, same numpy-in/numpy-out contract and the same AssertionErrors for
mismatched shapes (rl_algo_impls/shared/tensor_utils.py:7-31).  The device entry
`compute_advantages_device` runs on HBM-resident rollout buffers (the trainer's
path) and can also emit `returns = advantages + values` (vec_rollout.py:88) in
the same pass.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import _lib

NumOrArray = Union[float, np.ndarray]

EXACT = 0
FAST = 1


def _gamma_params(gamma: NumOrArray, gae_lambda: NumOrArray, value_col_shape: Tuple[int, ...]):
    """Broadcast gamma/lambda to per-column fp64 arrays following the reference's
    prepend_dims_to_match rule (gae.py:109-112); returns (gamma[K], lambda[K], is_vector)."""
    K = int(np.prod(value_col_shape[1:])) if len(value_col_shape) > 1 else 1

    def col_array(x, name):
        if isinstance(x, np.ndarray):
            assert x.shape == value_col_shape[-len(x.shape):], (
                f"Array {x.shape} must match later dims of {value_col_shape}"
            )
            if len(value_col_shape) < 2 or x.shape[0] != K or x.ndim != 1:
                raise NotImplementedError(f"{name} must be a float or an ndarray of shape (K,)")
            return np.ascontiguousarray(x, dtype=np.float64), True
        return np.full((K,), float(x), dtype=np.float64), False

    g, g_vec = col_array(gamma, "gamma")
    lam, _ = col_array(gae_lambda, "gae_lambda")
    if K > _lib.RAI_MAX_K:
        raise NotImplementedError(f"K={K} value columns exceeds RAI_MAX_K={_lib.RAI_MAX_K}")
    return g, lam, g_vec


def compute_advantages_device(
    rewards: torch.Tensor,
    values: torch.Tensor,
    episode_starts: torch.Tensor,
    next_episode_starts: torch.Tensor,
    next_values: torch.Tensor,
    gamma: NumOrArray,
    gae_lambda: NumOrArray,
    *,
    mode: int = EXACT,
    advantages_out: Optional[torch.Tensor] = None,
    returns_out: Optional[torch.Tensor] = None,
    want_returns: bool = False,
) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """GAE on device tensors: rewards/values (T, N[, K]) f32, episode_starts (T, N)
    bool/u8, next_episode_starts (N,), next_values (N[, K]).  Returns (adv, returns)."""
    _lib.require_device(rewards, values, episode_starts, next_episode_starts, next_values)
    if rewards.dtype != torch.float32 or values.dtype != torch.float32 or next_values.dtype != torch.float32:
        raise ValueError("rollout buffers must be float32 (reference sync_step_rollout.py:99-101)")
    assert rewards.shape == values.shape, f"rewards {tuple(rewards.shape)} != values {tuple(values.shape)}"
    T, N = int(values.shape[0]), int(values.shape[1])
    col_shape = tuple(values.shape[1:])
    assert tuple(next_values.shape) == col_shape, (
        f"next_values {tuple(next_values.shape)} must be {col_shape}"
    )
    assert tuple(episode_starts.shape) == (T, N), f"episode_starts must be {(T, N)}"
    assert tuple(next_episode_starts.shape) == (N,), (
        f"Array {tuple(next_episode_starts.shape)} must match early dims of {col_shape}"
    )
    g, lam, g_vec = _gamma_params(gamma, gae_lambda, col_shape)
    K = len(g)
    es = episode_starts.contiguous().view(torch.uint8) if episode_starts.dtype == torch.bool else episode_starts.to(torch.uint8).contiguous()
    nes = next_episode_starts.contiguous().view(torch.uint8) if next_episode_starts.dtype == torch.bool else next_episode_starts.to(torch.uint8).contiguous()
    r = rewards.contiguous()
    v = values.contiguous()
    nv = next_values.contiguous()
    adv = advantages_out if advantages_out is not None else torch.empty_like(v)
    ret = returns_out if returns_out is not None else (torch.empty_like(v) if want_returns else None)
    gp = g.ctypes.data_as(C.POINTER(C.c_double))
    lp = lam.ctypes.data_as(C.POINTER(C.c_double))
    rc = _lib.lib().rai_gae(
        r.data_ptr(), v.data_ptr(), es.data_ptr(), nes.data_ptr(), nv.data_ptr(), T, N, K, gp, lp,
        int(g_vec), int(mode), adv.data_ptr(), _lib.ptr(ret), _lib.stream_handle(v.device),
    )
    _lib.check(rc, "rai_gae")
    return adv, ret


def compute_advantages(
    rewards: np.ndarray,
    values: np.ndarray,
    episode_starts: np.ndarray,
    next_episode_starts: np.ndarray,
    next_values: np.ndarray,
    gamma: NumOrArray,
    gae_lambda: NumOrArray,
    device: Optional[torch.device] = None,
) -> np.ndarray:
    """Host-array drop-in for rl_algo_impls.shared.gae.compute_advantages; runs the
    exact-mode HIP kernel (bit-identical to the reference) and returns numpy."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    next_episode_starts = np.asarray(next_episode_starts)
    next_values = np.asarray(next_values)
    assert next_episode_starts.shape == next_values.shape[: len(next_episode_starts.shape)], (
        f"Array {next_episode_starts.shape} must match early dims of {next_values.shape}"
    )
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=False)
    adv, _ = compute_advantages_device(
        t(rewards), t(values), t(episode_starts.astype(np.bool_)), t(next_episode_starts.astype(np.bool_)),
        t(next_values), gamma, gae_lambda, mode=EXACT,
    )
    return adv.cpu().numpy()
