"""ctypes binding of the C ABI in include/rai_amd.h (librai_amd.so).

The library is loaded AFTER torch so that its DT_NEEDED libamdhip64.so.7 resolves
(by SONAME) to the HIP runtime torch already mapped: torch's streams and device
pointers are then valid arguments.  There is no CPU fallback: if the library is
missing or cannot be loaded, every product entry point raises.
"""
from __future__ import annotations

import ctypes as C
import re
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from .build import lib_path

RAI_MAX_K = 8
RAI_MAX_FIELDS = 8
RAI_GRID_MAX_G = 8
RAI_GRID_MAX_A = 256
RAI_WIDE_MAX_B = 256
RAI_MLP_EPOCH_MAX_B = 256  # rai_mlp_ppo_epoch's one-launch epoch kernels; larger minibatches: mlp_large.hip
RAI_WIDE_MAX_H = 256
RAI_WIDE_MAX_IN = 64
RAI_WIDE_MAX_OUT = 8
RAI_STAT_STRIDE = 5 + 2 * RAI_MAX_K
ABI_VERSION = 1
# the RAI_E_* return codes of include/rai_amd.h (tests/test_boundary.py checks them against the header)
RAI_E_NULLPTR = -1
RAI_E_SHAPE = -2
RAI_E_MODE = -3
RAI_E_TOO_MANY_COLUMNS = -4
RAI_E_WORKSPACE = -5
RAI_E_UNSUPPORTED = -6
RAI_E_DP_BASE = -1000


class PPOHparams(C.Structure):
    """Mirror of rai_ppo_hparams (device-resident hyperparameters)."""

    _fields_ = [
        ("clip_range", C.c_float),
        ("clip_range_vf", C.c_float),
        ("ent_coef", C.c_float),
        ("kl_cutoff", C.c_float),
        ("grad_scale", C.c_float),
        ("K", C.c_int32),
        ("has_clip_range_vf", C.c_int32),
        ("has_kl_cutoff", C.c_int32),
        ("normalize_advantage", C.c_int32),
        ("standardize_advantage", C.c_int32),
        ("normalize_after_scaling", C.c_int32),
        ("ppo2_vf_coef_halving", C.c_int32),
        ("has_vf_weights", C.c_int32),
        ("has_multi_reward_weights", C.c_int32),
        ("vf_loss_fn", C.c_int32),
        ("loss_kind", C.c_int32),
        ("vf_coef", C.c_float * RAI_MAX_K),
        ("vf_weights", C.c_float * RAI_MAX_K),
        ("multi_reward_weights", C.c_float * RAI_MAX_K),
        ("ext_moments", C.c_void_p),
    ]


class MinibatchDesc(C.Structure):
    """Mirror of rai_minibatch_desc."""

    _fields_ = [
        ("src", C.c_void_p * RAI_MAX_FIELDS),
        ("row_bytes", C.c_int64 * RAI_MAX_FIELDS),
        ("perm", C.c_void_p),
        ("n_rows", C.c_int64),
        ("batch_size", C.c_int64),
        ("mb", C.c_int64),
        ("n_fields", C.c_int32),
        ("arrivals", C.c_int32),
        ("group_arrivals", C.c_int32 * 128),
    ]


RAI_XFORM_COPY = 0
RAI_XFORM_U8_CHW_TO_F32_HWC = 1
RAI_XFORM_U8_CHW_TO_U8_HWC = 2


class GatherXform(C.Structure):
    """Mirror of rai_gather_xform (per-field output transform of the minibatch gather)."""

    _fields_ = [
        ("kind", C.c_int32),
        ("channels", C.c_int32),
        ("hw", C.c_int64),
        ("divisor", C.c_float),
        ("reserved", C.c_int32),
    ]


class MlpWideDesc(C.Structure):
    """Mirror of rai_mlp_wide_desc."""

    _fields_ = [
        ("w", (C.c_void_p * 6) * 2),
        ("g", (C.c_void_p * 6) * 2),
        ("log_std", C.c_void_p),
        ("g_log_std", C.c_void_p),
        ("in_dim", C.c_int32),
        ("hidden", C.c_int32),
        ("out_pi", C.c_int32),
        ("head", C.c_int32),
        ("activation", C.c_int32),
        ("accumulate", C.c_int32),
    ]


class OptimHparams(C.Structure):
    _fields_ = [
        ("lr", C.c_float),
        ("beta1", C.c_float),
        ("beta2", C.c_float),
        ("eps", C.c_float),
        ("alpha", C.c_float),
        ("max_grad_norm", C.c_float),
        ("kind", C.c_int32),
        ("pad", C.c_int32),
        ("beta1_d", C.c_double),
        ("beta2_d", C.c_double),
    ]


class TrainState(C.Structure):
    _fields_ = [
        ("opt_step", C.c_int64),
        ("stat_index", C.c_int32),
        ("pi_coef_zero", C.c_int32),
        ("norm_index", C.c_int32),
        ("err", C.c_int32),
    ]


_vp, _i32, _i64, _u64, _f64p = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.POINTER(C.c_double)

_SIGNATURES = {
    "rai_abi_version": (C.c_int, []),
    "rai_strerror": (C.c_char_p, [C.c_int]),
    "rai_gae": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _f64p, _f64p, _i32, _i32, _vp, _vp, _vp]),
    "rai_ppo_loss_workspace_bytes": (_i64, [_i64, _i32]),
    "rai_ppo_loss": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp,
                               _vp, _i32, _vp, _i64, _vp]),
    "rai_optim_workspace_bytes": (_i64, [_i64]),
    "rai_clip_optim_step": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_gather_rows": (C.c_int, [_i32, _vp, _vp, _vp, _vp, _i64, _vp]),
    "rai_feistel_permutation": (C.c_int, [_i64, C.c_uint64, _vp, _vp]),
    "rai_copy_d2h_sync": (C.c_int, [_vp, _vp, _i64, _vp]),
    "rai_mlp_policy_step_mapped": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _u64, _u64, _vp, _vp,
                                             _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "rai_host_alloc": (C.c_int, [_i64, _vp, _vp]),
    "rai_host_free": (C.c_int, [_vp]),
    "rai_stream_sync": (C.c_int, [_vp]),
    "rai_copy_h2d_multi": (C.c_int, [_i32, _vp, _vp, _vp, _vp]),
    "rai_gae_trajectories": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _f64p, _f64p, _i32, _i32, _vp, _vp, _vp]),
    "rai_gridnet_logp_entropy": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "rai_gridnet_backward": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "rai_se_residual_fwd": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp]),
    "rai_se_residual_bwd": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp]),
    "rai_bias_gelu_fwd": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "rai_bias_gelu_bwd": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp]),
    "rai_gridnet_sample": (C.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, C.c_uint64, C.c_uint64, _vp, _vp,
                                     _vp]),
    "rai_gridnet_num_actions": (C.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp, _vp]),
    "rai_mlp_wide_workspace_bytes": (_i64, [_i64, _i32]),
    "rai_mlp_wide_forward": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "rai_mlp_wide_forward_loss": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_mlp_wide_backward": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "rai_mlp_wide_dist_params": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp]),
    "rai_mlp_wide_epoch_workspace_bytes": (_i64, [_i32, _i32, _i64]),
    "rai_mlp_wide_epoch": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp,
                                     _vp, _vp, _i32, _vp, _i32, _vp, _i64, _vp]),
    "rai_mlp_wide_epoch_xdp": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i32,
                                         _i32, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _i32, _vp, _i64, _vp]),
    "rai_gae_skips": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "rai_gather_minibatch": (C.c_int, [_vp, _i32, _vp, _vp, _i64, _vp]),
    "rai_minibatch_advance": (C.c_int, [_vp, _vp]),
    "rai_gather_minibatch_next": (C.c_int, [_vp, _i32, _vp, _vp, _i64, _vp]),
    "rai_gather_minibatch_x": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _i64, _i32, _vp]),
    "rai_bias_relu_workspace_bytes": (_i64, [_i32]),
    "rai_categorical_critic_heads_fwd": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp,
                                                   _vp]),
    "rai_categorical_critic_heads_workspace_bytes": (_i64, [_i64, _i32]),
    "rai_categorical_critic_heads_bwd": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp,
                                                   _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_categorical_critic_heads_bwd_relu": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp,
                                                        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_bias_relu_fwd": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "rai_bias_relu_bwd": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_bias_relu_fwd_nchw": (C.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp]),
    "rai_conv2d_fwd_splitk_bytes": (_i64, [_i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32]),
    "rai_conv2d_bias_relu_fwd_splitk": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                                  _vp, _vp, _i64, _vp]),
    "rai_conv2d_bias_relu_fwd": (C.c_int, [_vp, _vp, _vp, _i64] + [_i32] * 8 + [_vp, _vp]),
    "rai_conv2d_bias_relu_fwd_v": (C.c_int, [_vp, _vp, _vp, _i64] + [_i32] * 8 + [_vp, _i32, _vp]),
    "rai_conv2d_wgrad_workspace_bytes": (_i64, [_i64] + [_i32] * 7),
    "rai_conv2d_wgrad": (C.c_int, [_vp, _vp, _i64] + [_i32] * 7 + [_vp, _i32, _vp, _i64, _vp]),
    "rai_conv2d_wgrad_v": (C.c_int, [_vp, _vp, _i64] + [_i32] * 7 + [_vp, _i32, _vp, _i64, _i32, _i32, _vp]),
    "rai_conv2d_wgrad_partials": (C.c_int, [_vp, _vp, _i64] + [_i32] * 7 + [_vp, _i64, _vp]),
    "rai_conv2d_wgrad_reduce": (C.c_int, [_vp, _i32, _i32, _vp]),
    "rai_conv2d_wgrad_relu_partials": (C.c_int, [_vp, _vp, _vp, _i64] + [_i32] * 7 + [_vp, _i64, _vp]),
    "rai_conv2d_bias_relu_fwd_u8": (C.c_int, [_vp, C.c_float, _vp, _vp, _i64] + [_i32] * 8 + [_vp, _vp]),
    "rai_conv2d_wgrad_partials_u8": (C.c_int, [_vp, C.c_float, _vp, _i64] + [_i32] * 7 + [_vp, _i64, _vp]),
    "rai_conv2d_wgrad_relu_partials_u8": (C.c_int, [_vp, _vp, _vp, C.c_float, _i64] + [_i32] * 7 + [_vp, _i64, _vp]),
    "rai_conv2d_dgrad": (C.c_int, [_vp, _vp, _i64] + [_i32] * 7 + [_vp, _vp]),
    "rai_conv2d_dgrad_v": (C.c_int, [_vp, _vp, _i64] + [_i32] * 7 + [_vp, _i32, _vp]),
    "rai_conv2d_dgrad_relu": (C.c_int, [_vp, _vp, _vp, _i64] + [_i32] * 7 + [_vp, _vp]),
    "rai_bias_relu_bwd_nchw": (C.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_mlp_ppo_workspace_bytes": (_i64, [C.c_int64, C.c_int32]),
    "rai_mlp_ppo_grads": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _i32, _i32,
                                    _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp]),
    "rai_mlp_ppo_epoch": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32,
                                    _i32, _vp, _vp, _vp, _vp, _i32, _vp, _i32, _vp, _i64, _vp]),
    "rai_mlp_large_timing": (C.c_int, [_i32]),
    "rai_mlp_large_timing_read": (C.c_int, [_vp, _i32, _vp]),
    "rai_categorical_sample": (C.c_int, [_vp, _vp, _i64, _i32, _u64, _u64, _vp, _vp, _vp, _vp, _i32, _vp]),
    "rai_gaussian_sample": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp,
                                      _i32, _vp]),
    "rai_mlp_policy_step": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _u64, _u64, _vp, _vp, _vp,
                                      _vp]),
    "rai_dp_available": (C.c_int, []),
    "rai_dp_unique_id": (C.c_int, [_vp, _i32]),
    "rai_dp_comm_init": (C.c_int, [C.POINTER(C.c_void_p), _vp, _i32, _i32]),
    "rai_dp_comm_destroy": (C.c_int, [_vp]),
    "rai_dp_allreduce_sum_f32": (C.c_int, [_vp, _vp, _i64, _vp]),
    "rai_mlp_ppo_epoch_dp": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp,
                                       _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _i32, _vp,
                                       _vp, _vp, _i64, _vp, _i64, _vp]),
    "rai_xdp_region_bytes": (_i64, [_i32]),
    "rai_xdp_handle_bytes": (C.c_int, []),
    "rai_xdp_alloc": (C.c_int, [_i64, C.POINTER(C.c_void_p)]),
    "rai_xdp_free": (C.c_int, [_vp]),
    "rai_xdp_handle": (C.c_int, [_vp, _vp, _i32]),
    "rai_xdp_open": (C.c_int, [_vp, C.POINTER(C.c_void_p)]),
    "rai_xdp_close": (C.c_int, [_vp]),
    "rai_xdp_selftest": (C.c_int, [_vp, _i32, _i32, _i64, _vp, _vp]),
    "rai_mlp_ppo_epoch_xdp": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i32, _i32,
                                        _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _i32,
                                        _vp, _i64, _vp]),
}
RAI_DP_UID_BYTES = 128
EXPORTED = tuple(_SIGNATURES)

_lock = threading.Lock()
_lib = None


def hip_runtimes_mapped() -> list[str]:
    try:
        maps = open("/proc/self/maps").read()
    except OSError:
        return []
    return sorted(set(re.findall(r"\S*libamdhip64\.so\S*", maps)))


def lib_sha256(path=None) -> str:
    """sha256 of the C-ABI library file (default: the one lib() loads).  PMC summaries record it, and
    bench.py reports a counter figure only when it was measured on this same binary."""
    import hashlib

    with open(path or lib_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def lib() -> C.CDLL:
    """Load (once) and return the C-ABI library; raises if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not path.exists():
            raise RuntimeError(
                f"rl_algo_impls_amd: HIP library {path} is missing; run __graft_entry__.build() "
                "(there is no CPU fallback for the product path)"
            )
        handle = C.CDLL(str(path))
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.rai_abi_version() != ABI_VERSION:
            raise RuntimeError("librai_amd ABI version mismatch")
        runtimes = hip_runtimes_mapped()
        if len(runtimes) > 1:
            raise RuntimeError(f"two HIP runtimes mapped in one process: {runtimes}")
        _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().rai_strerror(rc).decode()
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("rl_algo_impls_amd: device kernels require tensors on a HIP device")
