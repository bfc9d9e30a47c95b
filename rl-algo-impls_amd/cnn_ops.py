"""NatureCNN (config C3) layer epilogues on the GPU: conv / Linear -> bias + ReLU.

The reference encoder (rl_algo_impls/shared/encoder/nature_cnn.py:10-53, cnn.py:24-72) is
Conv2d -> ReLU x3, Flatten, Linear -> ReLU.  PyTorch-ROCm runs every layer as the MIOpen / hipBLASLt
contraction plus a bias add and a clamp, and its backward as threshold_backward, a bias-gradient
column sum and an accumulate of that gradient into .grad.  Here the contraction stays on
MIOpen / hipBLASLt (MFMA), bias-free, and the epilogue is one HIP pass each way
(rai_bias_relu_fwd / rai_bias_relu_bwd, csrc/se_block.hip):

    forward    y = relu(conv(x, W) + b)             conv bias-free, then one pass
    backward   dz = dy * (y > 0), db (+)= sum dz     one launch, deterministic order

Convolutions on hand-written MFMA kernels (round 3, csrc/conv.hip).  The forward of every NatureCNN
conv -> ReLU pair is ONE launch, rai_conv2d_bias_relu_fwd (f32 MFMA implicit GEMM, bias + ReLU in its
store, conv3 writing nn.Flatten's NCHW order directly), and the weight gradient is
rai_conv2d_wgrad (f32 MFMA, fixed-order split reduction) added straight into the flat .grad view.
The input gradient (conv2, conv3) is rai_conv2d_dgrad (f32 MFMA: per image, a GEMM over its output
pixels and a col2im in LDS).  Shapes those kernels do not take fall back to MIOpen (still on the GPU);
RAI_CONV_MFMA=0 selects MIOpen everywhere (same-box A/B).

Direct gradient accumulation.  Inside the trainer's update (`direct_grads(module)`), every
parameter's .grad is a view into the flat gradient buffer (optim.FlatParams), zeroed by the
optimizer step.  The bias gradient is then added by the backward kernel straight into that view,
and the Linear weight gradient by a beta = 1 GEMM (W.grad.addmm_(dz^T, x)), instead of autograd
materialising each gradient and launching an accumulate kernel per parameter.  Outside that
context the Functions return their gradients to autograd like any module (torch.autograd.grad
etc. see ordinary gradients).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading
import weakref
from typing import Dict

import torch
import torch.nn.functional as F

from . import _lib
from .dp_buckets import notify_grad_written

_state = threading.local()


@contextlib.contextmanager
def direct_grads(enabled: bool = True):
    """Within this context the fused epilogues accumulate parameter gradients in place (see the
    module docstring).  The trainer enters it around its own forward + backward only.

    The convolution weight gradients come back from MIOpen as fresh tensors; their accumulates into
    the flat gradient are deferred to the exit of this context and issued as ONE multi-tensor add
    (torch._foreach_add_) instead of an add launch per layer.  The list is handed to the backward
    through ctx (autograd runs CUDA backward nodes on its device thread, where this thread's
    state is not visible)."""
    prev = getattr(_state, "direct", False)
    prev_pending = getattr(_state, "pending", None)
    _state.direct = enabled
    pending = _PendingGrads()
    _state.pending = pending
    ok = False
    try:
        yield
        ok = True
    finally:
        _state.direct = prev
        _state.pending = prev_pending
        pending.close(flush=ok)


class _WgradJob(C.Structure):
    """rai_conv2d_wgrad_job (include/rai_amd.h)."""
    _fields_ = [("workspace", C.c_void_p), ("dw", C.c_void_p), ("db", C.c_void_p), ("B", C.c_int64), ("H", C.c_int32), ("W", C.c_int32),
                ("Ci", C.c_int32), ("Co", C.c_int32), ("KH", C.c_int32), ("KW", C.c_int32), ("stride", C.c_int32),
                ("reserved", C.c_int32)]


_MAX_JOBS = 4  # RAI_WGRAD_MAX_JOBS


# Weight-gradient partials on a side stream (round 4): a layer's partials depend only on its dz (or dy, y)
# and x, not on the input gradient the backward computes next, so they run beside the dgrad chain
# (conv3 wgrad || conv3 dgrad -> conv2 dgrad, conv2 wgrad || ...) instead of after it; the reduction joins
# the side stream first.  Inside a graph capture the fork and join are captured edges.  The operands are
# kept referenced by the pending job until that join, so the caching allocator cannot hand their memory
# to later work on the main stream while the side stream still reads it.  RAI_WGRAD_OVERLAP=0: in order.
# Measured SLOWER on C3 (161k vs 169k env-steps/s with it off, same box: profiles/r4j_ab_c3_wgrad_overlap.txt):
# the weight-gradient and input-gradient kernels each fill the GPU, and the fork / join add dependencies to the
# captured step.  Off by default; RAI_WGRAD_OVERLAP=1 turns it on.
_WGRAD_OVERLAP = os.environ.get("RAI_WGRAD_OVERLAP", "0") == "1"
_SIDE: Dict[str, "torch.cuda.Stream"] = {}


def _side_stream(device):
    """The device's weight-gradient side stream (created outside any capture), or None."""
    if not _WGRAD_OVERLAP or torch.device(device).type != "cuda":
        return None
    k = str(device)
    s = _SIDE.get(k)
    if s is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        s = torch.cuda.Stream(device)
        _SIDE[k] = s
    return s


def _join_side(device) -> None:
    s = _SIDE.get(str(device))
    if s is not None:
        torch.cuda.current_stream(device).wait_stream(s)


def _reduce_wgrad_jobs(jobs: list, device) -> None:
    """One rai_conv2d_wgrad_reduce launch per RAI_WGRAD_MAX_JOBS layers: each layer's partial tiles
    summed in a fixed order and added into its flat .grad view (after joining the side stream the
    partials ran on)."""
    _join_side(device)
    L = _lib.lib()
    for i in range(0, len(jobs), _MAX_JOBS):
        chunk = jobs[i:i + _MAX_JOBS]
        arr = (_WgradJob * len(chunk))(*[j[0] for j in chunk])
        _lib.check(L.rai_conv2d_wgrad_reduce(C.cast(arr, C.c_void_p), len(chunk), 1, _lib.stream_handle(device)),
                   "rai_conv2d_wgrad_reduce")
    for j in jobs:
        notify_grad_written(j[2])


class _PendingGrads:
    """Gradient accumulates deferred to the context's exit: (weight, gradient) pairs (one multi-tensor
    add) and MFMA weight-gradient partials (one reduction launch for the backward's convolutions).  A
    backward that runs after the context has closed (forward inside it, backward outside) accumulates
    its own at once."""

    def __init__(self):
        self.items: list = []
        self.jobs: list = []  # (rai_conv2d_wgrad_job, workspace tensor kept alive, weight)
        self.closed = False

    def add(self, w: torch.Tensor, dw: torch.Tensor) -> None:
        if self.closed:
            w.grad.add_(dw)
            notify_grad_written(w)
        else:
            self.items.append((w, dw))

    def add_wgrad(self, job: "_WgradJob", ws: torch.Tensor, w: torch.Tensor, keep=()) -> None:
        """keep: the partials' operands, referenced until the reduction has joined the side stream."""
        if self.closed:
            _reduce_wgrad_jobs([(job, ws, w, keep)], ws.device)
            return
        assert not any(ws is j[1] for j in self.jobs), "reserve(ws) before writing its partials"
        self.jobs.append((job, ws, w, keep))

    def reserve(self, ws: torch.Tensor) -> None:
        """Called BEFORE a weight-gradient partials launch writes `ws`: a job still pending on that
        workspace (the same layer run twice in one backward) is reduced first, while its partials are
        intact (stream order puts that reduction ahead of the overwrite)."""
        if not self.closed and any(ws is j[1] for j in self.jobs):
            self.flush_jobs()

    def flush_jobs(self) -> None:
        jobs, self.jobs = self.jobs, []
        if jobs:
            _reduce_wgrad_jobs(jobs, jobs[0][1].device)

    def close(self, flush: bool) -> None:
        self.closed = True
        if flush:
            self.flush_jobs()
        elif self.jobs:  # dropped unreduced: still join the side stream before their operands are released
            _join_side(self.jobs[0][1].device)
        self.jobs = []
        items, self.items = self.items, []
        if flush and items:
            torch._foreach_add_([w.grad for w, _ in items], [dw for _, dw in items])
            for w, _ in items:
                notify_grad_written(w)


def _direct(p: torch.Tensor, raw: bool = False) -> bool:
    """In-place accumulation applies: inside direct_grads() with a dense .grad (raw: a kernel writes
    it through its data pointer, so it must also be contiguous; conv weights stored channels_last
    are accumulated with Tensor.add_ instead)."""
    g = p.grad
    return getattr(_state, "direct", False) and g is not None and g.layout == torch.strided and (
        not raw or g.is_contiguous())


class _Workspaces:
    """Zeroed per-(layer, device) workspaces of rai_bias_relu_bwd (per-workgroup partial sums and
    an arrival counter the kernel re-arms): one allocation serves every eager call and graph replay
    of that layer.  Keyed weakly on the layer module itself, so a workspace is freed with its layer
    and a later module can never alias it (an id() key could be recycled after collection)."""

    def __init__(self):
        self._ws: "weakref.WeakKeyDictionary[torch.nn.Module, Dict[tuple, torch.Tensor]]" = \
            weakref.WeakKeyDictionary()

    def get(self, module: torch.nn.Module, C: int, device) -> torch.Tensor:
        per = self._ws.setdefault(module, {})
        k = (C, str(device))
        ws = per.get(k)
        if ws is None:
            # zeroed by an eager memset: one recorded into a graph capture would not run before the
            # first replay; every graphed step has eager warm-up runs that allocate it first
            if torch.device(device).type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("cnn_ops: bias + ReLU workspace first requested inside a graph capture")
            n = int(_lib.lib().rai_bias_relu_workspace_bytes(C))
            ws = torch.zeros(n, dtype=torch.uint8, device=device)
            per[k] = ws
        return ws

    def prewarm(self, module: torch.nn.Module, C: int, device) -> None:
        if torch.device(device).type != "cuda" or not torch.cuda.is_current_stream_capturing():
            self.get(module, C, device)


_WS = _Workspaces()

_CONV_MFMA = os.environ.get("RAI_CONV_MFMA", "1") != "0"
_FC_ADDMM_RELU = os.environ.get("RAI_FC_ADDMM_RELU", "1") != "0"  # +0.4 % C3 (r3zk)
_CONV_FUSE_RELU_BWD = os.environ.get("RAI_CONV_FUSE_RELU_BWD", "1") != "0"  # +0.45 % C3 (r3z)
# the per-image input-gradient kernel (round 4): conv2 26.8 vs MIOpen 33.2 us, conv3 21.0 vs 27.7 us at B = 256,
# C3 155.6-156.2k vs 150.9-152.9k env-steps/s same box (profiles/r4e_*); RAI_CONV_MFMA_DGRAD=0 restores MIOpen's dx
_CONV_MFMA_DGRAD = os.environ.get("RAI_CONV_MFMA_DGRAD", "1") == "1"
# the first layer on the uint8 frames (round 4): the gather writes the minibatch as uint8 NHWC and conv1's
# forward / weight gradient read x = u8 / range_size in-kernel (rai_conv2d_bias_relu_fwd_u8,
# rai_conv2d_wgrad_*partials_u8); RAI_CONV_U8=0 keeps the float32 prescale in the gather
_CONV_U8 = os.environ.get("RAI_CONV_U8", "1") == "1"


class _WgradWorkspaces:
    """rai_conv2d_wgrad's partial tiles per (layer, size): allocated outside graph capture (the
    graphed step's eager warm-up runs request it first), no zeroing needed."""

    def __init__(self):
        self._ws: "weakref.WeakKeyDictionary[torch.nn.Module, Dict[tuple, torch.Tensor]]" = \
            weakref.WeakKeyDictionary()

    def get(self, module: torch.nn.Module, nbytes: int, device) -> torch.Tensor:
        per = self._ws.setdefault(module, {})
        k = (nbytes, str(device))
        ws = per.get(k)
        if ws is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("cnn_ops: convolution weight-gradient workspace first requested inside a graph "
                                   "capture")
            ws = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
            per[k] = ws
        return ws


_WG_WS = _WgradWorkspaces()


def _mfma_conv_ok(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, stride, padding) -> bool:
    """The shapes and layouts csrc/conv.hip takes: NHWC fp32 input, channels_last weight, no padding,
    Ci % 4 == 0, Co 32 / 64, KH * KW * Ci % 64 == 0, 16-B aligned pointers; or a uint8 NHWC input with
    Ci == 4 (4-B aligned, under 2^31 bytes: the _u8 kernels)."""
    if not _CONV_MFMA or tuple(_pair(padding)) != (0, 0):
        return False
    Co, Ci, KH, KW = (int(v) for v in w.shape)
    # operand shapes must agree (the kernels take Ci, H, W from x): mismatches go to F.conv2d, which raises
    if x.dim() != 4 or int(x.shape[1]) != Ci or int(x.shape[2]) < KH or int(x.shape[3]) < KW:
        return False
    if x.dtype == torch.uint8:
        x_ok = (Ci == 4 and x.data_ptr() % 4 == 0 and x.numel() < 2 ** 31)
    else:
        x_ok = x.dtype == torch.float32 and x.data_ptr() % 16 == 0
    return (x_ok and x.is_contiguous(memory_format=torch.channels_last)
            and w.is_contiguous(memory_format=torch.channels_last) and Ci % 4 == 0 and Co in (32, 64)
            and (KH * KW * Ci) % 64 == 0 and KH * KW * Ci <= 8192 and b.is_contiguous()
            and all(t.data_ptr() % 16 == 0 for t in (w, b)))


def _u8_to_f32(x: torch.Tensor, x_div: float) -> torch.Tensor:
    """x.float() / x_div, channels_last: IEEE division by a device scalar (as the gather's prescale; a
    Python-scalar divisor would be a multiply by the rounded reciprocal on the GPU)."""
    d = torch.full((), float(x_div), dtype=torch.float32, device=x.device)  # a fill kernel: graph-capturable
    return (x.float() / d).contiguous(memory_format=torch.channels_last)


def _conv_fwd_mfma(x, w, b, stride, flatten, x_div=None) -> torch.Tensor:
    B, Ci, H, W = (int(v) for v in x.shape)
    Co, _, KH, KW = (int(v) for v in w.shape)
    s = _pair(stride)[0]
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    if flatten:
        y = torch.empty((B, Co * OH * OW), dtype=torch.float32, device=x.device)
    else:
        y = torch.empty((B, Co, OH, OW), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    L = _lib.lib()
    if x.dtype == torch.uint8:
        _lib.check(L.rai_conv2d_bias_relu_fwd_u8(x.data_ptr(), float(x_div), w.data_ptr(), b.data_ptr(), B, H, W, Ci,
                                                 Co, KH, KW, s, 1 if flatten else 0, y.data_ptr(),
                                                 _lib.stream_handle(x.device)), "rai_conv2d_bias_relu_fwd_u8")
        return y
    nb = int(L.rai_conv2d_fwd_splitk_bytes(B, H, W, Ci, Co, KH, KW, s, 1 if flatten else 0))
    if nb > 0:  # split-K where the tiling leaves CUs idle (conv2 / conv3 at B = 256): partials + ordered sum
        part = torch.empty(nb // 4, dtype=torch.float32, device=x.device)
        _lib.check(L.rai_conv2d_bias_relu_fwd_splitk(x.data_ptr(), w.data_ptr(), b.data_ptr(), B, H, W, Ci, Co, KH, KW,
                                                     s, 1 if flatten else 0, y.data_ptr(), part.data_ptr(), nb,
                                                     _lib.stream_handle(x.device)), "rai_conv2d_bias_relu_fwd_splitk")
        return y
    _lib.check(L.rai_conv2d_bias_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), B, H, W, Ci, Co, KH,
                                          KW, s, 1 if flatten else 0, y.data_ptr(),
                                          _lib.stream_handle(x.device)), "rai_conv2d_bias_relu_fwd")
    return y


def _conv_dgrad(x, dz, w, stride) -> torch.Tensor:
    """dx of the convolution: rai_conv2d_dgrad (MFMA) where it applies (Ci 32 / 64, kernel a multiple of
    the stride), else MIOpen."""
    B, Ci, H, W = (int(v) for v in x.shape)
    Co, _, KH, KW = (int(v) for v in w.shape)
    s = _pair(stride)[0]
    if _CONV_MFMA_DGRAD and Ci in (32, 64) and Co % 16 == 0 and KH % s == 0 and KW % s == 0:
        dx = torch.empty((B, Ci, H, W), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
        rc = _lib.lib().rai_conv2d_dgrad(dz.data_ptr(), w.data_ptr(), B, H, W, Ci, Co, KH, KW, s, dx.data_ptr(),
                                         _lib.stream_handle(x.device))
        if rc != _lib.RAI_E_UNSUPPORTED:  # no instantiation for the shape: MIOpen below
            _lib.check(rc, "rai_conv2d_dgrad")
            return dx
    return torch.ops.aten.convolution_backward(dz, x, w, None, _pair(stride), [0, 0], [1, 1], False, [0, 0], 1,
                                               [True, False, False])[0]


def _conv_dgrad_relu(x, dy, y, w, stride):
    """dx with the layer's ReLU backward folded in (rai_conv2d_dgrad_relu: dz = y > 0 ? dy : 0 formed on the
    fly); None where that kernel has no instantiation for the shape (the caller then materialises dz)."""
    B, Ci, H, W = (int(v) for v in x.shape)
    Co, _, KH, KW = (int(v) for v in w.shape)
    s = _pair(stride)[0]
    if not (dy.is_contiguous(memory_format=torch.channels_last) and dy.data_ptr() % 16 == 0):
        return None
    dx = torch.empty((B, Ci, H, W), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    rc = _lib.lib().rai_conv2d_dgrad_relu(dy.data_ptr(), y.data_ptr(), w.data_ptr(), B, H, W, Ci, Co, KH, KW, s,
                                          dx.data_ptr(), _lib.stream_handle(x.device))
    if rc == _lib.RAI_E_UNSUPPORTED:
        return None
    _lib.check(rc, "rai_conv2d_dgrad_relu")
    return dx


def _conv_wgrad_partials(module, x, dz, w, stride, grad: torch.Tensor, pending: "_PendingGrads", y=None, db=None,
                         x_div=None):
    """rai_conv2d_wgrad_partials for this layer (with y: rai_conv2d_wgrad_relu_partials, dz being the ReLU
    output's gradient dy, and the bias gradient reduced into db; a uint8 x: the _u8 forms, x / x_div);
    returns (job, workspace) for the deferred reduction.  A reduction still pending on the layer's
    workspace runs first (pending.reserve)."""
    B, Ci, H, W = (int(v) for v in x.shape)
    Co, _, KH, KW = (int(v) for v in w.shape)
    s = _pair(stride)[0]
    L = _lib.lib()
    nb = int(L.rai_conv2d_wgrad_workspace_bytes(B, H, W, Ci, Co, KH, KW, s))
    ws = _WG_WS.get(module, nb, x.device)
    pending.reserve(ws)
    side = _side_stream(x.device) if pending is not None and not pending.closed else None
    if side is not None:  # fork: the side stream waits for everything queued so far (dz / dy, y, x)
        side.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(side):
            _launch_wgrad_partials(L, x, dz, y, x_div, B, H, W, Ci, Co, KH, KW, s, ws, nb)
    else:
        _launch_wgrad_partials(L, x, dz, y, x_div, B, H, W, Ci, Co, KH, KW, s, ws, nb)
    return _WgradJob(ws.data_ptr(), grad.data_ptr(), None if db is None else db.data_ptr(), B, H, W, Ci, Co, KH, KW,
                     s, 0), ws


def _launch_wgrad_partials(L, x, dz, y, x_div, B, H, W, Ci, Co, KH, KW, s, ws, nb) -> None:
    st = _lib.stream_handle(x.device)
    if x.dtype == torch.uint8 and y is None:
        _lib.check(L.rai_conv2d_wgrad_partials_u8(x.data_ptr(), float(x_div), dz.data_ptr(), B, H, W, Ci, Co, KH, KW,
                                                  s, ws.data_ptr(), nb, st), "rai_conv2d_wgrad_partials_u8")
    elif x.dtype == torch.uint8:
        _lib.check(L.rai_conv2d_wgrad_relu_partials_u8(dz.data_ptr(), y.data_ptr(), x.data_ptr(), float(x_div), B, H,
                                                       W, Ci, Co, KH, KW, s, ws.data_ptr(), nb, st),
                   "rai_conv2d_wgrad_relu_partials_u8")
    elif y is None:
        _lib.check(L.rai_conv2d_wgrad_partials(x.data_ptr(), dz.data_ptr(), B, H, W, Ci, Co, KH, KW, s, ws.data_ptr(),
                                               nb, st), "rai_conv2d_wgrad_partials")
    else:
        _lib.check(L.rai_conv2d_wgrad_relu_partials(dz.data_ptr(), y.data_ptr(), x.data_ptr(), B, H, W, Ci, Co, KH, KW,
                                                    s, ws.data_ptr(), nb, st), "rai_conv2d_wgrad_relu_partials")


def _conv_wgrad_mfma(module, x, dz, w, stride, out: torch.Tensor, accumulate: bool) -> None:
    B, Ci, H, W = (int(v) for v in x.shape)
    Co, _, KH, KW = (int(v) for v in w.shape)
    s = _pair(stride)[0]
    L = _lib.lib()
    nb = int(L.rai_conv2d_wgrad_workspace_bytes(B, H, W, Ci, Co, KH, KW, s))
    ws = _WG_WS.get(module, nb, x.device)
    _lib.check(L.rai_conv2d_wgrad(x.data_ptr(), dz.data_ptr(), B, H, W, Ci, Co, KH, KW, s, out.data_ptr(),
                                  1 if accumulate else 0, ws.data_ptr(), nb, _lib.stream_handle(x.device)),
               "rai_conv2d_wgrad")


def _bias_relu_fwd(z: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    C = int(z.shape[1])
    y = torch.empty_like(z)
    _lib.check(_lib.lib().rai_bias_relu_fwd(z.data_ptr(), b.data_ptr(), z.numel() // C, C, y.data_ptr(),
                                            _lib.stream_handle(z.device)), "rai_bias_relu_fwd")
    return y


def _bias_relu_fwd_nchw(z: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """z (B, C, H, W) channels_last -> relu(z + b) flattened in NCHW order (B, C*H*W)."""
    B, C, H, W = (int(v) for v in z.shape)
    y = torch.empty((B, C * H * W), dtype=z.dtype, device=z.device)
    _lib.check(_lib.lib().rai_bias_relu_fwd_nchw(z.data_ptr(), b.data_ptr(), B, H * W, C, y.data_ptr(),
                                                 _lib.stream_handle(z.device)), "rai_bias_relu_fwd_nchw")
    return y


def _bias_relu_bwd_nchw(dy: torch.Tensor, y: torch.Tensor, b: torch.Tensor, ws: torch.Tensor, direct: bool,
                        zshape):
    """dy, y (B, C*H*W) in NCHW order -> (dz (B, C, H, W) channels_last, db or None)."""
    B, C, H, W = zshape
    dz = torch.empty(zshape, dtype=y.dtype, device=y.device, memory_format=torch.channels_last)
    db = b.grad if direct else torch.empty(C, dtype=torch.float32, device=y.device)
    _lib.check(_lib.lib().rai_bias_relu_bwd_nchw(dy.data_ptr(), y.data_ptr(), B, H * W, C, dz.data_ptr(),
                                                 db.data_ptr(), 1 if direct else 0, ws.data_ptr(), ws.numel(),
                                                 _lib.stream_handle(y.device)), "rai_bias_relu_bwd_nchw")
    return dz, (None if direct else db)


def _bias_relu_bwd(dy: torch.Tensor, y: torch.Tensor, b: torch.Tensor, ws: torch.Tensor, direct: bool):
    """(dz, db or None): db is added into b.grad when direct."""
    C = int(y.shape[1])
    dz = torch.empty_like(y)
    db = b.grad if direct else torch.empty(C, dtype=torch.float32, device=y.device)
    _lib.check(_lib.lib().rai_bias_relu_bwd(dy.data_ptr(), y.data_ptr(), y.numel() // C, C, dz.data_ptr(),
                                            db.data_ptr(), 1 if direct else 0, ws.data_ptr(), ws.numel(),
                                            _lib.stream_handle(y.device)), "rai_bias_relu_bwd")
    return dz, (None if direct else db)


class ConvBiasReLU(torch.autograd.Function):
    """relu(conv2d(x, W) + b) on NHWC (channels_last) fp32 activations; with flatten, returned as
    torch.flatten(., 1) of it (NCHW order, (B, C*H*W)) by the transposing epilogue pair."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, key, flatten=False, x_div=None):
        mfma = _mfma_conv_ok(x, w, b, stride, padding) and len(set(_pair(stride))) == 1
        if x.dtype == torch.uint8 and not mfma:  # uint8 frames outside the _u8 kernels: the prescale here
            x = _u8_to_f32(x, x_div)
            mfma = _mfma_conv_ok(x, w, b, stride, padding) and len(set(_pair(stride))) == 1
        ctx.x_div = x_div
        if mfma:
            y = _conv_fwd_mfma(x, w, b, stride, flatten, x_div)
            B, _, H, W = x.shape
            s = _pair(stride)[0]
            zshape = (int(B), int(w.shape[0]), (int(H) - int(w.shape[2])) // s + 1, (int(W) - int(w.shape[3])) // s + 1)
        else:
            z = F.conv2d(x, w, None, stride, padding)
            z = z.contiguous(memory_format=torch.channels_last)
            y = _bias_relu_fwd_nchw(z, b) if flatten else _bias_relu_fwd(z, b)
            zshape = tuple(int(v) for v in z.shape)
        ctx.save_for_backward(x, w, b, y)
        ctx.conf = (stride, padding, key, _direct(b, raw=True), _direct(w), flatten, zshape, mfma)
        ctx.pending = _state.pending if ctx.conf[4] else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, y = ctx.saved_tensors
        stride, padding, key, direct_b, direct_w, flatten, zshape, mfma = ctx.conf
        u8 = x.dtype == torch.uint8  # (never needs an input gradient)
        if (mfma and _CONV_FUSE_RELU_BWD and not flatten and direct_b and direct_w
                and (not ctx.needs_input_grad[0] or _CONV_MFMA_DGRAD)
                and w.grad.is_contiguous(memory_format=torch.channels_last) and w.grad.data_ptr() % 16 == 0
                and b.grad.data_ptr() % 16 == 0 and y.is_contiguous(memory_format=torch.channels_last)):
            # the bias + ReLU backward folded into its consumers, dz never materialised: the weight-gradient
            # partials (with the bias gradient) and, where the input needs a gradient (conv2), the input
            # gradient form dz = y > 0 ? dy : 0 on the fly (conv1's input needs none)
            dy = dy.contiguous(memory_format=torch.channels_last)
            dx = None
            if ctx.needs_input_grad[0]:
                dx = _conv_dgrad_relu(x, dy, y, w, stride)
            if dx is not None or not ctx.needs_input_grad[0]:
                job, wsp = _conv_wgrad_partials(key, x, dy, w, stride, w.grad, ctx.pending, y=y, db=b.grad,
                                                x_div=ctx.x_div)
                ctx.pending.add_wgrad(job, wsp, w, keep=(x, dy, y))
                return dx, None, None, None, None, None, None, None
        ws = _WS.get(key, zshape[1], y.device)
        if flatten:
            dz, db = _bias_relu_bwd_nchw(dy.contiguous(), y, b, ws, direct_b, zshape)
        else:
            dy = dy.contiguous(memory_format=torch.channels_last)
            dz, db = _bias_relu_bwd(dy, y, b, ws, direct_b)
        need_dx = ctx.needs_input_grad[0]
        if u8 and not (mfma and direct_w and w.grad.is_contiguous(memory_format=torch.channels_last)
                       and w.grad.data_ptr() % 16 == 0 and dz.is_contiguous(memory_format=torch.channels_last)
                       and dz.data_ptr() % 16 == 0):
            x = _u8_to_f32(x, ctx.x_div)  # the float32 forms below (outside the trainer's direct gradients)
        if mfma and dz.is_contiguous(memory_format=torch.channels_last) and dz.data_ptr() % 16 == 0:
            dx = None
            if need_dx:
                dx = _conv_dgrad(x, dz, w, stride)
            g = w.grad
            if (direct_w and g.is_contiguous(memory_format=torch.channels_last) and g.data_ptr() % 16 == 0):
                # partial tiles now; their reduction into the flat .grad joins the other layers' in one
                # launch at direct_grads() exit
                job, ws = _conv_wgrad_partials(key, x, dz, w, stride, g, ctx.pending, x_div=ctx.x_div)
                ctx.pending.add_wgrad(job, ws, w, keep=(x, dz))
                dw = None
            else:
                dw = torch.empty_like(w, memory_format=torch.channels_last)
                _conv_wgrad_mfma(key, x, dz, w, stride, dw, accumulate=False)
                if direct_w:
                    ctx.pending.add(w, dw)
                    dw = None
            return dx, dw, db, None, None, None, None, None
        dx, dw, _ = torch.ops.aten.convolution_backward(dz, x, w, None, _pair(stride), _pair(padding), [1, 1],
                                                        False, [0, 0], 1, [need_dx, True, False])
        if direct_w:  # accumulated with the other layers' at direct_grads() exit
            ctx.pending.add(w, dw)
            dw = None
        return dx, dw, db, None, None, None, None, None


class LinearBiasReLU(torch.autograd.Function):
    """relu(x W^T + b) for (B, in) x: hipBLASLt GEMM, then the bias + ReLU pass."""

    @staticmethod
    def forward(ctx, x, w, b, key):
        if _FC_ADDMM_RELU:
            # the GEMM library's bias + ReLU epilogue (hipBLASLt; F.linear's addmm(b, x, W^T) then relu)
            y = torch._addmm_activation(b, x, w.t(), use_gelu=False)
        else:
            z = torch.mm(x, w.t())
            y = _bias_relu_fwd(z, b)
        ctx.save_for_backward(x, w, b, y)
        ctx.conf = (key, _direct(b, raw=True), _direct(w))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, y = ctx.saved_tensors
        key, direct_b, direct_w = ctx.conf
        dz, db = _bias_relu_bwd(dy.contiguous(), y, b, _WS.get(key, int(y.shape[1]), y.device), direct_b)
        dx = torch.mm(dz, w) if ctx.needs_input_grad[0] else None
        if direct_w:
            w.grad.addmm_(dz.t(), x)  # beta = 1: the GEMM accumulates into the flat gradient view
            dw = None
            notify_grad_written(w)  # data parallel: this layer's gradient bucket may go (dp_buckets)
        else:
            dw = torch.mm(dz.t(), x)
        return dx, dw, db, None


def _pair(v):
    return list(v) if isinstance(v, (tuple, list)) else [v, v]


_BRT_MAX_ELEMS = 8192  # csrc/se_block.hip BRT_MAX_ELEMS: (C + 1) * H * W of the transposing pair


def conv_relu(conv: torch.nn.Conv2d, x: torch.Tensor, flatten: bool = False, x_div=None) -> torch.Tensor:
    """relu(conv(x)) for an NHWC fp32 GPU activation (fused epilogue), else the module path.
    flatten: return torch.flatten(relu(conv(x)), 1) (NCHW order), transposed inside the epilogue.
    x_div: x is uint8 frames and the layer's input is x / x_div (the NatureCNN prescale)."""
    if x.dtype == torch.uint8 and (x_div is None or not x.is_cuda):
        if x_div is None:
            raise ValueError("conv_relu: a uint8 input needs its divisor (x_div)")
        x = x.float() / x_div  # CPU: IEEE division
        x_div = None
    if (x.is_cuda and (x.dtype == torch.float32 or x.dtype == torch.uint8) and x.dim() == 4 and conv.bias is not None and conv.groups == 1
            and tuple(conv.dilation) == (1, 1) and conv.padding_mode == "zeros" and isinstance(conv.padding, tuple)
            and conv.out_channels % 4 == 0 and 256 % (conv.out_channels // 4) == 0):
        if flatten:
            hw = 1
            for d in range(2):
                hw *= (int(x.shape[2 + d]) + 2 * conv.padding[d] - conv.kernel_size[d]) // conv.stride[d] + 1
            flatten = (conv.out_channels + 1) * hw <= _BRT_MAX_ELEMS
            if not flatten:
                return torch.flatten(conv_relu(conv, x, x_div=x_div), 1)
        _WS.prewarm(conv, conv.out_channels, x.device)
        return ConvBiasReLU.apply(x, conv.weight, conv.bias, tuple(conv.stride), tuple(conv.padding), conv,
                                  flatten, x_div)
    if x.dtype == torch.uint8:
        x = _u8_to_f32(x, x_div)
    y = F.relu(conv(x))
    return torch.flatten(y, 1) if flatten else y


def linear_relu(lin: torch.nn.Linear, x: torch.Tensor) -> torch.Tensor:
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and lin.bias is not None
            and lin.out_features % 4 == 0 and 256 % (lin.out_features // 4) == 0):
        _WS.prewarm(lin, lin.out_features, x.device)
        return LinearBiasReLU.apply(x.contiguous(), lin.weight, lin.bias, lin)
    return F.relu(lin(x))


class CategoricalCriticHeads(torch.autograd.Function):
    """(logp(a), entropy, v) of a Categorical actor head Linear(D, A) and a critic head Linear(D, 1)
    over the encoder output (rai_categorical_critic_heads_fwd / _bwd, csrc/heads.hip): one launch
    forward, two backward, in place of the heads' GEMMs, the Categorical kernels, the bias
    reductions and the gradient accumulates."""

    @staticmethod
    def forward(ctx, enc, wpi, bpi, wv, bv, actions):
        B, D = int(enc.shape[0]), int(enc.shape[1])
        A = int(wpi.shape[0])
        logits = torch.empty((B, A), dtype=torch.float32, device=enc.device)
        logp = torch.empty(B, dtype=torch.float32, device=enc.device)
        ent = torch.empty_like(logp)
        v = torch.empty_like(logp)
        _lib.check(_lib.lib().rai_categorical_critic_heads_fwd(
            enc.data_ptr(), wpi.data_ptr(), bpi.data_ptr(), wv.data_ptr(), bv.data_ptr(), actions.data_ptr(), B, D, A,
            logits.data_ptr(), logp.data_ptr(), ent.data_ptr(), v.data_ptr(), _lib.stream_handle(enc.device)),
            "rai_categorical_critic_heads_fwd")
        ctx.save_for_backward(enc, wpi, bpi, wv, bv, actions, logits)
        ctx.direct = all(_direct(p, raw=True) for p in (wpi, bpi, wv, bv))
        ctx.mark_non_differentiable(logits)
        return logp, ent, v

    @staticmethod
    def backward(ctx, d_logp, d_ent, d_v):
        enc, wpi, bpi, wv, bv, actions, logits = ctx.saved_tensors
        B, D, A = int(enc.shape[0]), int(enc.shape[1]), int(wpi.shape[0])
        dev = enc.device
        z = lambda t: t.contiguous() if t is not None else torch.zeros(B, dtype=torch.float32, device=dev)
        d_logp, d_ent, d_v = z(d_logp), z(d_ent), z(d_v)
        d_enc = torch.empty_like(enc)
        if ctx.direct:
            grads = (wpi.grad, bpi.grad, wv.grad, bv.grad)
        else:
            grads = tuple(torch.empty_like(p) for p in (wpi, bpi, wv, bv))
        L = _lib.lib()
        ws = torch.empty(int(L.rai_categorical_critic_heads_workspace_bytes(B, A)), dtype=torch.uint8, device=dev)
        _lib.check(L.rai_categorical_critic_heads_bwd(
            enc.data_ptr(), wpi.data_ptr(), bpi.data_ptr(), wv.data_ptr(), bv.data_ptr(), actions.data_ptr(),
            logits.data_ptr(), B, D, A, d_logp.data_ptr(), d_ent.data_ptr(), d_v.data_ptr(), d_enc.data_ptr(),
            *[g.data_ptr() for g in grads], 1 if ctx.direct else 0, ws.data_ptr(), ws.numel(),
            _lib.stream_handle(dev)), "rai_categorical_critic_heads_bwd")
        if ctx.direct:
            return d_enc, None, None, None, None, None
        return (d_enc,) + grads + (None,)


class FcReluHeads(torch.autograd.Function):
    """The fc layer -> ReLU and the Categorical + critic heads over its output as ONE autograd node
    (round 4): forward = the fc GEMM with its bias + ReLU epilogue, then rai_categorical_critic_heads_fwd;
    backward = rai_categorical_critic_heads_bwd_relu, which writes the fc's dz (its ReLU backward folded
    into the heads' input gradient) and the fc's bias gradient, then dx = dz W and W.grad += dz^T x.  One
    node, so no other consumer of the fc output can add an unmasked gradient behind the fold.  Used inside
    direct_grads() only (every parameter gradient accumulated in place)."""

    @staticmethod
    def forward(ctx, x, w, b, wpi, bpi, wv, bv, actions):
        if _FC_ADDMM_RELU:
            y = torch._addmm_activation(b, x, w.t(), use_gelu=False)
        else:
            y = _bias_relu_fwd(torch.mm(x, w.t()), b)
        B, D = int(y.shape[0]), int(y.shape[1])
        A = int(wpi.shape[0])
        logits = torch.empty((B, A), dtype=torch.float32, device=y.device)
        logp = torch.empty(B, dtype=torch.float32, device=y.device)
        ent = torch.empty_like(logp)
        v = torch.empty_like(logp)
        _lib.check(_lib.lib().rai_categorical_critic_heads_fwd(
            y.data_ptr(), wpi.data_ptr(), bpi.data_ptr(), wv.data_ptr(), bv.data_ptr(), actions.data_ptr(), B, D, A,
            logits.data_ptr(), logp.data_ptr(), ent.data_ptr(), v.data_ptr(), _lib.stream_handle(y.device)),
            "rai_categorical_critic_heads_fwd")
        ctx.save_for_backward(x, w, b, y, wpi, bpi, wv, bv, actions, logits)
        ctx.mark_non_differentiable(logits)
        return logp, ent, v

    @staticmethod
    def backward(ctx, d_logp, d_ent, d_v):
        x, w, b, y, wpi, bpi, wv, bv, actions, logits = ctx.saved_tensors
        B, D, A = int(y.shape[0]), int(y.shape[1]), int(wpi.shape[0])
        dev = y.device
        z = lambda t: t.contiguous() if t is not None else torch.zeros(B, dtype=torch.float32, device=dev)
        d_logp, d_ent, d_v = z(d_logp), z(d_ent), z(d_v)
        dz = torch.empty_like(y)
        L = _lib.lib()
        ws = torch.empty(int(L.rai_categorical_critic_heads_workspace_bytes(B, A)), dtype=torch.uint8, device=dev)
        _lib.check(L.rai_categorical_critic_heads_bwd_relu(
            y.data_ptr(), wpi.data_ptr(), bpi.data_ptr(), wv.data_ptr(), bv.data_ptr(), actions.data_ptr(),
            logits.data_ptr(), B, D, A, d_logp.data_ptr(), d_ent.data_ptr(), d_v.data_ptr(), dz.data_ptr(),
            wpi.grad.data_ptr(), bpi.grad.data_ptr(), wv.grad.data_ptr(), bv.grad.data_ptr(), b.grad.data_ptr(), 1,
            ws.data_ptr(), ws.numel(), _lib.stream_handle(dev)), "rai_categorical_critic_heads_bwd_relu")
        dx = torch.mm(dz, w) if ctx.needs_input_grad[0] else None
        w.grad.addmm_(dz.t(), x)  # beta = 1: the GEMM accumulates into the flat gradient view
        notify_grad_written(w)  # data parallel: this layer's gradient bucket may go (dp_buckets)
        return dx, None, None, None, None, None, None, None


# the fc ReLU backward folded into the heads' backward (FcReluHeads); RAI_FC_HEADS_FOLD=0: separate nodes
_FC_HEADS_FOLD = os.environ.get("RAI_FC_HEADS_FOLD", "1") == "1"


def fc_relu_heads_fusable(network, lin: torch.nn.Linear, x: torch.Tensor, action_masks) -> bool:
    """FcReluHeads applies: the heads are fusable over the fc output, the fc is a GPU fp32 Linear with a
    bias, and every parameter involved accumulates its gradient in place (inside direct_grads())."""
    if not (_FC_HEADS_FOLD and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and lin.bias is not None
            and int(x.shape[1]) == lin.in_features):
        return False
    if not _heads_ok(network, action_masks):
        return False
    params = [lin.bias, network._pi._fc[0].weight, network._pi._fc[0].bias, network._v._fc[0][0].weight,
              network._v._fc[0][0].bias]
    return (all(_direct(p, raw=True) for p in params) and _direct(lin.weight)
            and lin.weight.grad.is_contiguous())


def fc_relu_heads(network, lin: torch.nn.Linear, x: torch.Tensor, actions: torch.Tensor):
    lin_pi = network._pi._fc[0]
    lin_v = network._v._fc[0][0]
    return FcReluHeads.apply(x.contiguous(), lin.weight, lin.bias, lin_pi.weight, lin_pi.bias, lin_v.weight,
                             lin_v.bias, actions.long().contiguous())


def heads_fusable(network, enc: torch.Tensor, action_masks) -> bool:
    """A ConnectedTrio network whose actor head is Categorical Linear(D, A) and critic head
    Linear(D, 1), no hidden layers, no action masks, fp32 on the GPU (the NatureCNN policy)."""
    return enc.is_cuda and enc.dtype == torch.float32 and enc.dim() == 2 and _heads_ok(network, action_masks)


def _heads_ok(network, action_masks) -> bool:
    from .policy import CategoricalActorHead

    pi = network._pi
    if not (action_masks is None and isinstance(pi, CategoricalActorHead) and network.pi_hidden_sizes == ()
            and network.v_hidden_sizes == ()):
        return False
    A = pi.act_dim
    return (2 <= A <= 10 or A == 12) and isinstance(pi._fc[0], torch.nn.Linear)


def categorical_critic_heads(network, enc: torch.Tensor, actions: torch.Tensor):
    lin_pi = network._pi._fc[0]
    lin_v = network._v._fc[0][0]
    return CategoricalCriticHeads.apply(enc.contiguous(), lin_pi.weight, lin_pi.bias, lin_v.weight,
                                        lin_v.bias, actions.long().contiguous())
