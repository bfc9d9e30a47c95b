"""HIP-graph replay of the generic per-minibatch update (policies the fused epoch kernels do not
cover: NatureCNN, Gaussian / 256-wide MLPs, A2C).

The reference runs one eager minibatch step per Python iteration (rl_algo_impls/ppo/ppo.py:
290-411): ~100 small launches (forward, loss, autograd backward, clip + Adam) whose host launch
cost exceeds their GPU time at these batch sizes.  Here the step is captured ONCE into a hipGraph
(torch.cuda.CUDAGraph) and replayed for every minibatch of every epoch:

    rai_gather_minibatch_x rows perm[mb*B + i] of every rollout field -> static minibatch
                           buffers (uint8 frames -> float32 / range_size, channels_last, for the
                           NatureCNN); the last workgroup to finish advances mb (device counter)
    policy forward         PyTorch-ROCm (MIOpen / hipBLASLt), static inputs
    rai_ppo_loss           loss + dLoss/d(logp, entropy, v), stats row at state.stat_index
    autograd backward      into the flat .grad buffer
    rai_clip_optim_step    clip_grad_norm_ + Adam/RMSprop (omitted under data parallel or
                           gradient accumulation: the all-reduce / epoch step stays eager)

Everything a replay needs to vary lives in device memory: the minibatch index (descriptor), the
hyperparameters and train state (stat_index, opt_step, kl latch), so a replay takes no host
input.  Per update the host writes the descriptor once (rollout field pointers) and per epoch
copies the permutation into a persistent buffer and zeroes the counter.

The first minibatches of the first update run eagerly on the capture stream (warm-up: lazy
library handles, autograd stream state), the capture itself executes nothing, and a ragged tail
minibatch always runs eagerly through the same gather with its own buffers.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import _lib

_DESC_MB_OFFSET = _lib.MinibatchDesc.mb.offset


class MinibatchStepGraph:
    """Static buffers + captured graph for one (batch_size, field layout) of one trainer."""

    WARMUP = 2

    def __init__(self, device: torch.device, fields: List[torch.Tensor], batch_size: int,
                 xforms: Optional[list] = None):
        # no reference to the step function (it closes over the trainer): the trainer owns the
        # graphs, so dropping the trainer frees them at once instead of in a later cyclic GC pass
        self.device = device
        self.B = int(batch_size)
        self.row_bytes = [int(f[0].numel() * f.element_size()) for f in fields]
        self.xforms = xforms
        self.static = static_buffers(fields, self.B, device, xforms)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.eager_runs = 0
        # RAI_GRAPH_EAGER=1 (diagnostic): the same step body, launched eagerly and never captured --
        # for profilers that cannot follow graph launches (rocprofv3 counter collection segfaults on
        # graph-replayed dispatches: profiles/r3c_pong_fetch_pmc_crash_mapped.txt)
        self.eager_only = os.environ.get("RAI_GRAPH_EAGER") == "1"

    def gather(self, desc: torch.Tensor, bufs: List[torch.Tensor]) -> None:
        gather_next(self.device, desc, bufs, self.row_bytes, self.xforms)

    def _body(self, desc: torch.Tensor, step: Callable[[List[torch.Tensor]], None]) -> None:
        self.gather(desc, self.static)
        step(self.static)

    def run(self, desc: torch.Tensor, stream: torch.cuda.Stream, step: Callable[[List[torch.Tensor]], None]) -> None:
        """One minibatch on `stream` (the caller has made it current); `step` runs the minibatch's
        forward / loss / backward / optimizer on the static buffers (eager warm-up and capture)."""
        if self.graph is not None:
            self.graph.replay()
            return
        if self.eager_only or self.eager_runs < self.WARMUP:
            self._body(desc, step)
            self.eager_runs += 1
            return
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            self._body(desc, step)
        self.graph = g
        g.replay()  # the capture executed nothing: this replay is the minibatch


def static_buffers(fields: List[torch.Tensor], rows: int, device, xforms: Optional[list]) -> List[torch.Tensor]:
    """Minibatch destination buffers: the fields' own row shape and dtype, except a transformed
    frame field: float32 channels_last (RAI_XFORM_U8_CHW_TO_F32_HWC) or uint8 channels_last
    (RAI_XFORM_U8_CHW_TO_U8_HWC)."""
    out = []
    for i, f in enumerate(fields):
        x = xforms[i] if xforms is not None else None
        if x is not None and x.kind in (_lib.RAI_XFORM_U8_CHW_TO_F32_HWC, _lib.RAI_XFORM_U8_CHW_TO_U8_HWC):
            dt = torch.float32 if x.kind == _lib.RAI_XFORM_U8_CHW_TO_F32_HWC else torch.uint8
            out.append(torch.empty((rows,) + tuple(f.shape[1:]), dtype=dt, device=device,
                                   memory_format=torch.channels_last))
        else:
            out.append(torch.empty((rows,) + tuple(f.shape[1:]), dtype=f.dtype, device=device))
    return out


def gather_next(device, desc: torch.Tensor, bufs: List[torch.Tensor], row_bytes: List[int],
                xforms: Optional[list]) -> None:
    """rai_gather_minibatch_x (advance): rows of the next minibatch into bufs."""
    n = len(bufs)
    dst = (C.c_void_p * n)(*[b.data_ptr() for b in bufs])
    rb = (C.c_int64 * n)(*row_bytes)
    xf = None
    if xforms is not None:
        arr = (_lib.GatherXform * n)()
        for i, x in enumerate(xforms):
            arr[i] = x if x is not None else _lib.GatherXform(kind=_lib.RAI_XFORM_COPY)
        xf = C.cast(arr, C.c_void_p)
    _lib.check(_lib.lib().rai_gather_minibatch_x(desc.data_ptr(), n, C.cast(dst, C.c_void_p), C.cast(rb, C.c_void_p),
                                                 xf, int(bufs[0].shape[0]), 1, _lib.stream_handle(device)),
               "rai_gather_minibatch_x")


class GraphedUpdate:
    """Per-trainer cache of minibatch graphs and the device descriptor."""

    def __init__(self, device: torch.device):
        self.device = device
        self.stream = torch.cuda.Stream(device)
        self.desc = torch.zeros(C.sizeof(_lib.MinibatchDesc), dtype=torch.uint8, device=device)
        self.graphs: Dict[Tuple, MinibatchStepGraph] = {}
        self.perm: Optional[torch.Tensor] = None
        self._tail_bufs: Dict[Tuple, List[torch.Tensor]] = {}

    def key(self, fields: List[torch.Tensor], B: int, tag, xforms=None) -> Tuple:
        xk = tuple((x.kind, x.channels, x.hw, x.divisor) if x is not None else None for x in xforms) if xforms else None
        return (B, tag, xk) + tuple((f.dtype, tuple(f.shape[1:])) for f in fields)

    def set_rollout(self, fields: List[torch.Tensor], batch_size: int, shuffle: bool) -> None:
        n = int(fields[0].shape[0])
        if shuffle and (self.perm is None or self.perm.numel() != n):
            self.perm = torch.empty(n, dtype=torch.int64, device=self.device)
        d = _lib.MinibatchDesc()
        for i, f in enumerate(fields):
            assert f.is_contiguous() and f.shape[0] == n
            d.src[i] = f.data_ptr()
            d.row_bytes[i] = int(f[0].numel() * f.element_size())
        d.perm = self.perm.data_ptr() if shuffle else None
        d.n_rows, d.batch_size, d.mb, d.n_fields = n, int(batch_size), 0, len(fields)
        raw = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8)
        self.desc.copy_(raw, non_blocking=False)

    def start_epoch(self, perm: Optional[torch.Tensor]) -> None:
        if perm is not None:
            self.perm.copy_(perm, non_blocking=True)
        self.desc[_DESC_MB_OFFSET:_DESC_MB_OFFSET + 8].view(torch.int64).zero_()

    def graph_for(self, fields: List[torch.Tensor], B: int, tag, xforms=None) -> MinibatchStepGraph:
        k = self.key(fields, B, tag, xforms)
        g = self.graphs.get(k)
        if g is None:
            g = MinibatchStepGraph(self.device, fields, B, xforms)
            self.graphs[k] = g
        return g

    def tail(self, fields: List[torch.Tensor], rows: int, step, xforms=None) -> None:
        """Eager ragged last minibatch through the same device gather."""
        k = self.key(fields, rows, "tail", xforms)
        bufs = self._tail_bufs.get(k)
        if bufs is None:
            bufs = static_buffers(fields, rows, self.device, xforms)
            self._tail_bufs[k] = bufs
        gather_next(self.device, self.desc, bufs, [int(f[0].numel() * f.element_size()) for f in fields], xforms)
        step(bufs)
