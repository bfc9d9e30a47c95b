"""Bucketed gradient all-reduce overlapped with the backward pass (SURVEY.md 8(e) "Overlap").

Data parallel PPO sums every optimizer step's gradient over the ranks (rl_algo_impls/ppo/ppo.py:375,
441-447: backward -> clip_grad_norm_ -> Adam).  The next minibatch's forward reads the updated
weights, so the exchange cannot overlap the NEXT forward; it can overlap the rest of the CURRENT
backward.  The flat gradient buffer (optim.FlatParams, parameters() order) is cut into buckets of
contiguous parameters.  As soon as the backward has written a bucket's last gradient, the bucket's
sum all-reduce is enqueued on a side stream (an event orders it after the writes on the compute
stream) while the compute stream continues with the earlier layers' backward; after the backward
the compute stream waits for the side stream.

NatureCNN (config C3, 6,750,876 gradient bytes): parameters() order is conv1, conv2, conv3, fc,
policy head, value head, and the backward produces them in reverse.  Bucket 1 = fc + heads
(6.43 MB, 95 % of the bytes) is complete when the fc layer's backward (cnn_ops.LinearBiasReLU, whose
weight gradient is a beta = 1 GEMM into the flat buffer) has run: the heads' AccumulateGrad nodes
run before it (autograd gives AccumulateGrad the highest priority, and the fc node needs both
heads' input gradients first).  Its all-reduce then overlaps the three convolutions' backward,
which is most of the backward's time.  Bucket 0 = the convolutions (0.31 MB) goes after the
backward.

The collective is our own RCCL communicator (rai_dp_allreduce_sum_f32, csrc/dp.hip), so the whole
minibatch step — gather, forward, loss, backward with the side-stream all-reduces, join — is
captured into one hipGraph and replayed (graphs.py).  With torch.distributed gloo (CPU tests) the
same buckets are summed after the backward instead.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch


class _Hooks:
    """The armed trigger callback.  Process-wide, not thread-local: autograd runs the backward of
    CUDA nodes on its per-device worker thread, not on the thread that called backward() (a
    thread-local hook armed by begin() is invisible there, and every bucket then waited for
    finish())."""
    cb: Optional[Callable[[torch.Tensor], None]] = None


_hooks = _Hooks()


def notify_grad_written(param: torch.Tensor) -> None:
    """Called by the fused layer backwards (cnn_ops) right after they wrote `param`'s gradient."""
    cb = _hooks.cb
    if cb is not None:
        cb(param)


class GradBuckets:
    """Buckets of the flat gradient and their stream-ordered all-reduce launches."""

    def __init__(self, flat, bounds: List[int], triggers: Dict[int, int], allreduce: Callable[[torch.Tensor], None],
                 device: torch.device, overlap: bool = True):
        """bounds: flat offsets [0, b1, ..., P] (bucket i = [bounds[i], bounds[i+1]));
        triggers: id(param) -> bucket index launched when that parameter's gradient is written;
        allreduce(view): enqueue an in-place sum all-reduce of `view` on the CURRENT stream."""
        assert bounds[0] == 0 and bounds[-1] == flat.P
        self.flat = flat
        self.bounds = bounds
        self.triggers = triggers
        self.allreduce = allreduce
        self.overlap = overlap and flat.grad.is_cuda
        self.side = torch.cuda.Stream(device) if self.overlap else None
        self.launched: List[bool] = []
        self.early_launches = 0  # buckets launched by a trigger, i.e. inside the backward

    @property
    def n(self) -> int:
        return len(self.bounds) - 1

    def view(self, i: int) -> torch.Tensor:
        return self.flat.grad[self.bounds[i]:self.bounds[i + 1]]

    def _launch(self, i: int) -> None:
        if self.launched[i]:
            return
        self.launched[i] = True
        if not self.overlap:
            self.allreduce(self.view(i))
            return
        cur = torch.cuda.current_stream(self.flat.grad.device)
        self.side.wait_stream(cur)  # the bucket's gradients are written (stream order)
        with torch.cuda.stream(self.side):
            self.allreduce(self.view(i))

    def _on_written(self, param: torch.Tensor) -> None:
        i = self.triggers.get(id(param))
        if i is not None and not self.launched[i]:
            self.early_launches += 1
            self._launch(i)

    def begin(self) -> None:
        """Before the backward: arm the triggers."""
        self.launched = [False] * self.n
        if self.overlap:
            _hooks.cb = self._on_written

    def finish(self, scale: Optional[float] = None) -> None:
        """After the backward: the remaining buckets, then the compute stream waits for them."""
        _hooks.cb = None
        for i in range(self.n - 1, -1, -1):
            self._launch(i)
        if self.overlap:
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(self.side)
        if scale is not None:
            self.flat.grad.mul_(scale)


def nature_cnn_buckets(policy, flat) -> Optional[tuple]:
    """(bounds, triggers) for a NatureCNN ActorCritic: bucket 0 = the convolutions, bucket 1 = fc +
    heads triggered by the fc weight's gradient.  None for other policies (one bucket)."""
    try:
        enc = policy.network._feature_extractor.feature_extractor
        fc_w = enc.fc[1].weight
    except AttributeError:
        return None
    params = flat.params
    idx = next((k for k, p in enumerate(params) if p is fc_w), None)
    if idx is None:
        return None
    return [0, flat.offsets[idx], flat.P], {id(fc_w): 1}
