"""Diagnostic: device time per launch of rai_bias_relu_fwd / rai_bias_relu_bwd at the C3 (Pong
NatureCNN, minibatch 256) layer shapes, against torch's own elementwise kernels over the same bytes
(relu_, threshold_backward, copy_) as a yardstick, with the HBM bytes each launch must move.
HIP events on the stream the kernels run on.  Not part of the product or the tests.

    python tools/bias_relu_bench.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
L = _lib.lib()
st = _lib.stream_handle(dev)
SHAPES = [("conv1 256x20x20x32", 256 * 400, 32), ("conv2 256x9x9x64", 256 * 81, 64),
          ("conv3 256x7x7x64", 256 * 49, 64), ("fc 256x512", 256, 512)]
REPS = 200


def timed(fn):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


tot = {}
for name, rows, C in SHAPES:
    g = torch.Generator(device=dev).manual_seed(1)
    z = torch.randn(rows, C, device=dev, generator=g)
    dy = torch.randn(rows, C, device=dev, generator=g)
    b = torch.randn(C, device=dev, generator=g)
    y = torch.empty_like(z)
    dx = torch.empty_like(z)
    db = torch.zeros(C, device=dev)
    ws = torch.zeros(int(L.rai_bias_relu_workspace_bytes(C)), dtype=torch.uint8, device=dev)
    nb = z.numel() * 4
    fwd = timed(lambda: L.rai_bias_relu_fwd(z.data_ptr(), b.data_ptr(), rows, C, y.data_ptr(), st))
    bwd = timed(lambda: L.rai_bias_relu_bwd(dy.data_ptr(), y.data_ptr(), rows, C, dx.data_ptr(), db.data_ptr(), 1,
                                            ws.data_ptr(), ws.numel(), st))
    t_relu = timed(lambda: torch.clamp_min(z, 0.0, out=y))
    t_thr = timed(lambda: torch.ops.aten.threshold_backward.grad_input(dy, y, 0.0, grad_input=dx))
    t_copy = timed(lambda: dx.copy_(dy))
    print(f"{name:20s} {nb / 1e6:6.2f} MB/tensor | fwd {fwd:6.2f} us ({2 * nb / fwd / 1e3:6.0f} GB/s)  "
          f"bwd {bwd:6.2f} us ({3 * nb / bwd / 1e3:6.0f} GB/s) | torch clamp_min {t_relu:6.2f}  "
          f"threshold_backward {t_thr:6.2f}  copy_ {t_copy:6.2f} us", flush=True)
    for k, v in (("fwd", fwd), ("bwd", bwd), ("clamp_min", t_relu), ("threshold_backward", t_thr)):
        tot[k] = tot.get(k, 0.0) + v
print("per minibatch (4 layers): " + ", ".join(f"{k} {v:.1f} us" for k, v in tot.items()), flush=True)
