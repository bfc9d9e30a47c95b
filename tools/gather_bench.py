"""Diagnostic: device time of the minibatch gather (rai_gather_minibatch_x) at the C3 shape (uint8
4x84x84 frames -> float NHWC / 255, plus the copied fields, B = 256 rows of a 131,072-row rollout),
HIP events over whole epochs of launches.  (Round 2 compared one, two and four workgroups per row
with a diagnostic switch since removed: profiles/r2zh_*, r2zi_*.)  Not part of the product or the tests.

    python tools/gather_bench.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd import _lib  # noqa: E402
from rl_algo_impls_amd.graphs import GraphedUpdate, gather_next, static_buffers  # noqa: E402

dev = torch.device("cuda", 0)
n, B = 131072, 256
g = torch.Generator(device="cpu").manual_seed(1)
fields = [torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev),
          torch.randint(0, 6, (n,), device=dev), torch.randn(n, device=dev), torch.randn(n, device=dev),
          torch.randn(n, device=dev), torch.randn(n, device=dev)]
xf = _lib.GatherXform(kind=_lib.RAI_XFORM_U8_CHW_TO_F32_HWC, channels=4, hw=84 * 84, divisor=255.0)
xforms = [xf] + [None] * 5
row_bytes = [int(f[0].numel() * f.element_size()) for f in fields]
gu = GraphedUpdate(dev)
gu.set_rollout(fields, B, True)
bufs = static_buffers(fields, B, dev, xforms)
nmb = n // B
times = []
for rep in range(3):
    gu.start_epoch(torch.randperm(n, generator=g).to(dev))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(nmb):
        gather_next(dev, gu.desc, bufs, row_bytes, xforms)
    e1.record()
    e1.synchronize()
    times.append(e0.elapsed_time(e1) * 1e3 / nmb)
mb_bytes = B * (4 * 84 * 84 * (1 + 4) + 8 + 4 * 4 + 8)
print(f"gather: {min(times):.2f} us per minibatch "
      f"(min of {len(times)} epochs of {nmb}), {mb_bytes / min(times) / 1e3:.0f} GB/s", flush=True)
