"""GAE kernel microbenchmark: algorithmic GB/s at the BASELINE shapes and in the
bandwidth regime (HIP events on the launch stream around back-to-back launches queued behind a
spin, so the per-launch figure is kernel time plus the kernel-boundary gap)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd.gae import EXACT, FAST, compute_advantages_device  # noqa: E402

import os  # noqa: E402

dev = torch.device("cuda", 0)
# kernel variants for the bandwidth-regime shapes: the tiled kernel (RAI_GAE_STREAM=0) and the
# streaming kernel at 8 / 4 rows in flight per chunk (RAI_GAE_STREAM_D); GAE_BENCH_VARIANTS=0: default only
VARIANTS = [("default", {})]
if os.environ.get("GAE_BENCH_VARIANTS", "1") != "0":
    VARIANTS += [("tiled", {"RAI_GAE_STREAM": "0"}), ("stream_d8", {"RAI_GAE_STREAM_D": "8", "RAI_GAE_STREAM_NT": "256"}),
                 ("stream_d4", {"RAI_GAE_STREAM_D": "4", "RAI_GAE_STREAM_NT": "256"}), ("stream_512", {"RAI_GAE_STREAM_NT": "512"}),
                 ("stream_1k_plain", {"RAI_GAE_STREAM_NT": "1024", "RAI_GAE_NT": "0"}),
                 ("stream_1k_nt", {"RAI_GAE_STREAM_NT": "1024"})]
CASES = [(128, 4096, 1), (512, 2048, 1), (128, 1024, 1), (512, 512, 3), (128, 1 << 20, 1), (512, 1 << 18, 3)]
for (T, N, K, vname, venv) in [c + v for c in CASES for v in (VARIANTS if c[1] >= (1 << 18) else VARIANTS[:1])]:
    for k in ("RAI_GAE_STREAM", "RAI_GAE_STREAM_D", "RAI_GAE_STREAM_NT", "RAI_GAE_NT"):
        os.environ.pop(k, None)
    os.environ.update(venv)
    shp = (T, N) if K == 1 else (T, N, K)
    r = torch.randn(shp, device=dev)
    v = torch.randn(shp, device=dev)
    es = torch.rand((T, N), device=dev) < 0.01
    nes = torch.rand(N, device=dev) < 0.01
    nv = torch.randn(shp[1:], device=dev)
    adv = torch.empty_like(v)
    ret = torch.empty_like(v)
    g = 0.99 if K == 1 else __import__("numpy").array([0.99, 0.995, 0.999])
    byts = 16 * T * N * K + T * N + 4 * N * K + N
    # fast: the chunked affine scan where it applies; fast_serial: the serial fp32 chain (RAI_GAE_SCAN=0)
    for mode, name, scan in ((EXACT, "exact", "1"), (FAST, "fast", "1"), (FAST, "fast_serial", "0")):
        os.environ["RAI_GAE_SCAN"] = scan
        for _ in range(5):
            compute_advantages_device(r, v, es, nes, nv, g, 0.95, mode=mode, advantages_out=adv, returns_out=ret)
        reps = 200
        torch.cuda.synchronize()
        # park the stream behind a spin so every launch is queued before the GPU reaches it: the
        # event pair then times back-to-back kernels, not the Python launch gap (as bench.py)
        torch.cuda._sleep(50_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            compute_advantages_device(r, v, es, nes, nv, g, 0.95, mode=mode, advantages_out=adv, returns_out=ret)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        print(f"T={T:4d} N={N:8d} K={K} {vname:9s} {name:11s}: {us:9.2f} us  {byts / us / 1e3:8.1f} GB/s  "
              f"({100 * byts / us / 1e3 / 8000:.1f}% of 8 TB/s)", flush=True)
