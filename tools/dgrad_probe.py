"""Diagnostic: time rai_conv2d_dgrad_v alone at the NatureCNN conv2 / conv3 input-gradient shapes
(B = 256), for A/B builds (RAI_AMD_LIB) and rocprofv3 counter passes.  Not part of the product or tests.

    python tools/dgrad_probe.py [--variants 3,4] [--reps 200]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from rl_algo_impls_amd import _lib  # noqa: E402

SHAPES = {"conv2": (32, 20, 64, 4, 2), "conv3": (64, 9, 64, 3, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="3,4")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--B", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    st = _lib.stream_handle(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    out = {}
    for name, (Ci, H, Co, k, s) in SHAPES.items():
        B = args.B
        OH = (H - k) // s + 1
        dz = torch.randn(B, Co, OH, OH, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        w = torch.randn(Co, Ci, k, k, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        x = torch.empty(B, Ci, H, H, device=dev).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        ref = torch.ops.aten.convolution_backward(dz, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                  [True, False, False])[0]
        for v in (int(t) for t in args.variants.split(",")):
            run = lambda: L.rai_conv2d_dgrad_v(dz.data_ptr(), w.data_ptr(), B, H, H, Ci, Co, k, k, s, dx.data_ptr(),
                                               v, st)
            dx.fill_(float("nan"))
            assert run() == 0
            torch.cuda.synchronize()
            err = float((dx - ref).abs().max() / ref.abs().max())
            for _ in range(10):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(20_000_000)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            flops = 2.0 * B * OH * OH * Co * k * k * Ci
            out[f"{name}_v{v}"] = {"us": round(us, 2), "tflops_useful": round(flops / us / 1e6, 1),
                                   "relerr_vs_miopen": err}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
