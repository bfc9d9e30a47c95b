"""Standalone repro for the C3 FETCH_SIZE crash (profiles/r2o_pong_fetch_pmc_crash.txt): NatureCNN's
three convolutions alone -- plain torch.nn.functional.conv2d on channels_last fp32 at the C3 minibatch
shape (B = 256, 4x84x84 -> 32x20x20 -> 64x9x9 -> 64x7x7), forward + backward, MIOpen find mode as in
bench.py -- with no rl_algo_impls_amd code loaded.  Run under `rocprofv3 --pmc FETCH_SIZE`: if it
faults the same way, the fault is in the profiler's handling of MIOpen's module-launched kernels,
not in this repository's kernels or launches.

    rocprofv3 --pmc FETCH_SIZE -d out -o run -- python3 tools/miopen_pmc_repro.py [--no-find] [--iters N]
"""
import argparse
import faulthandler
import os
import sys

import torch
import torch.nn.functional as F


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--no-find", action="store_true", help="MIOpen immediate mode instead of find mode")
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--diag", default=os.environ.get("RAI_DIAG_DIR"))
    args = p.parse_args()
    if args.diag:
        os.makedirs(args.diag, exist_ok=True)
        fh = open(os.path.join(args.diag, f"repro_faulthandler_{os.getpid()}.txt"), "w")
        faulthandler.enable(file=fh, all_threads=True)
    torch.backends.cudnn.benchmark = not args.no_find
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    cl = torch.channels_last
    x = (torch.rand(256, 4, 84, 84, generator=g) * 255).floor().div(255).to(dev).contiguous(memory_format=cl)
    ws = [torch.randn(32, 4, 8, 8, generator=g), torch.randn(64, 32, 4, 4, generator=g),
          torch.randn(64, 64, 3, 3, generator=g)]
    ws = [(w * 0.05).to(dev).contiguous(memory_format=cl).requires_grad_() for w in ws]
    strides = [4, 2, 1]
    if args.diag:
        with open("/proc/self/maps") as src, open(os.path.join(args.diag, f"repro_maps_{os.getpid()}.txt"), "w") as d:
            d.write(src.read())
    for it in range(args.iters):
        h = x
        for w, s in zip(ws, strides):
            h = F.relu(F.conv2d(h, w, None, s))
        h.sum().backward()
        torch.cuda.synchronize()
        print(f"iteration {it}: ok", flush=True)
    print("done", file=sys.stderr)


if __name__ == "__main__":
    main()
