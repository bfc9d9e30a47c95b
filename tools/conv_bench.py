"""Same-box timing of the NatureCNN (C3) convolution forward: hand-written f32 MFMA implicit GEMM with
the bias + ReLU in its store (rai_conv2d_bias_relu_fwd, csrc/conv.hip, every blocking variant) against
the product's previous path (MIOpen F.conv2d in find mode + rai_bias_relu_fwd), per layer at the update
minibatch B = 256 and the rollout batch B = 1024.  Also checks each variant against an fp64 CPU
convolution of the same inputs.

    python tools/conv_bench.py [--reps 50]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgload  # noqa: E402

_pkgload.load()

from rl_algo_impls_amd import _lib  # noqa: E402
from rl_algo_impls_amd import cnn_ops  # noqa: E402

LAYERS = [  # name, Ci, H, Co, k, stride, flatten
    ("conv1", 4, 84, 32, 8, 4, False),
    ("conv2", 32, 20, 64, 4, 2, False),
    ("conv3", 64, 9, 64, 3, 1, True),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batches", default="256,1024")
    ap.add_argument("--variants", default="0,12,13,14,15,16,17,18,19,20")
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda:0")
    L = _lib.lib()
    st = _lib.stream_handle(dev)
    out = []
    for B in [int(v) for v in args.batches.split(",")]:
        for name, Ci, H, Co, k, s, flat in LAYERS:
            g = torch.Generator().manual_seed(1)
            x = torch.rand(B, Ci, H, H, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
            w = (torch.randn(Co, Ci, k, k, generator=g) * (2.0 / (Ci * k * k)) ** 0.5).to(dev)
            w = w.contiguous(memory_format=torch.channels_last)
            b = (torch.randn(Co, generator=g) * 0.1).to(dev)
            OH = (H - k) // s + 1

            def ref_path():
                z = F.conv2d(x, w, None, s).contiguous(memory_format=torch.channels_last)
                return cnn_ops._bias_relu_fwd_nchw(z, b) if flat else cnn_ops._bias_relu_fwd(z, b)

            t_ref = timeit(ref_path, args.reps)
            # fp64 CPU check on the first 8 samples
            xd, wd, bd = x[:8].double().cpu(), w.double().cpu(), b.double().cpu()
            yd = torch.relu(F.conv2d(xd, wd, bd, s))
            yd = torch.flatten(yd, 1) if flat else yd.permute(0, 2, 3, 1).reshape(8, -1)
            row = {"B": B, "layer": name, "ref_us": round(t_ref, 2), "flops": 2 * B * OH * OH * Co * Ci * k * k}
            y = torch.empty((B, Co * OH * OH), dtype=torch.float32, device=dev)
            for v in [int(t) for t in args.variants.split(",")]:
                def mine():
                    return L.rai_conv2d_bias_relu_fwd_v(x.data_ptr(), w.data_ptr(), b.data_ptr(), B, H, H, Ci, Co,
                                                        k, k, s, 1 if flat else 0, y.data_ptr(), v, st)
                rc = mine()
                if rc != 0:
                    row[f"v{v}"] = f"rc={rc}"
                    continue
                torch.cuda.synchronize()
                err = (y[:8].double().cpu() - yd).abs().max().item() / max(yd.abs().max().item(), 1e-30)
                t = timeit(mine, args.reps)
                row[f"v{v}"] = {"us": round(t, 2), "tflops": round(row["flops"] / t / 1e6, 1), "relerr": err}
            nbs = int(L.rai_conv2d_fwd_splitk_bytes(B, H, H, Ci, Co, k, k, s, 1 if flat else 0))
            if nbs > 0:  # the split-K form the product takes for this shape (cnn_ops._conv_fwd_mfma)
                part = torch.empty(nbs // 4, dtype=torch.float32, device=dev)

                def mine_split():
                    return L.rai_conv2d_bias_relu_fwd_splitk(x.data_ptr(), w.data_ptr(), b.data_ptr(), B, H, H, Ci,
                                                             Co, k, k, s, 1 if flat else 0, y.data_ptr(),
                                                             part.data_ptr(), nbs, st)
                rc = mine_split()
                if rc == 0:
                    torch.cuda.synchronize()
                    err = (y[:8].double().cpu() - yd).abs().max().item() / max(yd.abs().max().item(), 1e-30)
                    t = timeit(mine_split, args.reps)
                    row["splitk"] = {"us": round(t, 2), "tflops": round(row["flops"] / t / 1e6, 1), "relerr": err}
                else:
                    row["splitk"] = f"rc={rc}"
            if Ci == 4:  # conv1 on the uint8 frames (the product's C3 path): the same forward with the /255 in-kernel
                xu = torch.randint(0, 256, (B, Ci, H, H), generator=g, dtype=torch.uint8).to(dev)
                xu = xu.contiguous(memory_format=torch.channels_last)

                def mine_u8():
                    return L.rai_conv2d_bias_relu_fwd_u8(xu.data_ptr(), C.c_float(255.0), w.data_ptr(), b.data_ptr(), B,
                                                         H, H, Ci, Co, k, k, s, 1 if flat else 0, y.data_ptr(), st)
                rc = mine_u8()
                row["u8_us"] = round(timeit(mine_u8, args.reps), 2) if rc == 0 else f"rc={rc}"
            # weight gradient: MIOpen (find mode) + the accumulate into .grad vs rai_conv2d_wgrad
            dz = (torch.randn(B, Co, OH, OH, generator=g) * 0.01).to(dev).contiguous(memory_format=torch.channels_last)
            grad = torch.zeros_like(w)

            def ref_wgrad():
                dw = torch.ops.aten.convolution_backward(dz, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                         [False, True, False])[1]
                grad.add_(dw)

            row["wgrad_ref_us"] = round(timeit(ref_wgrad, args.reps), 2)
            nb = int(L.rai_conv2d_wgrad_workspace_bytes(B, H, H, Ci, Co, k, k, s))
            ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            grad2 = torch.zeros_like(w)

            def mine_wgrad(tw=0, pf=0):
                return L.rai_conv2d_wgrad_v(x.data_ptr(), dz.data_ptr(), B, H, H, Ci, Co, k, k, s, grad2.data_ptr(), 1,
                                            ws.data_ptr(), nb, tw, pf, st)

            rc = mine_wgrad()
            if rc == 0:
                torch.cuda.synchronize()
                grad.zero_()
                grad2.zero_()
                ref_wgrad()
                mine_wgrad()
                torch.cuda.synchronize()
                row["wgrad_relerr"] = ((grad2 - grad).abs().max() / grad.abs().max()).item()
                row["wgrad_us"] = round(timeit(mine_wgrad, args.reps), 2)
                row["wgrad_tflops"] = round(row["flops"] / row["wgrad_us"] / 1e6, 1)
                for tw, pf in ((512, 4), (512, 8), (512, 104), (512, 108), (1024, 104), (1024, 108)):
                    row[f"wgrad_{tw}_{pf}_us"] = round(timeit(lambda: mine_wgrad(tw, pf), args.reps), 2)
                row["wgrad_ws_mb"] = round(nb / 2**20, 2)
            else:
                row["wgrad_us"] = f"rc={rc}"
            if Ci in (32, 64):  # input gradient: MIOpen dx-only vs rai_conv2d_dgrad
                wt = w

                def ref_dgrad():
                    return torch.ops.aten.convolution_backward(dz, x, wt, None, [s, s], [0, 0], [1, 1], False, [0, 0],
                                                               1, [True, False, False])[0]

                row["dgrad_ref_us"] = round(timeit(ref_dgrad, args.reps), 2)
                dx = torch.empty_like(x, memory_format=torch.channels_last)

                def mine_dgrad():
                    return L.rai_conv2d_dgrad(dz.data_ptr(), wt.data_ptr(), B, H, H, Ci, Co, k, k, s, dx.data_ptr(), st)

                rc = mine_dgrad()
                if rc == 0:
                    torch.cuda.synchronize()
                    r = ref_dgrad()
                    row["dgrad_relerr"] = ((dx - r).abs().max() / r.abs().max()).item()
                    row["dgrad_us"] = round(timeit(mine_dgrad, args.reps), 2)
                    for dv in (1, 2, 3):
                        def mine_dgrad_v():
                            return L.rai_conv2d_dgrad_v(dz.data_ptr(), wt.data_ptr(), B, H, H, Ci, Co, k, k, s,
                                                        dx.data_ptr(), dv, st)
                        rc = mine_dgrad_v()
                        torch.cuda.synchronize()
                        r = ref_dgrad()
                        row[f"dgrad_v{dv}_relerr"] = ((dx - r).abs().max() / r.abs().max()).item() if rc == 0 else rc
                        row[f"dgrad_v{dv}_us"] = round(timeit(mine_dgrad_v, args.reps), 2) if rc == 0 else rc
                else:
                    row["dgrad_us"] = f"rc={rc}"
            print(json.dumps(row), flush=True)
            out.append(row)
    return out


if __name__ == "__main__":
    main()
