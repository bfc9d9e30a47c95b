"""Per-phase shader-clock stamps of the large-minibatch gradient kernel (diagnostic build
lib/librai_amd_stamps.so, -DRAI_STAMPS; never the product).  Runs tools/large_bench.py's workload once
more after the timed epochs and prints, per phase, the median over waves of the cycles spent, and the
in-kernel clock from the constant 100 MHz counter.

    python tools/large_stamps.py [--batch 131072 --rows 524288]
"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ["RAI_AMD_LIB"] = str(ROOT / "rl-algo-impls_amd" / "lib" / "librai_amd_stamps.so")
sys.path.insert(0, str(ROOT / "tools"))
sys.argv += ["--epochs", "2"] if "--epochs" not in sys.argv else []
import large_bench  # noqa: E402

large_bench.main()
import numpy as np  # noqa: E402
from rl_algo_impls_amd import _lib  # noqa: E402

n = 256 * 4 * 32
buf = (C.c_ulonglong * n)()
assert _lib.lib().rai_mlp_large_debug_stamps(buf) == 0
a = np.array(buf, dtype=np.float64).reshape(256, 4, 32)
names = ["staging + sync", "register operands", "tile loop", "lane sums", "partials to LDS + sync",
         "sum + global write"]
for k, nm in enumerate(names):
    d = a[:, :, k + 1] - a[:, :, k]
    print(f"{nm:>26}: median {np.median(d):9.0f}  max {d.max():9.0f} cycles")
tot = a[:, :, 6] - a[:, :, 0]
rt = (a[:, :, 9] - a[:, :, 8]) / 100e6
print(f"{'total':>26}: median {np.median(tot):9.0f}  max {tot.max():9.0f} cycles;  "
      f"in-kernel clock {np.median(tot / rt) / 1e9:.3f} GHz; wall (100 MHz) median {np.median(rt) * 1e6:.1f} us")
names = ["P0 layer-1 MFMAs", "P1 dH1 blk0 | act H1", "P2 dH1 blk1 | act H1", "P3 dH1 blk2 | H1 store",
         "P4 dH1 blk3", "P5a L2 blk0 | dH1 store", "P5b L2 blk1 | dW operands", "P5c L2 blk2 | dZ1",
         "P5d L2 blk3", "P6 dW2 s0 | act H2", "P7 dW2 s1 | act H2", "P8 dW2 s2 | output layer",
         "P9 dW2 s3 | loss", "P10 dW1 | output backward"]
tot_ph = 0
for k, nm in enumerate(names):
    v = a[:, :, 10 + k]
    v = v[v > 0]
    if len(v):
        tot_ph += np.median(v)
        print(f"{nm:>30}: median {np.median(v) / 15:8.0f} cycles per step")
print(f"{'phases sum':>30}: {tot_ph / 15:8.0f} cycles per step (15 steps per wave at batch 131072)")
start = a[:, :, 8] - a[:, :, 8].min()
print(f"wave start spread (100 MHz ticks): median {np.median(start):.0f} max {start.max():.0f}")
