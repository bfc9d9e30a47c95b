"""Probe: host->device paths for one Pong observation batch (1024x4x84x84 u8, 29 MB) from a
pageable numpy array — (a) copy into pinned staging then async H2D (the rollout's current path),
(b) direct H2D from the pageable array (HIP stages internally), (c) threaded copy into pinned."""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

dev = torch.device("cuda", 0)
a = np.random.randint(0, 256, size=(1024, 4, 84, 84), dtype=np.uint8)
pinned = torch.empty(a.shape, dtype=torch.uint8).pin_memory()
d = torch.empty(a.shape, dtype=torch.uint8, device=dev)


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def staged():
    np.copyto(pinned.numpy(), a)
    d.copy_(pinned, non_blocking=True)


def direct():
    d.copy_(torch.from_numpy(a), non_blocking=True)


ex = ThreadPoolExecutor(8)
chunks = np.array_split(np.arange(1024), 8)
pn = pinned.numpy()


def threaded():
    list(ex.map(lambda ix: np.copyto(pn[ix[0]:ix[-1] + 1], a[ix[0]:ix[-1] + 1]), chunks))
    d.copy_(pinned, non_blocking=True)


def copy_only():
    np.copyto(pn, a)


def h2d_only():
    d.copy_(pinned, non_blocking=True)


for name, fn in [("np.copyto only", copy_only), ("pinned H2D only", h2d_only), ("staged (current)", staged),
                 ("direct pageable", direct), ("threaded x8 + H2D", threaded)]:
    print(f"{name:20s} {timeit(fn):7.2f} ms", flush=True)
