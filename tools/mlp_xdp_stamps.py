"""Diagnostic: per-phase stamp ticks of the CartPole epoch kernel (csrc/mlp_mc8.h) with the in-kernel
cross-GPU exchange at world 2 (two processes on this one GPU, regions IPC-mapped, gloo for setup)
next to the single-process kernel, to attribute the extra time per optimizer step.  Loads the
stamps build (lib/librai_amd_stamps.so).  Not part of the product or the tests.

    python tools/mlp_xdp_stamps.py > gpurun_out/xdp_stamps.txt
"""
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
NAMES = ["F1 (own columns) + barrier", "F2 + output partials + barrier", "loss + dZ2 + barrier",
         "dH1 + dZ1 + partials + barrier", "P_B dW2 + sums", "round 1: publish + counter wait",
         "share sum (+ xGMI push/flags/sum) + round 2 publish + wait", "all-gather + norm + adam"]


def run(rank, world, port, q):
    os.environ["RAI_AMD_LIB"] = str(ROOT / "rl-algo-impls_amd" / "lib" / "librai_amd_stamps.so")
    sys.path.insert(0, str(ROOT))
    import ctypes as C

    import numpy as np
    import torch

    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd import _lib
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator

    dev = torch.device("cuda", 0)
    if world > 1:
        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(1)
    env = SyntheticVecEnv(4096, "cartpole", seed=1 + rank)
    policy = ActorCritic(env).to(dev)
    gen = SyncStepRolloutGenerator(policy, env, n_steps=128, seed=7 + rank)
    algo = PPO(policy, dev, None, batch_size=256, n_epochs=1, learning_rate=1e-3, gamma=0.98, gae_lambda=0.8)
    if world > 1:
        algo.enable_data_parallel(xdp=True)
        assert algo._xdp is not None, "in-kernel exchange not set up"
    r = gen.rollout(gamma=0.98, gae_lambda=0.8)
    algo.update(r)  # warm
    torch.cuda.synchronize()
    out0 = (C.c_ulonglong * 64)()
    assert _lib.lib().rai_mlp_debug_stamps(out0) == 0
    if world > 1:
        torch.distributed.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    algo.update(r)
    ev1.record()
    ev1.synchronize()
    out1 = (C.c_ulonglong * 64)()
    assert _lib.lib().rai_mlp_debug_stamps(out1) == 0
    st = (np.array(out1, dtype=np.float64) - np.array(out0, dtype=np.float64)).reshape(2, 32)
    q.put((rank, ev0.elapsed_time(ev1), st.tolist(), r.total_steps // 256))
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    import numpy as np

    ctx = mp.get_context("spawn")
    for world in (1, 2):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        q = ctx.Queue()
        procs = [ctx.Process(target=run, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = sorted(q.get(timeout=300) for _ in procs)
        for p in procs:
            p.join(timeout=60)
        for rank, ms, st, nmb in res:
            st = np.array(st)
            print(f"=== world {world} rank {rank}: epoch {ms:.2f} ms for {nmb} steps -> {ms * 1e3 / nmb:.2f} us/step")
            for net in range(2):
                tot = st[net, 1:1 + len(NAMES)].sum()
                print(f"  --- {'actor' if net == 0 else 'critic'} workgroup 0: {tot / nmb:.0f} stamp-ticks/step")
                for i, n in enumerate(NAMES):
                    v = st[net, 1 + i] / nmb
                    print(f"    {n:60s} {v:8.1f} ticks/step {100 * v / max(tot / nmb, 1):5.1f}%")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
