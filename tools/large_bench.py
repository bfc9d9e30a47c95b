"""Microbenchmark of the large-minibatch PPO step (csrc/mlp_large.hip) at config C2's scaled batch
(SURVEY 8(d) policy (b)): 524,288 rollout rows, batch 131,072, synthetic inputs in HBM, rai_mlp_ppo_epoch
called per epoch; prints the gradient kernel's mean launch time (library HIP-event hook) and its MFMA
fraction.  Diagnostic only (bench.py is the measured line).

    python tools/large_bench.py [--epochs 20] [--rows 524288] [--batch 131072] [--act 0]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--rows", type=int, default=524288)
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--act", type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    import torch

    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd import _lib
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    env = SyntheticVecEnv(8, "cartpole", seed=1)
    policy = ActorCritic(env, activation_fn="relu" if args.act else "tanh").to(dev)
    algo = PPO(policy, dev, None, batch_size=args.batch, n_epochs=1, learning_rate=1e-4)
    n = args.rows
    g = torch.Generator(device=dev).manual_seed(1)
    obs = torch.randn((n, 4), device=dev, generator=g)
    act = torch.randint(0, 2, (n,), device=dev, generator=g)
    logp = -torch.rand(n, device=dev, generator=g) - 0.3
    val = torch.randn(n, device=dev, generator=g)
    adv = torch.randn(n, device=dev, generator=g)
    ret = val + adv
    nmb = (n + args.batch - 1) // args.batch
    blocks = algo.blocks
    blocks.ensure_tables(nmb * args.epochs, nmb * args.epochs)
    blocks.upload(algo._hparams(1, nmb), 0)
    algo._ensure_mlp_workspace(n)
    opt = algo.optimizer
    opt.sync_hparams()
    L = _lib.lib()
    st = _lib.stream_handle(dev)

    def epoch():
        rc = L.rai_mlp_ppo_epoch(algo.flat.flat.data_ptr(), opt.state1.data_ptr(), opt.state2.data_ptr(),
                                 obs.data_ptr(), act.data_ptr(), logp.data_ptr(), val.data_ptr(), adv.data_ptr(),
                                 ret.data_ptr(), n, args.batch, 4, 64, 2, args.act, blocks.hp.data_ptr(),
                                 opt.hp_dev.data_ptr(), blocks.state.data_ptr(), blocks.stats.data_ptr(),
                                 int(blocks.stats.shape[0]), blocks.norms.data_ptr(), int(blocks.norms.shape[0]),
                                 algo._mlp_ws.data_ptr(), algo._mlp_ws.numel(), st)
        _lib.check(rc, "rai_mlp_ppo_epoch")

    epoch()
    torch.cuda.synchronize()
    blocks.upload(algo._hparams(1, nmb), 0)
    cap = args.epochs * nmb
    _lib.check(L.rai_mlp_large_timing(cap), "timing")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.epochs):
        epoch()
    e1.record()
    torch.cuda.synchronize()
    buf, cnt = (C.c_float * cap)(), C.c_int32(0)
    _lib.check(L.rai_mlp_large_timing_read(buf, cap, C.byref(cnt)), "timing_read")
    ms = np.array(buf[:cnt.value])
    flops = 52352.0 * n / nmb
    print(f"lb_grads_kernel: {ms.mean() * 1e3:.1f} us mean ({ms.min() * 1e3:.1f} min) over {len(ms)} launches; "
          f"{flops / (ms.mean() * 1e-3) / 1e12:.2f} TFLOP/s = {flops / (ms.mean() * 1e-3) / 157.3e12:.4f} of f32 MFMA; "
          f"epoch {e0.elapsed_time(e1) / args.epochs * 1e3:.1f} us ({nmb} steps)")
    _lib.check(L.rai_mlp_large_timing(0), "timing")


if __name__ == "__main__":
    main()
