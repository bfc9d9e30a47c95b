#!/usr/bin/env python
"""bench.py — PPO rollout+update throughput on MI355X (BASELINE.json configs[1]).

One "step" = one PPO update (learn_epoch): a rollout of n_steps x num_envs env
steps on the seeded synthetic CartPole-shaped VecEnv (host), GAE on device, and
n_epochs x minibatches of fused loss / backward / clip+Adam — exactly the region
the reference times as train/steps_per_second (rl_algo_impls/ppo/ppo.py:221,422-427).

    python bench.py [--gpus N --steps K --warmup W]   (N > 1: the N ranks are started here unless a
                                                       launcher such as torch.distributed.run already did) [--config cartpole|pong|halfcheetah|microrts]
                    [--batch-policy yaml|scaled] [--env-partition split|per-rank] [--dp-batch global|per-rank]

Multi-GPU: one process per GPU (torch.distributed.run).  Default = SURVEY.md 8(d)/8(e): the config's
num_envs is the GLOBAL env count, split over the ranks (rank r owns envs [r N/R, (r+1) N/R) with its
own HBM rollout and local GAE), and every optimizer step's global minibatch is the YAML batch_size
(batch_size / R rows per rank), so the update is the single-process update and the total work is
fixed as R grows ("scaling": "strong").  --env-partition per-rank gives every rank num_envs envs
(weak scaling).  Gradients are exchanged once per optimizer step (in-kernel over xGMI for the
CartPole-class epoch kernel, RCCL otherwise).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

CONFIGS = {
    # BASELINE.json configs[1]: ppo CartPole-v1, num_envs=4096, n_steps=128 (YAML algo hyperparams,
    # rl_algo_impls/hyperparams/ppo.yml:1-23)
    "cartpole": dict(env="cartpole", num_envs=4096, n_steps=128, policy=dict(),
                     algo=dict(batch_size=256, n_epochs=20, gamma=0.98, gae_lambda=0.8, ent_coef=0.0,
                               learning_rate=1e-3, clip_range=0.2)),
    # configs[2]: PongNoFrameskip-v4 NatureCNN, num_envs=1024, n_steps=128 (ppo.yml:225-253 _atari)
    "pong": dict(env="pong", num_envs=1024, n_steps=128, policy=dict(activation_fn="relu"),
                 algo=dict(batch_size=256, n_epochs=4, learning_rate=2.5e-4, clip_range=0.1, vf_coef=0.5,
                           ent_coef=0.01)),
    # configs[3]: HalfCheetah-v4, num_envs=2048 (global; per-rank share under DP), n_steps=512 (ppo.yml:337-359)
    "halfcheetah": dict(env="halfcheetah", num_envs=2048, n_steps=512,
                        policy=dict(pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256], activation_fn="relu",
                                    log_std_init=-2, init_layers_orthogonal=False),
                        algo=dict(batch_size=64, n_epochs=20, gamma=0.98, gae_lambda=0.92, ent_coef=0.000401762,
                                  max_grad_norm=0.8, vf_coef=0.58096, learning_rate=2.0633e-05, clip_range=0.1)),
    # configs[4]: MicroRTS squnet-d16-128 GridNet selfplay, num_envs=512 (global; per-rank share under DP),
    # n_steps=512 (ppo-Microrts.yml:274-299,511-558: Microrts-squnet-d16-128-sc-cos-ga-selfplay; first
    # schedule phase :402-407); batch_size 6144 is the global minibatch (per rank 6144 / world)
    "microrts": dict(env="microrts", num_envs=512, n_steps=512,
                     policy=dict(actor_head_style="squeeze_unet", activation_fn="relu", cnn_flatten_dim=256,
                                 channels_per_level=[128, 128, 128], strides_per_level=[[2, 2], [2, 2]],
                                 deconv_strides_per_level=[[2, 2], [2, 2]],
                                 encoder_residual_blocks_per_level=[3, 2, 4],
                                 decoder_residual_blocks_per_level=[2, 3], increment_kernel_size_on_down_conv=True,
                                 additional_critic_activation_functions=["tanh", "identity"],
                                 subaction_mask={0: {1: 1, 2: 2, 3: 3, 4: 4, 5: 4, 6: 5}}),
                     algo=dict(batch_size=6144, n_epochs=2, gamma=[0.99, 0.999, 0.999],
                               gae_lambda=[0.95, 0.99, 0.99], clip_range=0.1, clip_range_vf=None,
                               ppo2_vf_coef_halving=True, max_grad_norm=0.5, gradient_accumulation=True,
                               multi_reward_weights=[0.8, 0.01, 0.19], vf_coef=[0.5, 0.1, 0.2], ent_coef=0.01,
                               learning_rate=1e-4)),
}


# algorithmic FLOPs per env step = rollout forward + n_epochs x (forward + backward)
UPDATE_FLOPS = {"pong": 18.69e6 + 4 * 49.53e6, "halfcheetah": 0.283e6 + 20 * 0.832e6, "microrts": 954e6 + 2 * 2818e6}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", default="cartpole", choices=sorted(CONFIGS))
    p.add_argument("--batch-policy", default="yaml", choices=["yaml", "scaled"],
                   help="yaml: the YAML batch_size; scaled: batch = T*N/4 (4 minibatches/epoch)")
    p.add_argument("--dp-batch", default="global", choices=["global", "per-rank"],
                   help="data-parallel minibatch rule, the same for every config: global (default) = SURVEY "
                        "8(e): batch_size / world rows per rank, so the global minibatch is the YAML batch_size "
                        "and the update equals the single-process one; per-rank = every rank takes batch_size "
                        "rows of its own rollout per optimizer step (global minibatch batch_size x world)")
    p.add_argument("--env-partition", default="split", choices=["split", "per-rank"],
                   help="split (default) = SURVEY 8(d): the config's num_envs is global, each rank owns "
                        "num_envs / world of them (total work fixed: strong scaling); per-rank = every rank "
                        "owns num_envs envs (per-GPU work fixed: weak scaling)")
    p.add_argument("--dp-update", default="auto", choices=["auto", "exchange", "replicated"],
                   help="data-parallel update (PPO.enable_data_parallel update_mode): exchange = the ranks' "
                        "gradients summed every optimizer step; replicated = one all-gather of the rollout per "
                        "update, the identical single-process update on every rank (global minibatch only); "
                        "auto (default) = replicated for the dependent-chain epoch kernels (C2 at the YAML "
                        "batch, C4), exchange otherwise")
    p.add_argument("--deterministic", type=int, default=0, choices=[0, 1],
                   help="1: torch.use_deterministic_algorithms + MIOpen deterministic solvers (the reference's "
                        "set_device_optimizations default, rl_algo_impls/runner/running_utils.py:161-166); off by "
                        "default: ~100x slower C3 convolutions on MI355X (rl-algo-impls_amd/running_utils.py)")
    p.add_argument("--cudnn-benchmark", type=int, default=None, choices=[0, 1],
                   help="MIOpen find mode (torch.backends.cudnn.benchmark) for the convolutions; default on for "
                        "pong; microrts runs immediate mode over the shipped find database (same solver picks)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--roofline-reps", type=int, default=200)
    p.add_argument("--num-envs", type=int, default=None, help="override (rehearsal/debug only; not a bench line)")
    p.add_argument("--dp-rehearsal", action="store_true",
                   help="single process: run the data-parallel update path over a 1-rank RCCL group "
                        "(measures the per-step DP machinery; not a bench line)")
    return p.parse_args()


def latency_roofline(G: int, avg_ms: float, steps_per_launch: int, kname: str) -> dict:
    """Per-optimizer-step latency floor of the fused CartPole epoch kernel (csrc/mlp_mc8.h) from the
    MI355X price list (/opt/skills/guides/MI355X_MICROARCH.md), against the measured step time.

    A launch is `steps_per_launch` DEPENDENT optimizer steps (step k+1's forward reads step k's Adam
    output, rl_algo_impls/ppo/ppo.py:375,441-447), so the bound is the critical path of one step:
      * the MFMA chain of one wave: at G = 16 a wave owns one 16-row tile x 16 hidden columns, so
        layer 2 forward and dH1 are 16 dependent v_mfma_f32_16x16x4f32 each (40-cycle dependent
        latency, constants table), layer 1 one more, and dW2 16 independent-accumulator MFMAs at
        the 32-cycle issue rate: (1 + 16 + 16) x 40 + 16 x 32 = 1,832 cycles at 2.4 GHz (G = 8:
        two tiles of 32 columns per wave, 3,136 cycles);
      * two cross-CU all-to-all edges among the network's G CUs (reduce-scatter of the partial
        gradients, then all-gather of the summed shares and their norms).  Priced (round 6) for the
        exchange the kernel runs: G = 16 readers, one network's CUs inside one XCD.  Each edge moves one
        network's gradient, 4,610 floats = 18 KB of payload, i.e. a 32 KB sweep in the price list's
        granule bytes (an edge size counts 2x the payload); the 'allgather' row prices a 32 KB sweep at
        2.9 us parked (the waiting CUs run no HBM stream) for 256 readers, and the same row's reader
        correction takes 1.9 us off for <= 32 readers ("256 -> 32 readers -1.9 on a 16 KB sweep, 32 -> 8
        no further gain"): 1.0 us per edge.  No same-XCD credit is taken (the price list's cross-XCD
        delta, +0.1-0.3 us, is the 'handoff-1to1' row's).  Rounds 1-5 priced each edge at the row's
        256-reader 8 KB figure (2.4 us), a floor of 5.56 us that overstated the frac by ~2x.
    frac = floor / measured us per step: the share of the step the hardware's latencies account for."""
    RC = 256 // G  # rows per CU; CT 16-column tiles per wave (csrc/mlp_mc8.h M8Geo)
    CT = 64 // 16 // (4 // (RC // 16))
    chain = lambda n_dep, n_issue: max(n_dep * 40, n_issue * 32)  # dependent latency vs issue rate
    mfma_cycles = chain(1, CT) + 2 * chain(16, 16 * CT) + chain(RC // 4, RC)
    t_mfma = mfma_cycles / 2.4e3  # us at 2.4 GHz
    t_edge = 2.9 - 1.9  # 'allgather' 32 KB parked, <= 32 readers (MI355X_MICROARCH.md price list)
    floor_us = t_mfma + 2 * t_edge
    step_us = avg_ms * 1e3 / max(steps_per_launch, 1)
    return {"kernel": kname, "bound": "latency", "achieved": round(step_us, 3), "peak": round(floor_us, 3),
            "unit": "us per dependent optimizer step", "frac": round(floor_us / step_us, 4),
            "floor_terms_us": {"mfma_chain": round(t_mfma, 3), "allgather_edges": round(2 * t_edge, 3)},
            "edge_pricing": "allgather row, 32 KB sweep (18 KB payload) parked 2.9 us, -1.9 us for <= 32 readers",
            "steps_per_launch": steps_per_launch}


def latency_roofline_wide(avg_ms: float, steps_per_launch: int, kname: str) -> dict:
    """Per-optimizer-step latency floor of the C4 whole-epoch kernel (csrc/mlp_wide_epoch.hip,
    mlp_wide_epoch_kernel<1>) from the MI355X price list (/opt/skills/guides/MI355X_MICROARCH.md),
    against the measured step time.  A launch is `steps_per_launch` DEPENDENT optimizer steps
    (rl_algo_impls/ppo/ppo.py:375,441-447), so the bound is one step's critical path:
      * MFMA issue: each of the 16 workgroups of a network issues ~270 v_mfma_f32_16x16x4f32 per step
        (fwd2 64, dW2 64, dH1 64, dW1 16, small-parameter tiles 48, fwd1 5) over its
        4 SIMDs at the 32-cycle issue rate: 2,160 cycles at 2.4 GHz;
      * three all-to-all edges among the 16 workgroups (A: the H1 all-gather, B: the output-layer
        partials, C: the dZ2 all-gather), each at least the price list's 'allgather' row at its cheapest
        (8 KB published by 32 CUs, parked: 2.4 us);
      * the norm-share exchange D as tagged 8-B granules: the 'handoff-1to1' row, idle, 8 B (0.8 us).
    frac = floor / measured us per step."""
    t_mfma = 270 * 32 / 4 / 2.4e3
    t_edges = 3 * 2.4
    t_gran = 0.8
    floor_us = t_mfma + t_edges + t_gran
    step_us = avg_ms * 1e3 / max(steps_per_launch, 1)
    return {"kernel": kname, "bound": "latency", "achieved": round(step_us, 3), "peak": round(floor_us, 3),
            "unit": "us per dependent optimizer step", "frac": round(floor_us / step_us, 4),
            "floor_terms_us": {"mfma_issue": round(t_mfma, 3), "allgather_edges": t_edges, "granule_edge": t_gran},
            "steps_per_launch": steps_per_launch}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(args, N: int, T: int, algo_kw: dict) -> dict:
    """The reference's CPU trainer restated (oracle/cpu_trainer.py, pinned to the reference's own
    learn_epoch and NatureCNN steps by tests/test_cpu_trainer.py) on the host cores, rank 0 only.
    A whole C2 update is ~60 s of CPU, so the C2 line times the full rollout + GAE and a bounded
    sample of the update's minibatch steps (extrapolated); the extrapolation's error is measured on a
    whole update 32x smaller (N/32 envs, the same 20 epochs), timed whole and sampled at the same
    fraction of its steps."""
    import torch

    sys.path.insert(0, str(ROOT / "oracle"))
    import cpu_trainer  # checker/baseline only

    # the host cores this process may use: the GPU box grants 16 threads per GPU (its OMP_NUM_THREADS /
    # MAX_JOBS are 16), while os.cpu_count() reports the whole machine's CPUs, most of them not ours
    share = int(os.environ.get("OMP_NUM_THREADS") or 16)
    torch.set_num_threads(max(1, min(os.cpu_count() or 1, share)))
    kw = dict(n_steps=T, batch_size=algo_kw["batch_size"], n_epochs=algo_kw["n_epochs"])
    res = cpu_trainer.time_update(args.cpu_baseline_seconds, num_envs=N, **kw)
    # the same sampled fraction of a whole update 32x smaller, against that update timed whole
    frac = res["minibatches_timed"] / res["minibatches_total"]
    small_n = max(1, N // 32)
    full_small = cpu_trainer.time_update(None, num_envs=small_n, **kw)
    budget = frac * (full_small["update_s"] - full_small["rollout_s"] - full_small["gae_s"])
    est_small = cpu_trainer.time_update(max(budget, 0.05), num_envs=small_n, **kw)
    err = est_small["update_s"] / full_small["update_s"] - 1.0
    return {"value": round(res["env_steps_per_s"], 1), "unit": "env-steps/s", "cores": res["threads"],
            "kind": "port", "cpu_model": cpu_model(),
            "cores_note": ("threads = the box's per-GPU CPU share (OMP_NUM_THREADS, 16 on the GPU box); "
                           "os.cpu_count() = %d counts the whole machine" % (os.cpu_count() or 0)),
            "sample": (f"full rollout {T}x{N} + numpy GAE + {res['minibatches_timed']} of "
                       f"{res['minibatches_total']} minibatch steps timed, update time extrapolated "
                       f"(oracle/cpu_trainer.py, torch CPU eager like the reference)"),
            "extrapolation_check": {"num_envs": small_n, "full_update_s": round(full_small["update_s"], 3),
                                    "extrapolated_update_s": round(est_small["update_s"], 3),
                                    "sampled_steps": est_small["minibatches_timed"],
                                    "total_steps": est_small["minibatches_total"], "rel_error": round(err, 4)}}


def _diagnostics(tag: str) -> None:
    """RAI_DIAG_DIR=<dir>: Python stacks of every thread on a fatal signal (faulthandler) and
    this process's /proc/self/maps at each stage, so a native crash's PCs (which are per process
    under ASLR) can be mapped to a library and offset afterwards."""
    d = os.environ.get("RAI_DIAG_DIR")
    if not d:
        return
    import faulthandler

    os.makedirs(d, exist_ok=True)
    if not faulthandler.is_enabled():
        _diagnostics.fh = open(os.path.join(d, f"faulthandler_{os.getpid()}.txt"), "w")
        faulthandler.enable(file=_diagnostics.fh, all_threads=True)
    with open("/proc/self/maps") as src, open(os.path.join(d, f"maps_{os.getpid()}_{tag}.txt"), "w") as dst:
        dst.write(src.read())
    print(f"[bench] diag: {tag} pid {os.getpid()}", file=sys.stderr, flush=True)


def _heartbeat(period: float = 45.0) -> None:
    """A daemon thread printing one stderr line per `period` seconds, so a long silent stretch (the first
    update's MIOpen find-mode tuning of every convolution shape in C3 / C5 runs minutes without output)
    is not taken for a hang by a runner that kills commands after minutes of silence."""
    import threading

    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(period)
            print(f"[bench] alive {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def self_launch(args) -> int | None:
    """`bench.py --gpus N` (N > 1) run without a launcher: start the N ranks here, one child process
    per GPU with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (what torch.distributed.run exports), wait
    for all of them and return the job's exit status.  Rank 0's JSON line is the job's output.  Runs
    before anything touches the GPU, and starts the ranks as children (no exec).  Returns None when this
    process already is a rank (a launcher set WORLD_SIZE) or N == 1."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        if args.gpus > 1 and int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']}")
        return None
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=os.environ.get("MASTER_PORT", str(port)))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    status = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            rc = p.poll()
            if rc is None:
                continue
            pending.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in pending:  # a failed rank leaves the others waiting in a collective: stop them
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return status


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    _diagnostics("start")
    if int(os.environ.get("RANK", "0")) == 0:
        _heartbeat()
    import numpy as np
    import torch

    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd import _lib
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.gae import compute_advantages_device
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("RAI_DIST_BACKEND", "nccl")  # nccl == RCCL over xGMI; gloo only to rehearse
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(ndev, 1))
    if args.dp_rehearsal and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(dev)
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if world > 1:
        torch.cuda.set_device(dev)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
    _lib.lib()
    from rl_algo_impls_amd.running_utils import set_device_optimizations

    # TunableOp for the torch library GEMMs (C3's fc layer) is the trainer's own setting: on whenever
    # deterministic mode is off (running_utils.set_gemm_tuning, called by set_device_optimizations;
    # RAI_TUNABLEOP=0 turns it off).  The bench points its results file at this run's TMPDIR, so every
    # bench run tunes in its warm-up update instead of inheriting an earlier run's picks
    os.environ.setdefault("RAI_TUNABLEOP_FILE", os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                             f"rai_bench_{os.getpid()}_tunableop%d.csv"))

    # the shipped MIOpen find database (running_utils.seed_miopen_find_db) is seeded into this run's TMPDIR,
    # not the user's cache: every bench run starts from the shipped records only
    os.environ.setdefault("RAI_MIOPEN_DB_DIR", os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                            f"rai_bench_{os.getpid()}_miopen"))
    set_device_optimizations(dev, use_deterministic_algorithms=bool(args.deterministic))
    tunableop = torch.cuda.tunable.is_enabled()
    # RAI_AUTOGRAD_MT=0 (profiling runs): autograd runs the backward on the calling thread instead of its
    # device worker thread, so every dispatch of the update is submitted from one host thread (the
    # rocprofv3 counter-collection crashes of r3zd / r3ze faulted with launches in flight on two)
    if os.environ.get("RAI_AUTOGRAD_MT") == "0":
        torch.autograd.set_multithreading_enabled(False)
    # MIOpen find mode for the CNN convolutions (C3 / C5): every candidate solver timed at the first call
    # of each problem, the fastest kept.  Measured C3: 1.10 s per update against 1.26 s with the default
    # immediate-mode choice (profiles/r2o_pong_find_mode_bench_line.json vs r2l)
    # C5 (microrts): immediate mode reads the solver choices from the shipped find database (running_utils.
    # seed_miopen_find_db), which are find mode's own picks: same update time (13.75k vs 13.76k env-steps/s,
    # profiles/r6d_c5_bench_immediate.json vs r6c_c5_bench.json) without the first update's search (30.5 s
    # warm-up instead of 193 s with the database and 543 s without: torch passes benchmark as MIOpen's
    # exhaustiveSearch, which re-times every solver of every problem even when the database holds it)
    cudnn_benchmark = args.cudnn_benchmark if args.cudnn_benchmark is not None else args.config == "pong"
    if os.environ.get("RAI_CUDNN_BENCHMARK") is not None:
        cudnn_benchmark = os.environ["RAI_CUDNN_BENCHMARK"] == "1"
    torch.backends.cudnn.benchmark = bool(cudnn_benchmark) and not args.deterministic
    # GEMM library A/B for the torch GEMMs left in the CNN configs (the fc layer): RAI_BLAS_ROCBLAS=1 routes
    # them to rocBLAS, RAI_TUNABLEOP=1 lets PyTorch's TunableOp time hipBLASLt / rocBLAS solutions per shape
    if os.environ.get("RAI_BLAS_ROCBLAS") == "1":
        torch.backends.cuda.preferred_blas_library("cublas")  # = rocBLAS on ROCm

    cfg = CONFIGS[args.config]
    N, T = (args.num_envs or cfg["num_envs"]), cfg["n_steps"]
    algo_kw = dict(cfg["algo"])
    # env partition (the same rule for every config): split = SURVEY 8(d)'s "global N fixed; per-GPU
    # N = N/R" (each rank owns N / world envs); per-rank = every rank owns N envs
    split = args.env_partition == "split"
    if split and world > 1:
        if N % world:
            raise SystemExit(f"--env-partition split: num_envs {N} not divisible by {world}")
        N = N // world
    if args.config == "microrts" and args.num_envs:  # rehearsal at fewer envs: keep the YAML's minibatches
        algo_kw["batch_size"] = max(1, algo_kw["batch_size"] * N // cfg["num_envs"])
    if args.batch_policy == "scaled":
        algo_kw["batch_size"] = T * N // 4
    if args.dp_batch == "global" and algo_kw["batch_size"] % world:
        raise SystemExit(f"--dp-batch global: batch_size {algo_kw['batch_size']} not divisible by {world}")
    torch.manual_seed(1 + rank)
    env = SyntheticVecEnv(N, cfg["env"], seed=1000 * rank + 1)
    policy = ActorCritic(env, **cfg["policy"]).to(dev)
    if world > 1:  # identical initial weights on every rank
        with torch.no_grad():
            for p in policy.parameters():
                torch.distributed.broadcast(p.data, 0)
    # the reference runner's rollout kwargs: the policy's subaction_mask goes to the generator too
    # (rl_algo_impls/runner/train.py:159-162), where it gates Batch.num_actions
    rollout_kw = {"subaction_mask": cfg["policy"]["subaction_mask"]} if "subaction_mask" in cfg["policy"] else {}
    gen = SyncStepRolloutGenerator(policy, env, n_steps=T, seed=1234 + rank, **rollout_kw)
    algo = PPO(policy, dev, None, **algo_kw)
    if world > 1 or args.dp_rehearsal:  # minibatch rule: one for every config, named in the JSON line
        algo.enable_data_parallel(dp_batch=args.dp_batch,
                                  update_mode=None if args.dp_update == "auto" else args.dp_update)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    def progress(tag, i, t_start):
        if rank == 0:
            print(f"[bench] {tag} update {i}: {time.perf_counter() - t_start:.2f} s "
                  f"(this update: rollout {getattr(algo, 'last_rollout_seconds', 0.0):.3f} s of "
                  f"{getattr(algo, 'last_update_seconds', 0.0):.3f} s)", file=sys.stderr, flush=True)

    # SURVEY 8(d) batch policy (b) on the CartPole-class MLP: the large-minibatch kernels (csrc/mlp_large.hip);
    # their gradient kernel is the dominant one, timed per launch by the library's HIP-event hook
    large = (args.config == "cartpole" and algo.fused_mlp_spec() is not None
             and algo.batch_size > _lib.RAI_MLP_EPOCH_MAX_B)
    nmb = (T * N + algo.batch_size - 1) // algo.batch_size
    large_steps = large
    _diagnostics("setup")
    for i in range(args.warmup):
        tw = time.perf_counter()
        algo.learn_epoch(0, 1, gen, None)
        progress("warmup", i, tw)
    barrier()
    algo.kernel_events = []  # HIP events around every fused epoch launch (same stream as the kernel)
    if large:
        _lib.check(_lib.lib().rai_mlp_large_timing(args.steps * algo_kw["n_epochs"] * nmb), "rai_mlp_large_timing")
    t0 = time.perf_counter()
    for i in range(args.steps):
        algo.learn_epoch(0, 1, gen, None)
        progress("timed", i, t0)
        if i == 0:
            _diagnostics("update0")
    barrier()
    elapsed = time.perf_counter() - t0
    epoch_ms = [e0.elapsed_time(e1) for e0, e1 in algo.kernel_events]
    algo.kernel_events = None
    large_ms = []
    if large:
        import ctypes as C

        cap = args.steps * algo_kw["n_epochs"] * nmb
        buf, cnt = (C.c_float * cap)(), C.c_int32(0)
        _lib.check(_lib.lib().rai_mlp_large_timing_read(buf, cap, C.byref(cnt)), "rai_mlp_large_timing_read")
        large_ms = list(buf[:cnt.value])
        _lib.check(_lib.lib().rai_mlp_large_timing(0), "rai_mlp_large_timing")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    total_steps = args.steps * T * N * world
    value = total_steps / elapsed

    # ---- roofline of the GAE kernel (named by the BASELINE metric): each launch bracketed by its
    # own HIP event pair on the stream it is launched on (torch's current stream = the stream passed
    # to rai_gae), so host launch overhead between launches is not counted as kernel time
    r = gen.rollout(gamma=algo.gamma, gae_lambda=algo.gae_lambda)
    K = int(r.values.shape[2]) if r.values.dim() > 2 else 1
    gae_bytes = (4 * T * N * K) * 4 + T * N + 4 * N * K + N  # r, V, adv, returns + starts + next V/starts
    adv = torch.empty_like(r.values)
    ret = torch.empty_like(r.values)

    def gae():
        compute_advantages_device(r.rewards, r.values, r.episode_starts, r.next_episode_starts, r.next_values,
                                  algo.gamma, algo.gae_lambda, advantages_out=adv, returns_out=ret)

    for _ in range(10):
        gae()
    torch.cuda.synchronize()
    # park the stream behind a ~20 ms spin so every (event, launch, event) triple below is queued
    # before the GPU reaches it: the pairs then time the kernel, not the Python launch gap
    torch.cuda._sleep(50_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.roofline_reps):  # back to back: kernel time + the kernel-boundary gap
        gae()
    e1.record()
    torch.cuda.synchronize()
    gae_us = e0.elapsed_time(e1) * 1e3 / args.roofline_reps
    # the same kernel in its bandwidth regime (SURVEY.md 8(d)'s (128, 2^20) microbench shape): the
    # workload shape above is bound by the serial fp64 chain and launch latency, not by HBM
    Tl, Nl = 128, 1 << 20
    gl_ = torch.Generator(device=dev).manual_seed(3)
    rl_, vl_ = (torch.randn((Tl, Nl), device=dev, generator=gl_) for _ in range(2))
    esl = (torch.rand((Tl, Nl), device=dev, generator=gl_) < 0.01).to(torch.uint8)
    nesl = torch.zeros(Nl, dtype=torch.uint8, device=dev)
    nvl, advl, retl = torch.randn(Nl, device=dev, generator=gl_), torch.empty_like(rl_), torch.empty_like(rl_)
    large = lambda: compute_advantages_device(rl_, vl_, esl, nesl, nvl, 0.99, 0.95, advantages_out=advl,
                                              returns_out=retl)
    for _ in range(3):
        large()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        large()
    e1.record()
    torch.cuda.synchronize()
    large_us = e0.elapsed_time(e1) * 1e3 / 20
    large_bytes = 16 * Tl * Nl + Tl * Nl + 5 * Nl
    # rai_gae's pick at >= 2^18 columns, K = 1 (csrc/gae.hip): the streaming kernel, 1024 threads,
    # nontemporal loads / stores
    roof_gae_large = {"kernel": "gae_stream_kernel<double, 4, true, 1024, true>", "shape": [Tl, Nl, 1], "bound": "hbm",
                      "achieved": round(large_bytes / (large_us * 1e-6) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                      "frac": round(large_bytes / (large_us * 1e-6) / 1e9 / 8000.0, 4), "avg_us": round(large_us, 2),
                      "bytes_per_launch": large_bytes}
    del rl_, vl_, esl, advl, retl
    workload = f"ppo {args.config} num_envs={N}/rank n_steps={T}"
    if args.batch_policy == "scaled":
        workload += f" batch_policy=scaled batch={algo.batch_size}"
    lib_sha = _lib.lib_sha256()
    pmc, pmc_src = {}, None
    # the newest PMC summary (profiles/r<round><letter>_pmc.json, tools/pmc_summary.py) holding this workload
    for pmc_path in sorted((ROOT / "profiles").glob("r*_pmc.json"), reverse=True):
        pmc = json.loads(pmc_path.read_text()).get(workload, {})
        if pmc:
            pmc_src = pmc_path.name
            break

    def traffic(kernel):
        """HBM bytes per launch from the PMC summary, only when its counters were collected on the very
        library this process loaded (lib_sha256); otherwise None (a stale figure is not reported)."""
        e = pmc.get(kernel, {})
        return e.get("traffic_bytes_per_launch") if e.get("lib_sha256") == lib_sha else None

    def traffic_source(kernel):
        e = pmc.get(kernel, {})
        if not e:
            return None
        if e.get("lib_sha256") != lib_sha:
            return f"{pmc_src}: measured on another librai_amd.so build (sha256 {str(e.get('lib_sha256'))[:12]}), not reported"
        return f"{pmc_src} (2 x FETCH_SIZE + WRITE_SIZE per launch, same library sha256 {lib_sha[:12]})"

    # the instantiation rai_gae picks (csrc/gae.hip): columns per workgroup by column count
    C = N * K
    gae_name = "gae_kernel<double, %d>" % (64 if C >= 256 * 64 else (32 if C >= 256 * 32 else 16))
    roof_gae = {"kernel": gae_name, "bound": "hbm", "achieved": round(gae_bytes / (gae_us * 1e-6) / 1e9, 1),
                "peak": 8000.0, "unit": "GB/s", "frac": round(gae_bytes / (gae_us * 1e-6) / 1e9 / 8000.0, 4),
                "traffic": traffic(gae_name), "traffic_source": traffic_source(gae_name), "avg_us": round(gae_us, 3),
                "bytes_per_launch": gae_bytes}
    # rows one update's epoch launches cover: the whole env group's under the replicated data-parallel update
    # (every rank runs the single-process update over the gathered rollout), this rank's otherwise
    TN = T * N * (world if getattr(algo, "dp_update_mode", "exchange") == "replicated" and world > 1 else 1)
    if epoch_ms and args.config == "halfcheetah":
        # dominant kernel: the persistent wide-MLP epoch (rai_mlp_wide_epoch, csrc/mlp_wide_epoch.hip):
        # one launch = every minibatch step of one epoch = T*N samples of forward+backward at SURVEY.md
        # 8(d)'s 0.832 MFLOP/sample (HalfCheetah MLP, torch.utils.flop_counter), f32 MFMA peak
        flops = 0.832e6 * TN
        ms = float(np.mean(epoch_ms))
        tf = flops / (ms * 1e-3) / 1e12
        head = 1  # Gaussian
        kname = "mlp_wide_epoch_kernel<%d>" % head
        roofline = {"kernel": kname + " (rai_mlp_wide_epoch, 16 CUs per network)", "bound": "mfma",
                    "achieved": round(tf, 4), "peak": 157.3, "unit": "TFLOP/s", "frac": round(tf / 157.3, 6),
                    "traffic": traffic(kname), "traffic_source": traffic_source(kname), "avg_ms": round(ms, 3),
                    "flops_per_launch": flops, "launches_timed": len(epoch_ms)}
        steps_per_launch = (TN + algo.batch_size - 1) // algo.batch_size
        roof_lat = latency_roofline_wide(ms, steps_per_launch, kname)
    elif large_ms:
        # dominant kernel: the large-minibatch gradient kernel (csrc/mlp_large.hip, lb_grads_kernel), one launch
        # per optimizer step = one minibatch of forward + loss + backward at SURVEY.md 8(d)'s 52,352 FLOP per
        # sample (CartPole MLP, torch.utils.flop_counter), f32 MFMA peak.  Throughput-bound: the minibatch's
        # rows are spread over every CU (there is no dependent chain inside a launch)
        rows = T * N / nmb
        flops = 52352.0 * rows
        ms = float(np.mean(large_ms))
        tf = flops / (ms * 1e-3) / 1e12
        act = int(cfg["policy"].get("activation_fn", "tanh") == "relu")
        kname = "lb_grads_kernel<%d>" % act
        roofline = {"kernel": kname + " (rai_mlp_ppo_epoch, batch > 256: all-CU large-minibatch step)",
                    "bound": "mfma", "achieved": round(tf, 3), "peak": 157.3, "unit": "TFLOP/s",
                    "frac": round(tf / 157.3, 4), "traffic": traffic(kname), "traffic_source": traffic_source(kname),
                    "avg_ms": round(ms, 4), "flops_per_launch": flops, "rows_per_launch": rows,
                    "launches_timed": len(large_ms),
                    "epoch_ms": round(float(np.mean(epoch_ms)), 4) if epoch_ms else None}
        roof_lat = None
    elif epoch_ms:
        # dominant kernel: one fused PPO epoch per launch = T*N samples of forward+backward at
        # SURVEY.md 8(d)'s 52,352 FLOP/sample (CartPole MLP, torch.utils.flop_counter), f32 MFMA peak
        flops = 52352.0 * TN
        ms = float(np.mean(epoch_ms))
        tf = flops / (ms * 1e-3) / 1e12
        # the kernel rai_mlp_ppo_epoch dispatches for in_dim <= 4, n_actions <= 2 (csrc/mlp_ppo.hip
        # mlp_launch): G = 16 CUs per network unless RAI_MLP_CUS=8
        act = int(cfg["policy"].get("activation_fn", "tanh") == "relu")
        G = 8 if os.environ.get("RAI_MLP_CUS") == "8" else 16
        RC = 256 // G  # rows per CU (M8Geo<G, RC>)
        if G == 16 and algo.batch_size <= 128 and os.environ.get("RAI_MLP_PER_RANK_GEO") != "0":
            G, RC = 8, 16  # the per-rank geometry for <= 128-row minibatches (data parallel)
        kname = "mlp_ppo_mc8_kernel<%d, %d, %d>" % (act, G, RC)
        roofline = {"kernel": kname + f" (rai_mlp_ppo_epoch, {G} CUs per network)", "bound": "mfma",
                    "achieved": round(tf, 4), "peak": 157.3, "unit": "TFLOP/s", "frac": round(tf / 157.3, 6),
                    "traffic": traffic(kname), "traffic_source": traffic_source(kname), "avg_ms": round(ms, 3),
                    "flops_per_launch": flops, "launches_timed": len(epoch_ms)}
        roof_lat = latency_roofline(G, ms, (TN + algo.batch_size - 1) // algo.batch_size, kname)
    elif args.config in UPDATE_FLOPS:
        # no fused epoch kernel: the update's convolutions / GEMMs on MFMA (MIOpen, hipBLASLt) against
        # the f32 MFMA peak, from SURVEY.md 8(d)'s algorithmic FLOPs per env step (rollout forward +
        # n_epochs x forward/backward, torch.utils.flop_counter) and the measured update time;
        # per-kernel MFMA-busy PMC in profiles/r2k_pong_mfma_pmc_kernels.json (C3)
        fl = UPDATE_FLOPS[args.config] * T * N
        tf = fl / (elapsed / args.steps) / 1e12
        # traffic: L2-miss (fabric) bytes per update, 2 x FETCH_SIZE + WRITE_SIZE summed over the update's
        # kernels (tools/c3_pmc.sh + tools/c3_traffic.py; the newest profiles/r*_<config>_traffic.json)
        upd_traffic, traffic_src = None, None
        for tp in sorted((ROOT / "profiles").glob(f"r*_{args.config}_traffic.json"), reverse=True):
            td = json.loads(tp.read_text())
            if td.get("workload", "").startswith(workload):
                if td.get("lib_sha256") == lib_sha:  # counters collected on this very library
                    upd_traffic = td.get("bytes_per_update")
                    traffic_src = tp.name + (" (" + td["contractions"] + ")" if td.get("contractions") else "")
                else:
                    traffic_src = (f"{tp.name}: measured on another librai_amd.so build, not reported")
                break
        kname = "whole update (MIOpen / hipBLASLt contractions + HIP epilogues)"
        if args.config == "pong":
            from rl_algo_impls_amd import cnn_ops as _cnn
            if _cnn._CONV_MFMA:
                dgrad = ("weight + input gradients" if _cnn._CONV_MFMA_DGRAD
                         else "weight gradient, MIOpen input gradient")
                kname = (f"whole update (hand-written MFMA convolution forward + {dgrad}, hipBLASLt fc GEMMs, "
                         "HIP epilogues)")
        roofline = {"kernel": kname, "bound": "mfma",
                    "achieved": round(tf, 3), "peak": 157.3, "unit": "TFLOP/s", "frac": round(tf / 157.3, 4),
                    "traffic": upd_traffic, "traffic_source": traffic_src, "traffic_unit": "bytes per update",
                    "flops_per_update": fl}
        roof_lat = None
    else:
        roofline = roof_gae
        roof_lat = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "cartpole":
        cpu = cpu_baseline(args, N, T, dict(algo_kw, batch_size=algo.batch_size))

    if rank == 0:
        line = {
            "metric": "env-steps/sec (rollout+update) at 1/2/4/8 MI355X; GAE kernel HBM GB/s",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if split else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded host VecEnv with the config's obs/action shapes; random-init policy)",
            "config": {"workload": workload,
                       "global_batch": algo.global_batch_size if algo.dp_enabled else algo.batch_size,
                       "per_rank_batch": algo.batch_size,
                       "dp_batch": args.dp_batch, "env_partition": args.env_partition,
                       "global_num_envs": N * world,
                       "n_epochs": algo_kw["n_epochs"], "batch_policy": args.batch_policy, "seq_len": T,
                       "deterministic": bool(args.deterministic),
                       "miopen_find_mode": bool(torch.backends.cudnn.benchmark),
                       "miopen_user_db": os.environ.get("MIOPEN_USER_DB_PATH"),
                       "gemm_tunableop": bool(tunableop),
                       "parallelism": f"dp{world}"},
            "roofline": roofline,
            "roofline_latency": roof_lat,
            "roofline_gae": roof_gae,
            "roofline_gae_bandwidth_regime": roof_gae_large,
            "cpu_baseline": cpu,
            "lib_sha256": lib_sha,
        }
        if args.dp_rehearsal or world > 1:
            line["config"]["dp_update"] = algo.dp_update_mode
            if algo.dp_update_mode == "replicated":
                line["dp_path"] = ("replicated update: each rank steps its env share, one all-gather of the rollout "
                                   "per update (" + backend + "), the identical single-process update on every "
                                   "rank (strong scaling of the rollout only; the update is a dependent chain)")
            elif algo._xdp is not None and large_steps:
                line["dp_path"] = ("in-kernel cross-GPU exchange (IPC-mapped xGMI regions) inside each optimizer "
                                   "step's reduce launch; no host sync or RCCL call per step")
            elif algo._xdp is not None:
                line["dp_path"] = "in-kernel cross-GPU exchange (IPC-mapped xGMI regions), one launch per epoch"
            elif algo._dp_comm is not None and getattr(algo, "_buckets", None) is not None:
                line["dp_path"] = ("bucketed RCCL all-reduce per optimizer step on a side stream, overlapped with "
                                   "the backward, captured with the step's hipGraph")
            elif algo._dp_comm is not None:
                line["dp_path"] = "native RCCL loop (all-reduce per optimizer step)"
            else:
                line["dp_path"] = "python loop (" + backend + ")"
        print(json.dumps(line), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
