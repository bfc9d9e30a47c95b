"""Run setup of a training process — drop-in for rl_algo_impls/runner/running_utils.py:161-184.

The reference calls `set_seeds(seed)` then `set_device_optimizations(device, **device_hyperparams)`
before it builds the policy (rai/runner/train.py:87,102); `use_deterministic_algorithms` defaults to
True there (running_utils.py:164) and only the Lux YAML turns it off (ppo-LuxAI_S2.yml:4131).

On MI355X the switch reaches every kernel of the update:
  * this package's HIP kernels are deterministic by construction in both modes (fixed reduction
    orders, no float atomics: the in-L2 / cross-GPU gradient exchanges sum partials in CU / rank
    order, GAE is a serial chain per column);
  * PyTorch-ROCm ops (the NatureCNN / squeeze-U-Net convolutions on MIOpen, hipBLASLt GEMMs,
    index ops) follow torch.use_deterministic_algorithms, and torch.backends.cudnn.deterministic
    restricts MIOpen to solvers whose reductions have a fixed order (the implicit-GEMM backward
    solvers otherwise split K and accumulate with atomics into zero-filled outputs).

Measured cost on MI355X (C3, Pong NatureCNN, B = 256 minibatch step, graph-replayed): 0.554 ms per
step by default, 56.8 ms with the deterministic solvers (tools/replay_timing.py, profiles/
r2h_replay_timing.txt) — two orders of magnitude, so bench.py runs with --deterministic 0 and says
so in its JSON line; the reproducibility test pins the deterministic mode itself.

MIOpen records its solver choices per problem in a user database (~/.config/miopen): a
deterministic run would leave its slow solvers there for later default runs of the same shapes.
Deterministic mode therefore points MIOPEN_USER_DB_PATH (when the caller has not set it) at a
database of its own; like every MIOpen setting it only takes effect if it is set before the first
convolution of the process.
"""
from __future__ import annotations

import logging
import os
import random
from typing import Optional

import numpy as np
import torch


def set_device_optimizations(device: torch.device, set_float32_matmul_precision: Optional[str] = None,
                             use_deterministic_algorithms: bool = True) -> None:
    """running_utils.py:161-172, plus GEMM tuning when determinism is off (set_gemm_tuning) and the
    shipped MIOpen find database (seed_miopen_find_db)."""
    set_gemm_tuning(device, not use_deterministic_algorithms)
    torch.use_deterministic_algorithms(use_deterministic_algorithms)
    torch.backends.cudnn.deterministic = bool(use_deterministic_algorithms)
    if use_deterministic_algorithms and "MIOPEN_USER_DB_PATH" not in os.environ:
        os.environ["MIOPEN_USER_DB_PATH"] = os.path.join(os.path.expanduser("~"), ".cache", "rl_algo_impls_amd",
                                                         "miopen-deterministic")
    elif not use_deterministic_algorithms and torch.device(device).type == "cuda":
        seed_miopen_find_db()
    if torch.device(device).type == "cuda" and set_float32_matmul_precision:
        logging.info(f"Setting torch.set_float32_matmul_precision to {set_float32_matmul_precision}")
        torch.set_float32_matmul_precision(set_float32_matmul_precision)


MIOPEN_DB_SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")


def seed_miopen_find_db(dst: Optional[str] = None) -> Optional[str]:
    """Point MIOpen's user database at a directory seeded with the find / perf records this package ships
    (miopen_db/: MIOpen's find-mode solver timings for the squeeze-U-Net (C5) and NatureCNN (C3) problem
    shapes on gfx950 with 256 CUs, recorded by a bench run on MI355X).  Without them the first C5 update
    times every candidate solver of ~130 convolution problems: 534 s on a fresh box (profiles/
    r5d_c5_bench_stderr.txt), 543 s again in round 6 (r6c_c5_bench_stderr.txt); with them MIOpen reads
    the recorded choice and only compiles the chosen kernels.  MIOpen keys the files by architecture,
    CU count and its own version, so a different GPU or MIOpen build ignores them and searches as
    before.  Shipped files are copied (never overwriting) into dst = RAI_MIOPEN_DB_DIR or
    ~/.cache/rl_algo_impls_amd/miopen, since MIOpen appends to the user database.  Only when the caller
    has not set MIOPEN_USER_DB_PATH; like every MIOpen setting it must precede the first convolution of
    the process.  Returns the directory used (None: caller's own setting kept)."""
    if "MIOPEN_USER_DB_PATH" in os.environ:
        return None
    dst = dst or os.environ.get("RAI_MIOPEN_DB_DIR") or os.path.join(
        os.path.expanduser("~"), ".cache", "rl_algo_impls_amd", "miopen")
    try:
        os.makedirs(dst, exist_ok=True)
        import shutil

        for name in sorted(os.listdir(MIOPEN_DB_SHIPPED)) if os.path.isdir(MIOPEN_DB_SHIPPED) else []:
            if name.endswith(".txt") and not os.path.exists(os.path.join(dst, name)):
                shutil.copyfile(os.path.join(MIOPEN_DB_SHIPPED, name), os.path.join(dst, name))
    except OSError as e:  # an unwritable home: MIOpen's default database, a search on first use
        logging.warning(f"MIOpen find database not seeded ({e})")
        return None
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst


def set_gemm_tuning(device: torch.device, enabled: bool) -> bool:
    """PyTorch TunableOp for the library GEMMs the update leaves to PyTorch (C3: the NatureCNN fc layer's
    forward, dx and beta = 1 weight-gradient GEMMs; hipBLASLt's heuristic picks ran them at ~40
    TFLOP/s).  Each GEMM shape's hipBLASLt and rocBLAS solutions are timed once, at its first call, and
    the fastest is kept (C3: 147.2k -> 152.7-153.5k env-steps/s, profiles/r3zb_c3_blas_ab.txt).

    On only when deterministic mode is off: the pick is by timing, so it can differ between runs.
    RAI_TUNABLEOP=0 turns it off.  The picks are kept in a results file per device,
    RAI_TUNABLEOP_FILE or ~/.cache/rl_algo_impls_amd/tunableop_results<device>.csv, which later runs
    of the same user READ instead of re-tuning: delete it to re-tune (e.g. after a driver or library
    update).  Returns whether tuning is on."""
    if torch.device(device).type != "cuda":
        # a CPU run (the reference's CPU path) never touches the HIP runtime: torch.cuda.tunable raises
        # hipErrorNoDevice on a host without a GPU and would initialise HIP on one that has it
        return False
    on = bool(enabled) and os.environ.get("RAI_TUNABLEOP", "1") != "0"
    if on:
        path = os.environ.get("RAI_TUNABLEOP_FILE") or os.path.join(
            os.path.expanduser("~"), ".cache", "rl_algo_impls_amd", "tunableop_results%d.csv")
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        torch.cuda.tunable.set_filename(path)
        torch.cuda.tunable.set_max_tuning_duration(20)
    torch.cuda.tunable.enable(on)
    torch.cuda.tunable.tuning_enable(on)
    return on


def set_seeds(seed: Optional[int]) -> None:
    """running_utils.py:175-184 (the cuBLAS workspace variable is the reference's; hipBLASLt ignores it)."""
    if seed is None:
        return
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.backends.cudnn.benchmark = False
    os.environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"
    os.environ["TF_ENABLE_ONEDNN_OPTS"] = "0"
