"""PPO on MI355X — drop-in for rl_algo_impls/ppo/ppo.py:106-447.

Same constructor kwargs, same mutable attributes (learning_rate, clip_range,
ent_coef, gamma, gae_lambda, vf_coef, ... — what HyperparamTransitions and
LearningRateByKLDivergence set), same learn()/learn_epoch() contract, same
TrainStats and tensorboard tags, same `train/steps_per_second` definition
(wall time of learn_epoch before callbacks, ppo.py:221,422-427).

Per minibatch the work is: PyTorch-ROCm forward of the policy on a contiguous
slice of the permuted HBM rollout -> ONE fused HIP loss kernel (advantage
normalisation, clipped surrogate, value/entropy loss, gradients w.r.t. the
network outputs, stats row) -> PyTorch-ROCm backward seeded with those
gradients -> ONE fused clip_grad_norm_ + Adam step (two HIP launches) over the
flat parameter buffer.  No host synchronisation until the update ends.
"""
from __future__ import annotations

import ctypes as C
import gc
import logging
import os
from time import perf_counter
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .optim import FlatOptimizer, FlatParams
from .pg_common import (DeviceBlocks, TrainStats, launch_loss, load_optimizer, log_scalars, make_hparams,
                        num_or_array, save_optimizer, unsupported, value_columns)


class PPO:
    def __init__(self, policy, device: torch.device, tb_writer, learning_rate: float = 3e-4,
                 batch_size: int = 64, n_epochs: int = 10, gamma=0.99, gae_lambda=0.95, clip_range: float = 0.2,
                 clip_range_vf: Optional[float] = None, normalize_advantage: bool = True,
                 standardize_advantage: bool = False, ent_coef: float = 0.0, vf_coef=0.5,
                 ppo2_vf_coef_halving: bool = False, max_grad_norm: float = 0.5,
                 multi_reward_weights: Optional[List[float]] = None, gradient_accumulation: bool = False,
                 kl_cutoff: Optional[float] = None, freeze_policy_head: bool = False,
                 freeze_value_head: bool = False, freeze_backbone: bool = False, switch_range=None,
                 guide_probability=None, normalize_advantages_after_scaling: bool = False,
                 autocast_loss: bool = False, vf_loss_fn: str = "mse_loss", vf_weights=None,
                 teacher_kl_loss_coef=None, teacher_kl_loss_fn=None, teacher_loss_importance_sampling=True):
        unsupported(freeze_policy_head=freeze_policy_head, freeze_value_head=freeze_value_head,
                    freeze_backbone=freeze_backbone, switch_range=switch_range is not None,
                    guide_probability=guide_probability is not None, autocast_loss=autocast_loss,
                    teacher_kl_loss_coef=teacher_kl_loss_coef is not None)
        assert not (normalize_advantage and standardize_advantage), "Cannot both normalize and standardize advantage"
        self.policy = policy
        self.device = torch.device(device)
        self.tb_writer = tb_writer
        self.learning_rate = learning_rate
        cl = policy.channels_last_params() if self.device.type == "cuda" and hasattr(policy, "channels_last_params") else ()
        self.flat = FlatParams(policy, self.device, channels_last=cl)
        self.optimizer = FlatOptimizer(self.flat, FlatOptimizer.ADAM, lr=learning_rate, eps=1e-7,
                                       max_grad_norm=max_grad_norm)
        self.gamma = num_or_array(gamma)
        self.gae_lambda = num_or_array(gae_lambda)
        self.max_grad_norm = max_grad_norm
        self.clip_range = clip_range
        self.clip_range_vf = clip_range_vf
        self.normalize_advantage = normalize_advantage
        self.standardize_advantage = standardize_advantage
        self.ent_coef = ent_coef
        self.vf_coef = num_or_array(vf_coef)
        self.vf_weights = np.array(vf_weights) if vf_weights is not None else None
        self.ppo2_vf_coef_halving = ppo2_vf_coef_halving
        self.batch_size = batch_size
        self.n_epochs = n_epochs
        self.multi_reward_weights = np.array(multi_reward_weights) if multi_reward_weights else None
        self.gradient_accumulation = gradient_accumulation
        self.kl_cutoff = kl_cutoff
        self.normalize_advantages_after_scaling = normalize_advantages_after_scaling
        self.vf_loss_fn = vf_loss_fn
        self.blocks = DeviceBlocks(self.device)
        self.last_update_seconds: Optional[float] = None
        self.force_generic = False  # True: always use the per-minibatch (PyTorch network) path
        # generic path: capture the minibatch step into a hipGraph and replay it (graphs.py);
        # RAI_GRAPHS=0 keeps the eager loop
        self.use_graphs = os.environ.get("RAI_GRAPHS", "1") != "0"
        self._graphed = None
        # wide MLP actor-critics (HalfCheetah class): fused forward/backward kernels instead of the
        # PyTorch module + autograd (mlp_wide.py); RAI_WIDE=0 keeps the PyTorch network path
        self.use_wide = os.environ.get("RAI_WIDE", "1") != "0"
        self._wide = None
        self._wide_out: dict = {}
        # bench/profiling hook: when a list, (start, end) HIP events bracket every fused epoch launch
        self.kernel_events: Optional[list] = None
        self._mlp_ws: Optional[torch.Tensor] = None
        self.dp_group = None
        self.world = 1
        self._dp_comm = None
        self.dp_enabled = False  # enable_data_parallel() called (any world size, incl. 1-rank rehearsal)
        self.dp_batch = "per-rank"
        self.dp_update_mode = "exchange"  # or "replicated" (enable_data_parallel)
        self.global_batch_size = batch_size
        self._yaml_batch_size = batch_size  # enable_data_parallel derives the per-rank size from it
        self._buckets = None

    # -- data parallel (one process per GPU) ------------------------------------------------
    def enable_data_parallel(self, group=None, native_dp: bool = True, xdp: Optional[bool] = None,
                             dp_batch: str = "global", update_mode: Optional[str] = None) -> None:
        """Data parallelism: every rank owns its own env group and HBM rollout; a global
        minibatch is the union of the ranks' minibatch slices, gradients are summed over ranks
        with one all-reduce per optimizer step (RCCL over xGMI via torch.distributed, or the
        in-kernel exchange), and every rank applies the identical clip+Adam step.  The
        advantage normalisation uses global per-minibatch moments (one small all-reduce per
        epoch), reproducing the reference's normalisation over the whole (global) minibatch:
        on the fused MLP path through the kernels' moments argument, on the per-minibatch path
        through rai_ppo_hparams.ext_moments (per advantage column, or of the weighted advantage
        under normalize_advantages_after_scaling).

        dp_batch: "per-rank" — each rank takes batch_size rows per optimizer step (global
        minibatch batch_size x world); "global" — SURVEY.md 8(e)'s rule: batch_size / world rows
        per rank, so the global minibatch is batch_size (rl_algo_impls/ppo/ppo.py:314,
        rollout/vec_rollout.py:108-111) and the update equals the single-process one over the
        ranks' interleaved rollouts.

        update_mode: "exchange" — every optimizer step sums the ranks' gradients (in-kernel over the
        IPC-mapped regions, native RCCL loop, bucketed all-reduce or the Python loop, in that order of
        preference); "replicated" (dp_batch "global" only) — each rank steps its own env group, ONE
        all-gather per update assembles the rollout of the whole env group (GAE is per env column, so
        the local advantages / returns concatenate), and every rank runs the identical single-process
        update over it: bitwise the single-process update, with no cross-rank traffic inside the
        dependent optimizer-step chain; "auto" (default; RAI_DP_UPDATE overrides) — replicated where
        the update is a dependent chain of one-launch-per-epoch steps (the fused CartPole-class epoch
        kernel at <= 256 rows, the wide whole-epoch kernel), whose per-step cross-GPU hop costs more
        than the rows it spreads, exchange otherwise."""
        import torch.distributed as dist

        self.dp_group = group
        self.dp_enabled = True
        self.world = dist.get_world_size(group)
        if dp_batch not in ("per-rank", "global"):
            raise ValueError(f"dp_batch must be 'per-rank' or 'global', not {dp_batch!r}")
        self.dp_batch = dp_batch
        # idempotent: derived from the YAML batch_size every call, never from a previous division
        yaml_bs = self._yaml_batch_size
        self.batch_size = yaml_bs
        self.global_batch_size = yaml_bs * self.world
        if dp_batch == "global":
            if yaml_bs % self.world:
                raise ValueError(f"dp_batch='global': batch_size {yaml_bs} is not divisible by the "
                                 f"world size {self.world}")
            self.global_batch_size = yaml_bs
            self.batch_size = yaml_bs // self.world
        self._dp_comm = None
        self._xdp = None
        # the bucketed all-reduce closes over the communicator, and the captured minibatch-step
        # graphs over the buckets: both are rebuilt against the new communicator
        self._buckets = None
        self._graphed = None
        if update_mode is None:
            update_mode = os.environ.get("RAI_DP_UPDATE", "auto")
        if update_mode not in ("auto", "exchange", "replicated"):
            raise ValueError(f"update_mode must be 'auto', 'exchange' or 'replicated', not {update_mode!r}")
        if update_mode == "replicated" and dp_batch != "global":
            raise ValueError("update_mode='replicated' runs the single-process update over the whole env "
                             "group: it needs dp_batch='global'")
        self.dp_update_mode = "exchange"
        if update_mode != "exchange" and dp_batch == "global":
            self.batch_size = yaml_bs  # the single-process minibatch, for the path check below
            if update_mode == "replicated" or (self.world > 1 and self.flat.flat.is_cuda
                                               and self._dependent_chain_update()):
                self.dp_update_mode = "replicated"
            else:
                self.batch_size = yaml_bs // self.world
        if self.dp_update_mode == "replicated":
            self._broadcast_params(group)
            return
        if xdp is None:
            xdp = os.environ.get("RAI_XDP", "1") != "0"
        spec = self.fused_mlp_spec()
        # the CartPole-class fused epoch kernel (<= 256 rows per rank) and the large-minibatch steps (batch
        # policy (b): the exchange inside each step's reduce launch, mlp_large.hip)
        c2_xdp = (spec is not None and spec["in_dim"] <= 4
                  and (spec["n_act"] <= 2 if self.batch_size <= _lib.RAI_MLP_EPOCH_MAX_B else spec["n_act"] == 2))
        # the wide whole-epoch kernel (C4) keeps its one launch per epoch under data parallel too
        wide_xdp = spec is None and self._wide_epoch_options_ok() and self._wide_step() is not None
        if xdp and self.flat.flat.is_cuda and self.world > 1 and self.world <= 8 and (c2_xdp or wide_xdp):
            try:
                self._xdp = self._setup_xdp(group)
            except RuntimeError as e:  # e.g. IPC unavailable: fall back to the per-step RCCL loop
                logging.warning(f"in-kernel cross-GPU exchange unavailable ({e}); using the RCCL loop")
                self._xdp = None
        if self._xdp is None and self.flat.flat.is_cuda and dist.get_backend(group) == "nccl" and native_dp:
            self._dp_comm = self._native_comm(group)
        self._broadcast_params(group)

    def _broadcast_params(self, group) -> None:
        """Identical starting weights on every rank (rank 0's)."""
        import torch.distributed as dist

        with torch.no_grad():
            src = dist.get_global_rank(group, 0) if group is not None else 0
            if self.flat.flat.is_cuda and dist.get_backend(group) == "gloo":
                h = self.flat.flat.cpu()
                dist.broadcast(h, src=src, group=group)
                self.flat.flat.copy_(h)
            else:
                dist.broadcast(self.flat.flat, src=src, group=group)

    def _dependent_chain_update(self) -> bool:
        """True when this trainer's single-process update is a chain of one-launch-per-epoch dependent
        optimizer steps (rai_mlp_ppo_epoch's fused kernel at <= 256 rows, rai_mlp_wide_epoch): there a
        per-step cross-GPU exchange adds its hop to every step and shrinks nothing the step waits on."""
        spec = self.fused_mlp_spec()
        if spec is not None:
            return self.batch_size <= _lib.RAI_MLP_EPOCH_MAX_B
        return self._wide_epoch_options_ok() and self._wide_step() is not None

    def _replicated_rollout(self, r):
        """The rollout of the whole env group from every rank's own (T, N/R, ...) rollout: one all-gather
        per field (RCCL over xGMI; gloo through host memory), rank r's envs as columns [r N/R, (r+1) N/R).
        The epoch permutations must agree on every rank: a perm_source the caller injected is used as
        is, otherwise the shuffle keys derive from rank 0's next key (one 8-byte broadcast)."""
        import torch.distributed as dist

        from .rollout import DeviceRollout

        g, W = self.dp_group, self.world
        gloo = dist.get_backend(g) == "gloo"

        def gather(t):
            if t is None:
                return None
            src = t.contiguous()
            if gloo:
                h = src.cpu()
                parts = [torch.empty_like(h) for _ in range(W)]
                dist.all_gather(parts, h, group=g)
                out = torch.stack(parts).to(src.device)
            else:
                out = torch.empty((W,) + tuple(src.shape), dtype=src.dtype, device=src.device)
                dist.all_gather_into_tensor(out, src, group=g)
            return out.transpose(0, 1).reshape((src.shape[0], W * src.shape[1]) + tuple(src.shape[2:]))

        keys = None
        if r._perm_source is None:
            k = torch.tensor([r._perm_keys() if r._perm_keys is not None else 0], dtype=torch.int64)
            if not gloo:
                k = k.to(self.device)
            dist.broadcast(k, src=dist.get_global_rank(g, 0) if g is not None else 0, group=g)
            k0, count = int(k.item()), [0]

            def keys():
                count[0] += 1
                return (k0 * 0x9E3779B97F4A7C15 + count[0]) & (2**63 - 1)

        return DeviceRollout.from_fields(
            self.device, gather(r.obs), gather(r.actions), gather(r.values), gather(r.advantages),
            gather(r.returns), gather(r.logprobs), gather(r.action_masks), gather(r.num_actions),
            perm_keys=keys, perm_source=r._perm_source)

    def _setup_xdp(self, group) -> dict:
        """Exchange regions for the in-kernel cross-GPU all-reduce (rai_mlp_ppo_epoch_xdp): one
        uncached device region per rank, shared by IPC handle over `group`, mapped by every rank."""
        import ctypes as C

        import torch.distributed as dist

        L = _lib.lib()
        rank = dist.get_rank(group)

        def agreed(ok: bool) -> bool:
            # every rank learns whether every rank's local step succeeded, so a failure on one rank
            # turns into the same RuntimeError (and the RCCL-loop fallback) on all of them instead
            # of leaving the others blocked in the next collective
            f = torch.tensor([0 if ok else 1], dtype=torch.int64, device=self.device)
            if dist.get_backend(group) == "gloo":
                f = f.cpu()
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
            return int(f.item()) == 0

        nbytes = int(L.rai_xdp_region_bytes(self.world))
        region = C.c_void_p()
        torch.cuda.synchronize(self.device)
        hb = int(L.rai_xdp_handle_bytes())
        hbuf = (C.c_uint8 * hb)()
        ok = L.rai_xdp_alloc(nbytes, C.byref(region)) == 0 and L.rai_xdp_handle(region, hbuf, hb) == 0
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(hbuf) if ok else b"", group=group)
        def release(opened):
            for p in opened:
                L.rai_xdp_close(p)
            if region.value:
                L.rai_xdp_free(region)

        if not all(handles):
            release([])
            raise RuntimeError("cross-GPU exchange: region allocation / IPC export failed on some rank")
        ptrs, opened = [], []
        for r, h in enumerate(handles):
            if r == rank:
                ptrs.append(region.value)
                continue
            peer = C.c_void_p()
            if L.rai_xdp_open(h, C.byref(peer)) != 0:
                ok = False
                break
            opened.append(peer)
            ptrs.append(peer.value)
        if not agreed(ok):
            release(opened)
            raise RuntimeError("cross-GPU exchange: IPC mapping of a peer region failed on some rank")
        peers = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
        torch.cuda.synchronize(self.device)
        dist.barrier(group=group)  # every region zeroed and mapped before any kernel pushes into it
        # canary: the epoch kernel's memory, scopes and flag protocol on a known payload, on every rank
        bad = torch.zeros(2, dtype=torch.int32, device=self.device)
        if os.environ.get("RAI_XDP_INJECT_FAIL_RANK", "") == str(rank):
            rc = -1  # test hook: this rank's canary "fails" without launching (its partners time out)
        else:
            rc = L.rai_xdp_selftest(peers.data_ptr(), self.world, rank, 1, bad.data_ptr(),
                                    _lib.stream_handle(self.device))
        torch.cuda.synchronize(self.device)
        verdict = bad.to(torch.int64)
        if rc != 0:  # a launch failure joins the verdict instead of raising on this rank alone
            verdict[0] += 1
        if dist.get_backend(group) == "gloo":
            verdict = verdict.cpu()
        dist.all_reduce(verdict, op=dist.ReduceOp.MAX, group=group)
        if int(verdict.sum()) != 0:
            release(opened)
            raise RuntimeError(f"cross-GPU exchange self-test failed (wrong values, timeouts) = {verdict.tolist()}")
        return dict(region=region, opened=opened, peers=peers, rank=rank, step=0)

    def _params_agree(self) -> bool:
        """Cheap cross-rank consistency check of the (bitwise-identical by construction) weights."""
        import torch.distributed as dist

        v = self.flat.flat.double()
        t = torch.stack([v.sum(), (v * v).sum(), -v.sum(), -(v * v).sum()])
        if dist.get_backend(self.dp_group) == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.dp_group)
        return bool((t[0] == -t[2]) and (t[1] == -t[3]))

    def _native_comm(self, group):
        """An RCCL communicator of our own (same ranks as `group`) for the natively driven
        per-minibatch loop (rai_mlp_ppo_epoch_dp); the unique id travels over `group`."""
        import ctypes as C

        import torch.distributed as dist

        L = _lib.lib()
        if not L.rai_dp_available():
            raise RuntimeError("librccl.so.1 is not mapped in this process: native data parallelism unavailable")
        uid = torch.zeros(_lib.RAI_DP_UID_BYTES, dtype=torch.uint8)
        if dist.get_rank(group) == 0:
            buf = (C.c_uint8 * _lib.RAI_DP_UID_BYTES)()
            _lib.check(L.rai_dp_unique_id(buf, _lib.RAI_DP_UID_BYTES), "rai_dp_unique_id")
            uid.copy_(torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8))
        dev_uid = uid.to(self.device)
        dist.broadcast(dev_uid, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        raw = bytes(dev_uid.cpu().numpy().tobytes())
        comm = C.c_void_p()
        torch.cuda.synchronize(self.device)
        _lib.check(L.rai_dp_comm_init(C.byref(comm), raw, self.world, dist.get_rank(group)), "rai_dp_comm_init")
        return comm

    def _all_reduce(self, t: torch.Tensor, average: bool = False) -> None:
        import torch.distributed as dist

        if t.is_cuda and dist.get_backend(self.dp_group) == "gloo":  # test/rehearsal backend
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.dp_group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.dp_group)  # RCCL over xGMI
        if average:
            t.mul_(1.0 / self.world)

    def _global_adv_moments(self, adv: torch.Tensor, nmb: int) -> torch.Tensor:
        """(mean, den) of every global minibatch of this epoch, per advantage column (or of the
        multi_reward_weights-weighted advantage under normalize_advantages_after_scaling):
        local per-minibatch (count, sum, sum of squares) in fp64, one all-reduce, unbiased std
        (ppo.py:307-318).  Returns (nmb, columns, 2) f32; the loss kernel applies the
        normalize / standardize rule itself."""
        B = self.batch_size
        a = adv.double()
        a = a.reshape(a.shape[0], -1)
        if self.normalize_advantages_after_scaling:
            w = self.multi_reward_weights
            if w is not None:
                a = (a.float() * torch.as_tensor(np.asarray(w, np.float32), device=a.device)).sum(1, keepdim=True)
                a = a.double()
            else:
                a = a[:, :1]
        rows, kc = a.shape
        n_full = rows // B
        full = a[:n_full * B].view(n_full, B, kc)
        parts = [torch.stack([torch.full((n_full, kc), float(B), dtype=torch.float64, device=a.device),
                              full.sum(1), (full ** 2).sum(1)], -1)]
        if n_full < nmb:
            tail = a[n_full * B:]
            parts.append(torch.stack([torch.full((kc,), float(tail.shape[0]), dtype=torch.float64, device=a.device),
                                      tail.sum(0), (tail ** 2).sum(0)], -1).view(1, kc, 3))
        m = torch.cat(parts, 0)
        self._all_reduce(m)
        n, s1, s2 = m[..., 0], m[..., 1], m[..., 2]
        mean = s1 / n
        std = torch.sqrt(torch.clamp(s2 - n * mean * mean, min=0.0) / (n - 1)).float()
        out = torch.empty((nmb, kc, 2), dtype=torch.float32, device=a.device)
        out[..., 0] = mean.float()
        out[..., 1] = std + 1e-8
        return out.contiguous()

    def _update_fused_dp(self, r, spec) -> Tuple[np.ndarray, np.ndarray, int]:
        nmb = r.num_minibatches(self.batch_size)
        n_steps = self.n_epochs * nmb
        blocks = self.blocks
        blocks.ensure_tables(n_steps, n_steps)
        blocks.upload(self._hparams(1, nmb), self.optimizer.step_count)
        self._ensure_mlp_workspace(r.total_steps)
        opt = self.optimizer
        L = _lib.lib()
        st = _lib.stream_handle(self.device)
        for _ in range(self.n_epochs):
            b = r.epoch_batch(shuffle=True)
            moments = self._global_adv_moments(b.advantages, nmb).view(nmb, 2)
            # the fused epoch kernels apply A = (A - mean) / den as given: encode the reference's rule
            if not self.normalize_advantage:
                moments[:, 0] = 0.0
                if not self.standardize_advantage:
                    moments[:, 1] = 1.0
            obs = (b.obs if b.obs.dtype == torch.float32 else b.obs.float()).contiguous()
            acts = b.actions.contiguous()
            if self._xdp is not None:  # one launch per epoch, cross-GPU sums inside the kernel
                x = self._xdp
                f = self.flat
                ev = None
                if self.kernel_events is not None:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()
                rc = L.rai_mlp_ppo_epoch_xdp(
                    f.flat.data_ptr(), opt.state1.data_ptr(), opt.state2.data_ptr(), obs.data_ptr(), acts.data_ptr(),
                    b.logprobs.data_ptr(), b.values.data_ptr(), b.advantages.data_ptr(), b.returns.data_ptr(),
                    r.total_steps, self.batch_size, moments.data_ptr(), self.world, x["rank"],
                    x["peers"].data_ptr(), x["step"], spec["in_dim"], 64, spec["n_act"], spec["activation"],
                    blocks.hp.data_ptr(), opt.hp_dev.data_ptr(), blocks.state.data_ptr(), blocks.stats.data_ptr(),
                    int(blocks.stats.shape[0]), blocks.norms.data_ptr(), int(blocks.norms.shape[0]),
                    self._mlp_ws.data_ptr(), self._mlp_ws.numel(), st)
                _lib.check(rc, "rai_mlp_ppo_epoch_xdp")
                if ev is not None:
                    ev[1].record()
                    self.kernel_events.append(ev)
                x["step"] += nmb
                opt.step_count += nmb
                continue
            if self._dp_comm is not None:  # natively driven: grads -> RCCL all-reduce -> clip+Adam
                f = self.flat
                if getattr(self, "_grad_alt", None) is None or self._grad_alt.numel() != f.P:
                    self._grad_alt = torch.zeros_like(f.grad)
                rc = L.rai_mlp_ppo_epoch_dp(
                    f.flat.data_ptr(), f.grad.data_ptr(), opt.state1.data_ptr(), opt.state2.data_ptr(), f.P,
                    obs.data_ptr(), acts.data_ptr(), b.logprobs.data_ptr(), b.values.data_ptr(),
                    b.advantages.data_ptr(), b.returns.data_ptr(), r.total_steps, self.batch_size,
                    moments.data_ptr(), self.world, spec["in_dim"], 64, spec["n_act"], spec["activation"],
                    blocks.hp.data_ptr(), opt.hp_dev.data_ptr(), blocks.state.data_ptr(), blocks.stats.data_ptr(),
                    int(blocks.stats.shape[0]), blocks.norms.data_ptr(), int(blocks.norms.shape[0]), self._dp_comm,
                    self._grad_alt.data_ptr(), self._mlp_ws.data_ptr(), self._mlp_ws.numel(),
                    opt.workspace.data_ptr(), opt.workspace.numel(), st)
                _lib.check(rc, "rai_mlp_ppo_epoch_dp")
                opt.step_count += nmb
                continue
            for i in range(nmb):
                rc = L.rai_mlp_ppo_grads(
                    self.flat.flat.data_ptr(), obs.data_ptr(), acts.data_ptr(), b.logprobs.data_ptr(),
                    b.values.data_ptr(), b.advantages.data_ptr(), b.returns.data_ptr(), r.total_steps,
                    self.batch_size, i, 1, moments.data_ptr(), self.world, spec["in_dim"], 64, spec["n_act"],
                    spec["activation"], blocks.hp.data_ptr(), opt.hp_dev.data_ptr(), blocks.state.data_ptr(),
                    self.flat.grad.data_ptr(), blocks.stats.data_ptr(), int(blocks.stats.shape[0]),
                    self._mlp_ws.data_ptr(), self._mlp_ws.numel(), st)
                _lib.check(rc, "rai_mlp_ppo_grads")
                self._all_reduce(self.flat.grad)
                opt.step(blocks.state, blocks.norms)
        stats_t = blocks.stats[:n_steps].clone()
        self._all_reduce(stats_t)  # every rank holds its share of the global means
        host = torch.cat([stats_t.reshape(-1), blocks.norms[:n_steps],
                          blocks.state.view(torch.float32)]).cpu().numpy()
        stats = host[: n_steps * _lib.RAI_STAT_STRIDE].reshape(n_steps, _lib.RAI_STAT_STRIDE).copy()
        norms = host[n_steps * _lib.RAI_STAT_STRIDE: n_steps * _lib.RAI_STAT_STRIDE + n_steps]
        state = host[n_steps * _lib.RAI_STAT_STRIDE + n_steps:].view(np.int32)
        if state[5] != 0:
            raise RuntimeError("fused data-parallel update: a device-side exchange timed out (err flag set)")
        if self._xdp is not None and not self._params_agree():
            raise RuntimeError("ranks' parameters diverged after the in-kernel cross-GPU exchange")
        stats[:, 0] += float(self.vf_coef) * stats[:, 5]
        return stats, norms, 1

    # -- reference API -------------------------------------------------------------------
    def learn(self, train_timesteps: int, rollout_generator, callbacks=None, total_timesteps=None,
              start_timesteps: int = 0) -> "PPO":
        if total_timesteps is None:
            total_timesteps = train_timesteps
        assert start_timesteps + train_timesteps <= total_timesteps
        timesteps_elapsed = start_timesteps
        while timesteps_elapsed < start_timesteps + train_timesteps:
            timesteps_elapsed, should_continue = self.learn_epoch(timesteps_elapsed, total_timesteps,
                                                                  rollout_generator, callbacks)
            gc.collect()
            if not should_continue:
                break
        return self

    def _hparams(self, K: int, num_minibatches: int):
        return make_hparams(
            loss_kind=0, K=K, clip_range=self.clip_range, clip_range_vf=self.clip_range_vf,
            ent_coef=self.ent_coef, vf_coef=self.vf_coef, vf_weights=self.vf_weights,
            multi_reward_weights=self.multi_reward_weights, normalize_advantage=self.normalize_advantage,
            standardize_advantage=self.standardize_advantage,
            normalize_after_scaling=self.normalize_advantages_after_scaling,
            ppo2_vf_coef_halving=self.ppo2_vf_coef_halving, kl_cutoff=self.kl_cutoff, vf_loss_fn=self.vf_loss_fn,
            grad_scale=(1.0 / num_minibatches) if self.gradient_accumulation else 1.0)

    def learn_epoch(self, timesteps_elapsed: int, total_timesteps: int, rollout_generator,
                    callbacks=None) -> Tuple[int, bool]:
        start_time = perf_counter()
        self.optimizer.param_groups[0]["lr"] = self.learning_rate  # update_learning_rate (schedule.py:64-66)
        self.optimizer.max_grad_norm = self.max_grad_norm
        self.optimizer.sync_hparams()
        chart = {"learning_rate": self.learning_rate, "ent_coef": self.ent_coef, "pi_clip": self.clip_range,
                 "gamma": self.gamma, "gae_lambda": self.gae_lambda, "vf_coef": self.vf_coef}
        if self.clip_range_vf is not None:
            chart["v_clip"] = self.clip_range_vf
        if self.multi_reward_weights is not None:
            chart["reward_weights"] = self.multi_reward_weights
        if self.vf_weights is not None:
            chart["vf_weights"] = self.vf_weights
        log_scalars(self.tb_writer, "charts", chart, timesteps_elapsed)

        r = rollout_generator.rollout(gamma=self.gamma, gae_lambda=self.gae_lambda)
        self.last_rollout_seconds = perf_counter() - start_time  # host env + policy steps (synced per step)
        timesteps_elapsed += r.total_steps
        stats, norms, K = self.update(r)
        ru = getattr(self, "last_update_rollout", None) or r  # the whole env group's under replicated DP
        explained_var = ru.explained_variance()
        train_stats = self._train_stats(stats, norms, K, ru.num_minibatches(self.batch_size), explained_var)
        train_stats.write_to_tensorboard(self.tb_writer)
        end_time = perf_counter()
        self.last_update_seconds = end_time - start_time
        if self.tb_writer is not None:
            self.tb_writer.add_scalar("train/steps_per_second", r.total_steps / (end_time - start_time))
            if hasattr(self.tb_writer, "on_steps"):
                self.tb_writer.on_steps(r.total_steps)
        self.last_train_stats = train_stats
        if callbacks:
            if not all(c.on_step(timesteps_elapsed=r.total_steps, train_stats=train_stats) for c in callbacks):
                logging.info(f"Callback terminated training at {timesteps_elapsed} timesteps")
                return timesteps_elapsed, False
        return timesteps_elapsed, True

    # -- fused MLP path ---------------------------------------------------------------------
    def fused_mlp_spec(self) -> Optional[dict]:
        """Shape descriptor if the policy/options fit rai_mlp_ppo_epoch (CartPole-class MLP
        actor-critic: Flatten encoder, [in -> 64 -> 64 -> out] actor and critic, Categorical
        head); None otherwise (the generic per-minibatch path then runs)."""
        from .policy import mlp_actor_critic_spec

        if self.force_generic:
            return None
        spec = mlp_actor_critic_spec(self.policy)
        if spec is None or self.batch_size < 2:
            return None
        # > 256 rows per minibatch (SURVEY 8(d) batch policy (b)): the all-CU large-minibatch kernels of
        # rai_mlp_ppo_epoch / rai_mlp_ppo_grads (csrc/mlp_large.hip) cover in_dim <= 4, two actions
        if self.batch_size > _lib.RAI_MLP_EPOCH_MAX_B and not (spec["in_dim"] <= 4 and spec["n_act"] == 2):
            return None
        if (self.gradient_accumulation or self.kl_cutoff is not None or self.multi_reward_weights is not None
                or self.vf_weights is not None or self.normalize_advantages_after_scaling
                or np.ndim(self.vf_coef) > 0):
            return None
        return spec

    def _ensure_mlp_workspace(self, n_rows: int) -> None:
        need = int(_lib.lib().rai_mlp_ppo_workspace_bytes(n_rows, self.batch_size))
        if self._mlp_ws is None or self._mlp_ws.numel() < need:
            self._mlp_ws = torch.zeros(need, dtype=torch.uint8, device=self.device)

    def _update_fused(self, r, spec) -> Tuple[np.ndarray, np.ndarray, int]:
        nmb = r.num_minibatches(self.batch_size)
        if r.total_steps % self.batch_size == 1:
            raise ValueError("a 1-row minibatch has no unbiased std (reference would produce NaN)")
        n_steps = self.n_epochs * nmb
        blocks = self.blocks
        blocks.ensure_tables(n_steps, n_steps)
        blocks.upload(self._hparams(1, nmb), self.optimizer.step_count)
        self._ensure_mlp_workspace(r.total_steps)
        opt = self.optimizer
        L = _lib.lib()
        st = _lib.stream_handle(self.device)
        # Epoch k + 1's permutation and gather (rai_feistel_permutation + one gather) run on a
        # side stream into the other of two permuted copies while epoch k's kernel (32 CUs) runs, so
        # the 20 launches follow each other without them.  Same permutations: the shuffle keys are
        # drawn on the host in the same order.
        cur = torch.cuda.current_stream(self.device)
        two_slots = hasattr(r, "alloc_epoch_buffers")  # DeviceRollout; other rollouts: in order
        side = self._epoch_prep_stream() if two_slots else cur
        if two_slots:
            for slot in (0, 1):
                r.alloc_epoch_buffers(slot)
            side.wait_stream(cur)  # the rollout, its GAE and the parameters are ready

        def prep(k):
            with torch.cuda.stream(side):
                bk = r.epoch_batch(shuffle=True, slot=k % 2) if two_slots else r.epoch_batch(shuffle=True)
                assert bk.logprobs is not None, "PPO needs rollout logprobs (include_logp=True)"
                obs_k = bk.obs if bk.obs.dtype == torch.float32 else bk.obs.float()
                obs_k = obs_k.contiguous()
                if obs_k.data_ptr() != bk.obs.data_ptr():
                    obs_k.record_stream(cur)
                ready = torch.cuda.Event()
                ready.record(side)
            return bk, obs_k, ready

        nxt = prep(0)
        done: List[torch.cuda.Event] = []
        for k in range(self.n_epochs):
            b, obs, ready = nxt
            cur.wait_event(ready)
            ev = None
            if self.kernel_events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            rc = L.rai_mlp_ppo_epoch(
                self.flat.flat.data_ptr(), opt.state1.data_ptr(), opt.state2.data_ptr(), obs.contiguous().data_ptr(),
                b.actions.contiguous().data_ptr(), b.logprobs.data_ptr(), b.values.data_ptr(),
                b.advantages.data_ptr(), b.returns.data_ptr(), r.total_steps, self.batch_size, spec["in_dim"], 64,
                spec["n_act"], spec["activation"], blocks.hp.data_ptr(), opt.hp_dev.data_ptr(),
                blocks.state.data_ptr(), blocks.stats.data_ptr(), int(blocks.stats.shape[0]),
                blocks.norms.data_ptr(), int(blocks.norms.shape[0]), self._mlp_ws.data_ptr(), self._mlp_ws.numel(),
                st)
            _lib.check(rc, "rai_mlp_ppo_epoch")
            if ev is not None:
                ev[1].record()
                self.kernel_events.append(ev)
            opt.step_count += nmb
            done.append(torch.cuda.Event())
            done[-1].record(cur)
            if k + 1 < self.n_epochs:
                if k >= 1 and two_slots:
                    side.wait_event(done[k - 1])  # slot (k + 1) % 2 was read by epoch k - 1
                nxt = prep(k + 1)
        cur.wait_stream(side)
        host = torch.cat([blocks.stats[:n_steps].reshape(-1), blocks.norms[:n_steps],
                          blocks.state.view(torch.float32)]).cpu().numpy()
        stats = host[: n_steps * _lib.RAI_STAT_STRIDE].reshape(n_steps, _lib.RAI_STAT_STRIDE).copy()
        norms = host[n_steps * _lib.RAI_STAT_STRIDE: n_steps * _lib.RAI_STAT_STRIDE + n_steps]
        state = host[n_steps * _lib.RAI_STAT_STRIDE + n_steps:].view(np.int32)
        if state[5] != 0:
            raise RuntimeError("rai_mlp_ppo_epoch: device-side exchange timed out (err flag set)")
        stats[:, 0] += float(self.vf_coef) * stats[:, 5]  # value term of the loss
        return stats, norms, 1

    def _wide_epoch_options_ok(self) -> bool:
        """The options rai_mlp_wide_epoch covers: K = 1, Adam, minibatches of 2..64 rows (per rank), no
        gradient accumulation / kl_cutoff / multi-reward weights / vf_weights."""
        if os.environ.get("RAI_WIDE_EPOCH", "1") == "0":
            return False
        if (self.gradient_accumulation or self.kl_cutoff is not None or self.multi_reward_weights is not None
                or self.vf_weights is not None or self.normalize_advantages_after_scaling
                or np.ndim(self.vf_coef) > 0 or self.optimizer.kind != self.optimizer.ADAM):
            return False
        return 2 <= self.batch_size <= 64

    def _wide_epoch_step(self, r):
        """The WideStep (descriptor) when the whole epoch can run as ONE persistent launch
        (rai_mlp_wide_epoch): a wide-MLP policy within _wide_epoch_options_ok, single process or data
        parallel over the in-kernel cross-GPU exchange (rai_mlp_wide_epoch_xdp).
        RAI_WIDE_EPOCH=0 keeps the graph-replayed per-minibatch path."""
        if not hasattr(r, "epoch_batch") or (self.dp_enabled and self._xdp is None):
            return None
        if not self._wide_epoch_options_ok():
            return None
        if r.total_steps < 2 or (not self.dp_enabled and r.total_steps % self.batch_size == 1):
            return None
        return self._wide_step()

    def _update_wide_epoch(self, r, wide) -> Tuple[np.ndarray, np.ndarray, int]:
        """One rai_mlp_wide_epoch launch per epoch over the epoch's permuted rollout copy; epoch
        k + 1's permutation and gather are prepared on a side stream while epoch k runs (as
        _update_fused)."""
        nmb = r.num_minibatches(self.batch_size)
        n_steps = self.n_epochs * nmb
        blocks = self.blocks
        blocks.ensure_tables(n_steps, n_steps)
        blocks.upload(self._hparams(1, nmb), self.optimizer.step_count)
        opt = self.optimizer
        L = _lib.lib()
        st = _lib.stream_handle(self.device)
        ws_bytes = int(L.rai_mlp_wide_epoch_workspace_bytes(wide.spec["hidden"], wide.desc.in_dim, r.total_steps))
        if getattr(self, "_we_ws", None) is None or self._we_ws.numel() < ws_bytes:
            self._we_ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=self.device)
        cur = torch.cuda.current_stream(self.device)
        two_slots = hasattr(r, "alloc_epoch_buffers")
        side = self._epoch_prep_stream() if two_slots else cur
        if two_slots:
            for slot in (0, 1):
                r.alloc_epoch_buffers(slot)
            side.wait_stream(cur)

        def prep(k):
            with torch.cuda.stream(side):
                bk = r.epoch_batch(shuffle=True, slot=k % 2) if two_slots else r.epoch_batch(shuffle=True)
                assert bk.logprobs is not None, "PPO needs rollout logprobs (include_logp=True)"
                obs_k = bk.obs if bk.obs.dtype == torch.float32 else bk.obs.float()
                obs_k = obs_k.contiguous()
                if obs_k.data_ptr() != bk.obs.data_ptr():
                    obs_k.record_stream(cur)
                ready = torch.cuda.Event()
                ready.record(side)
            return bk, obs_k, ready

        f = self.flat
        nxt = prep(0)
        done: List[torch.cuda.Event] = []
        for k in range(self.n_epochs):
            b, obs, ready = nxt
            cur.wait_event(ready)
            ev = None
            if self.kernel_events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            rc = L.rai_mlp_wide_epoch(
                C.byref(wide.desc), f.flat.data_ptr(), opt.state1.data_ptr(), opt.state2.data_ptr(), f.P,
                obs.data_ptr(), b.actions.contiguous().data_ptr(), b.logprobs.data_ptr(), b.values.data_ptr(),
                b.advantages.data_ptr(), b.returns.data_ptr(), r.total_steps, self.batch_size, blocks.hp.data_ptr(),
                opt.hp_dev.data_ptr(), blocks.state.data_ptr(), blocks.stats.data_ptr(), int(blocks.stats.shape[0]),
                blocks.norms.data_ptr(), int(blocks.norms.shape[0]), self._we_ws.data_ptr(), self._we_ws.numel(), st)
            _lib.check(rc, "rai_mlp_wide_epoch")
            if ev is not None:
                ev[1].record()
                self.kernel_events.append(ev)
            opt.step_count += nmb
            done.append(torch.cuda.Event())
            done[-1].record(cur)
            if k + 1 < self.n_epochs:
                if k >= 1 and two_slots:
                    side.wait_event(done[k - 1])
                nxt = prep(k + 1)
        cur.wait_stream(side)
        host = torch.cat([blocks.stats[:n_steps].reshape(-1), blocks.norms[:n_steps],
                          blocks.state.view(torch.float32)]).cpu().numpy()
        stats = host[: n_steps * _lib.RAI_STAT_STRIDE].reshape(n_steps, _lib.RAI_STAT_STRIDE).copy()
        norms = host[n_steps * _lib.RAI_STAT_STRIDE: n_steps * _lib.RAI_STAT_STRIDE + n_steps]
        state = host[n_steps * _lib.RAI_STAT_STRIDE + n_steps:].view(np.int32)
        if state[5] != 0:
            raise RuntimeError("rai_mlp_wide_epoch: a device-side hand-off timed out (err flag set)")
        stats[:, 0] += float(self.vf_coef) * stats[:, 5]  # value term of the loss
        return stats, norms, 1

    def _update_wide_epoch_xdp(self, r, wide) -> Tuple[np.ndarray, np.ndarray, int]:
        """Data-parallel whole-epoch form (rai_mlp_wide_epoch_xdp): per epoch the permuted copy, the global
        minibatches' advantage moments (one small all-reduce) and ONE launch whose workgroups sum their
        owned gradients over the ranks inside the kernel; stats rows summed over the ranks after."""
        nmb = r.num_minibatches(self.batch_size)
        n_steps = self.n_epochs * nmb
        blocks = self.blocks
        blocks.ensure_tables(n_steps, n_steps)
        blocks.upload(self._hparams(1, nmb), self.optimizer.step_count)
        opt = self.optimizer
        L = _lib.lib()
        st = _lib.stream_handle(self.device)
        ws_bytes = int(L.rai_mlp_wide_epoch_workspace_bytes(wide.spec["hidden"], wide.desc.in_dim, r.total_steps))
        if getattr(self, "_we_ws", None) is None or self._we_ws.numel() < ws_bytes:
            self._we_ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=self.device)
        f = self.flat
        x = self._xdp
        for _ in range(self.n_epochs):
            b = r.epoch_batch(shuffle=True)
            assert b.logprobs is not None, "PPO needs rollout logprobs (include_logp=True)"
            moments = self._global_adv_moments(b.advantages, nmb).view(nmb, 2)
            if not self.normalize_advantage:  # the kernel applies A = (A - mean) / den as given
                moments[:, 0] = 0.0
                if not self.standardize_advantage:
                    moments[:, 1] = 1.0
            obs = (b.obs if b.obs.dtype == torch.float32 else b.obs.float()).contiguous()
            ev = None
            if self.kernel_events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            rc = L.rai_mlp_wide_epoch_xdp(
                C.byref(wide.desc), f.flat.data_ptr(), opt.state1.data_ptr(), opt.state2.data_ptr(), f.P,
                obs.data_ptr(), b.actions.contiguous().data_ptr(), b.logprobs.data_ptr(), b.values.data_ptr(),
                b.advantages.data_ptr(), b.returns.data_ptr(), r.total_steps, self.batch_size, moments.data_ptr(),
                self.world, x["rank"], x["peers"].data_ptr(), x["step"], blocks.hp.data_ptr(), opt.hp_dev.data_ptr(),
                blocks.state.data_ptr(), blocks.stats.data_ptr(), int(blocks.stats.shape[0]), blocks.norms.data_ptr(),
                int(blocks.norms.shape[0]), self._we_ws.data_ptr(), self._we_ws.numel(), st)
            _lib.check(rc, "rai_mlp_wide_epoch_xdp")
            if ev is not None:
                ev[1].record()
                self.kernel_events.append(ev)
            x["step"] += nmb
            opt.step_count += nmb
        stats_t = blocks.stats[:n_steps].clone()
        self._all_reduce(stats_t)  # every rank holds its share of the global means
        host = torch.cat([stats_t.reshape(-1), blocks.norms[:n_steps], blocks.state.view(torch.float32)]).cpu().numpy()
        stats = host[: n_steps * _lib.RAI_STAT_STRIDE].reshape(n_steps, _lib.RAI_STAT_STRIDE).copy()
        norms = host[n_steps * _lib.RAI_STAT_STRIDE: n_steps * _lib.RAI_STAT_STRIDE + n_steps]
        state = host[n_steps * _lib.RAI_STAT_STRIDE + n_steps:].view(np.int32)
        if state[5] != 0:
            raise RuntimeError("rai_mlp_wide_epoch_xdp: a device-side hand-off timed out (err flag set)")
        if not self._params_agree():
            raise RuntimeError("ranks' parameters diverged after the in-kernel cross-GPU exchange")
        stats[:, 0] += float(self.vf_coef) * stats[:, 5]
        return stats, norms, 1

    def _epoch_prep_stream(self) -> torch.cuda.Stream:
        if getattr(self, "_prep_stream", None) is None:
            self._prep_stream = torch.cuda.Stream(self.device)
        return self._prep_stream

    def _wide_step(self):
        """The wide-MLP fused step for this policy, or None (structure / options not covered)."""
        if self.force_generic or not self.use_wide or not self.flat.flat.is_cuda:
            return None
        if self._wide is None:
            from .mlp_wide import WideStep, wide_mlp_spec

            if wide_mlp_spec(self.policy) is None or not (1 <= self.batch_size <= _lib.RAI_WIDE_MAX_B):
                self._wide = False
            else:
                self._wide = WideStep(self.policy, self.device, accumulate=self.gradient_accumulation)
        if self._wide is False:
            return None
        self._wide.check_pointers()
        return self._wide

    def _minibatch_loss_grads(self, wide, obs, actions, masks, values, adv, ret, logprobs, K_box,
                              obs_prepared: bool = False) -> None:
        """Forward, fused loss and backward of one minibatch into the flat gradient buffer: the
        wide-MLP kernels when available, else the PyTorch network + autograd (NatureCNN layers
        with the cnn_ops epilogues accumulating straight into the flat gradient views)."""
        if wide is not None and masks is None:
            B = int(obs.shape[0])
            outs = self._wide_out.get(B)
            if outs is None:
                outs = self._wide_out[B] = wide.outputs(B)
            logp, ent, v = outs
            K_box[0] = 1
            d_logp, d_ent, d_v = wide.forward_loss(obs, actions, logp, ent, v, self.blocks, logprobs, values, adv,
                                                   ret)
            wide.backward(obs, actions, d_logp, d_ent, d_v)
            return
        from .cnn_ops import direct_grads

        with direct_grads(self.flat.flat.is_cuda):
            if obs_prepared:
                logp, ent, v = self.policy(obs, actions, action_masks=masks, obs_prepared=True)
            else:
                logp, ent, v = self.policy(obs, actions, action_masks=masks)
            if K_box[0] is None:
                K_box[0] = value_columns(v)
            d_logp, d_ent, d_v = launch_loss(self.blocks, logp, ent, v, logprobs, values, adv, ret, K_box[0])
            torch.autograd.backward([logp, ent, v], [d_logp, d_ent, d_v])

    def update(self, r) -> Tuple[np.ndarray, np.ndarray, int]:
        """All epochs x minibatches of one update, enqueued without host syncs;
        returns the per-minibatch stats rows and grad norms (one D2H copy)."""
        self.last_update_rollout = r
        if self.dp_enabled and self.dp_update_mode == "replicated":
            # data parallel by replication: the whole env group's rollout on every rank, then the
            # single-process update (no exchange inside it); the ranks' weights are checked equal after
            g = self._replicated_rollout(r)
            self.last_update_rollout = g
            self.dp_enabled = False
            try:
                out = self.update(g)
            finally:
                self.dp_enabled = True
                self.last_update_rollout = g
            if self.world > 1 and not self._params_agree():
                raise RuntimeError("ranks' parameters diverged under the replicated data-parallel update")
            return out
        spec = self.fused_mlp_spec() if hasattr(r, "epoch_batch") else None
        if spec is not None:
            return self._update_fused_dp(r, spec) if self.dp_enabled else self._update_fused(r, spec)
        wide_epoch = self._wide_epoch_step(r)
        if wide_epoch is not None:
            if self.dp_enabled:
                return self._update_wide_epoch_xdp(r, wide_epoch)
            return self._update_wide_epoch(r, wide_epoch)
        nmb = r.num_minibatches(self.batch_size)
        n_steps = self.n_epochs * nmb
        n_norms = self.n_epochs if self.gradient_accumulation else n_steps
        blocks = self.blocks
        blocks.ensure_tables(n_steps, n_norms)
        K = None
        self.flat.check_views()
        if (self.use_graphs and self.flat.flat.is_cuda and hasattr(r, "_flat_fields")
                and r.logprobs is not None and not (self.dp_enabled and self.world > 1
                                                    and torch.distributed.get_backend(self.dp_group) != "nccl")):
            K = self._update_graphed(r, nmb)
            return self._read_stats(n_steps, n_norms, K)
        wide = self._wide_step()
        shuffle = not self.gradient_accumulation
        ext = None
        for e in range(self.n_epochs):
            if hasattr(r, "epoch_batch"):  # DeviceRollout: the epoch's permuted copy, sliced
                full = r.epoch_batch(shuffle)
                mbs = [r._batch_from([full.obs, full.actions, full.values, full.advantages, full.returns]
                                     + ([full.logprobs] if full.logprobs is not None else [])
                                     + ([full.action_masks] if full.action_masks is not None else []),
                                     slice(i, i + self.batch_size)) for i in range(0, r.total_steps, self.batch_size)]
            else:
                full, mbs = None, r.minibatches(self.batch_size, shuffle=shuffle)
            for mb in mbs:
                if K is None:
                    with torch.no_grad():  # K (value columns) before the device blocks are written
                        K = value_columns(self.policy(mb.obs[:1], mb.actions[:1], action_masks=(
                            mb.action_masks[:1] if mb.action_masks is not None else None))[2])
                    ext = self._dp_moments_table(K, n_steps)
                    hp = self._hparams(K, nmb)
                    hp.ext_moments = ext.data_ptr() if ext is not None else None
                    blocks.upload(hp, self.optimizer.step_count)
                    if ext is not None and full is not None:
                        self._fill_epoch_moments(ext, e, full.advantages, nmb)
                elif ext is not None and mb is mbs[0] and full is not None:
                    self._fill_epoch_moments(ext, e, full.advantages, nmb)
                if mb.logprobs is None:
                    raise ValueError("PPO needs rollout logprobs (include_logp=True)")
                self._minibatch_loss_grads(wide, mb.obs, mb.actions, mb.action_masks, mb.values, mb.advantages,
                                           mb.returns, mb.logprobs, [K])
                if not self.gradient_accumulation:
                    if self.dp_enabled:
                        self._all_reduce(self.flat.grad, average=True)
                    self.optimizer.step(blocks.state, blocks.norms)
            if self.gradient_accumulation:
                if self.dp_enabled:
                    self._all_reduce(self.flat.grad, average=True)
                self.optimizer.step(blocks.state, blocks.norms)
        return self._read_stats(n_steps, n_norms, K)

    def _dp_moments_table(self, K: int, n_steps: int) -> Optional[torch.Tensor]:
        """Data parallel on the per-minibatch path: the global minibatches' advantage (mean, den),
        one row per stats row, for the loss kernel (rai_ppo_hparams.ext_moments); None when the
        minibatch's own moments are the reference's (single rank) or no normalisation is asked for.
        Layout (n_steps, columns, 2): K columns, or one under normalize_advantages_after_scaling."""
        if not self.dp_enabled or self.world == 1:
            return None
        if self.normalize_advantages_after_scaling:
            return torch.zeros((n_steps, 1, 2), dtype=torch.float32, device=self.device)
        if not (self.normalize_advantage or self.standardize_advantage):
            return None
        return torch.zeros((n_steps, K, 2), dtype=torch.float32, device=self.device)

    def _fill_epoch_moments(self, ext: torch.Tensor, epoch: int, adv_epoch: torch.Tensor, nmb: int) -> None:
        """Rows [epoch*nmb, (epoch+1)*nmb) of the table from this rank's permuted advantages (one
        small all-reduce; stream-ordered before the epoch's loss launches)."""
        ext[epoch * nmb:(epoch + 1) * nmb].copy_(self._global_adv_moments(adv_epoch, nmb))

    def _read_stats(self, n_steps: int, n_norms: int, K: Optional[int]) -> Tuple[np.ndarray, np.ndarray, int]:
        blocks = self.blocks
        stats_t = blocks.stats[:n_steps]
        if self.dp_enabled:
            stats_t = stats_t.clone()
            self._all_reduce(stats_t, average=True)
        host = torch.cat([stats_t.reshape(-1), blocks.norms[:n_norms]]).cpu().numpy()
        stats = host[: n_steps * _lib.RAI_STAT_STRIDE].reshape(n_steps, _lib.RAI_STAT_STRIDE)
        return stats, host[n_steps * _lib.RAI_STAT_STRIDE:], K or 1

    def _update_graphed(self, r, nmb: int) -> int:
        """The generic update with the minibatch step replayed from a hipGraph (graphs.py).
        Same minibatches, same kernels, same order as the eager loop above."""
        from .graphs import GraphedUpdate

        if self._graphed is None:
            self._graphed = GraphedUpdate(self.device)
        gu = self._graphed
        blocks = self.blocks
        fields = r._flat_fields()
        shuffle = not self.gradient_accumulation
        n = r.total_steps
        B = min(self.batch_size, n)
        n_full, tail = n // B, n % B
        # data parallel over our RCCL communicator: the gradient all-reduce is bucketed, overlapped
        # with the backward on a side stream and captured with the step (dp_buckets.py)
        buckets = self._grad_buckets() if not self.gradient_accumulation else None
        optim_in_step = not self.gradient_accumulation and (not self.dp_enabled or buckets is not None)
        has_masks = r.action_masks is not None
        K_box = [None]

        wide = self._wide_step()
        # NatureCNN on uint8 frames: the gather emits obs.float() / range_size in channels_last
        xf = getattr(self.policy, "obs_transform", lambda o: None)(fields[0]) if wide is None else None
        xforms = [xf] + [None] * (len(fields) - 1) if xf is not None else None

        def step(bufs):
            obs, actions, values, adv, ret, logprobs = bufs[:6]
            masks = bufs[6] if has_masks else None
            if buckets is not None:
                buckets.begin()
            self._minibatch_loss_grads(wide, obs, actions, masks, values, adv, ret, logprobs, K_box,
                                       obs_prepared=xforms is not None)
            if buckets is not None:
                buckets.finish(scale=1.0 / self.world)
            if optim_in_step:
                self.optimizer.step(blocks.state, blocks.norms, count=False)

        # K (value columns) before the device blocks are written: one forward of one row
        with torch.no_grad():
            _, _, v0 = self.policy(fields[0][:1], fields[1][:1],
                                   action_masks=fields[6][:1] if has_masks else None)
        K = value_columns(v0)
        K_box[0] = K
        ext = self._dp_moments_table(K, self.n_epochs * nmb)
        hp = self._hparams(K, nmb)
        hp.ext_moments = ext.data_ptr() if ext is not None else None
        blocks.upload(hp, self.optimizer.step_count)
        # a graph bakes in every device pointer it touches: key it on the ones that can change
        tag = (optim_in_step, wide is not None, buckets is not None, blocks.stats.data_ptr(), blocks.norms.data_ptr(), blocks.hp.data_ptr(),
               blocks.state.data_ptr(), self.flat.flat.data_ptr(), self.flat.grad.data_ptr(),
               self.optimizer.hp_dev.data_ptr())
        g = gu.graph_for(fields, B, tag, xforms)
        cur = torch.cuda.current_stream(self.device)
        gu.stream.wait_stream(cur)
        with torch.cuda.stream(gu.stream):
            gu.set_rollout(fields, B, shuffle)
            for e in range(self.n_epochs):
                perm = r.permutation() if shuffle else None
                if ext is not None:
                    self._fill_epoch_moments(ext, e, fields[3][perm] if perm is not None else fields[3], nmb)
                gu.start_epoch(perm)
                for _ in range(n_full):
                    g.run(gu.desc, gu.stream, step)
                    if not optim_in_step and not self.gradient_accumulation:
                        self._all_reduce(self.flat.grad, average=True)
                        self.optimizer.step(blocks.state, blocks.norms)
                if tail:
                    gu.tail(fields, tail, step, xforms)
                    if not optim_in_step and not self.gradient_accumulation:
                        self._all_reduce(self.flat.grad, average=True)
                        self.optimizer.step(blocks.state, blocks.norms)
                if self.gradient_accumulation:
                    if self.dp_enabled:
                        self._all_reduce(self.flat.grad, average=True)
                    self.optimizer.step(blocks.state, blocks.norms)
        cur.wait_stream(gu.stream)
        if optim_in_step:  # replays stepped the optimizer on device; keep the host count in sync
            self.optimizer.step_count += self.n_epochs * (n_full + (1 if tail else 0))
        return K

    def _grad_buckets(self):
        """GradBuckets for the bucketed, backward-overlapped all-reduce (dp_buckets.py) when data
        parallel runs over our own RCCL communicator and the policy has a bucket layout (NatureCNN),
        else None (one all-reduce of the whole flat gradient after the step).  RAI_DP_BUCKETS=0: off."""
        if not self.dp_enabled or self._dp_comm is None or os.environ.get("RAI_DP_BUCKETS", "1") == "0":
            return None
        if self._buckets is not None:
            return self._buckets
        from .dp_buckets import GradBuckets, nature_cnn_buckets

        layout = nature_cnn_buckets(self.policy, self.flat)
        if layout is None:
            return None
        bounds, triggers = layout
        L, comm, dev = _lib.lib(), self._dp_comm, self.device

        def allreduce(v: torch.Tensor) -> None:
            _lib.check(L.rai_dp_allreduce_sum_f32(comm, v.data_ptr(), v.numel(), _lib.stream_handle(dev)),
                       "rai_dp_allreduce_sum_f32")

        self._buckets = GradBuckets(self.flat, bounds, triggers, allreduce, dev)
        return self._buckets

    def _train_stats(self, stats: np.ndarray, norms: np.ndarray, K: int, nmb: int, explained_var: float):
        last = stats[-nmb:].astype(np.float64)  # only the last epoch's stats are kept (ppo.py:288-289)
        vl = last[:, 5:5 + K]
        vc = last[:, 5 + _lib.RAI_MAX_K:5 + _lib.RAI_MAX_K + K]
        if self.vf_weights is not None:
            w = np.asarray(self.vf_weights, np.float64)
            v_loss = float(np.mean(vl @ w))
        else:
            v_loss = np.mean(vl, axis=0)
            v_loss = float(v_loss[0]) if K == 1 else v_loss
        val_clipped = np.mean(vc, axis=0)
        last_norms = norms[-1:] if self.gradient_accumulation else norms[-nmb:]
        return TrainStats(
            loss=float(last[:, 0].mean()), pi_loss=float(last[:, 1].mean()), v_loss=v_loss,
            entropy_loss=float(last[:, 2].mean()), approx_kl=float(last[:, 3].mean()),
            clipped_frac=float(last[:, 4].mean()),
            val_clipped_frac=float(val_clipped[0]) if K == 1 else val_clipped, additional_losses={},
            explained_var=explained_var, grad_norm=float(np.mean(last_norms)))

    def save(self, path: str) -> None:
        save_optimizer(self.optimizer, path)

    def load(self, path: str) -> None:
        load_optimizer(self.optimizer, path, self.device)
