"""Data-parallel PPO update with real kernels: 2 ranks (gloo, both on cuda:0) vs the
single-process fused update over the equivalent global minibatches."""
import multiprocessing as mp
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("dp_batch", ["global", "per-rank"])
@pytest.mark.parametrize("xdp", ["1", "0"], ids=["in_kernel_xgmi_exchange", "per_step_loop"])
def test_fused_dp_world2_matches_single_process_global_minibatches(xdp, dp_batch, monkeypatch):
    """xdp=1: one launch per epoch per rank, gradients summed across the two processes inside
    the kernel through IPC-mapped regions (both ranks on this one GPU, running concurrently);
    xdp=0: the per-step loop (grads kernel -> gloo all-reduce -> clip+Adam).
    dp_batch="global" is SURVEY.md 8(e)'s rule (PPO(batch_size=256) on every rank, 128 rows per
    rank per step): the update equals the single-process update at batch 256 over the ranks'
    interleaved rollouts; "per-rank" gets there from batch_size=128 per rank."""
    monkeypatch.setenv("RAI_XDP", xdp)
    _fused_dp_world2_check(dp_batch=dp_batch)


def test_xdp_canary_failure_on_one_rank_falls_back_on_every_rank(monkeypatch):
    """Rank 1's in-kernel exchange canary fails (RAI_XDP_INJECT_FAIL_RANK: it never launches, so
    rank 0's canary times out waiting for it): both ranks must agree, release the mappings and
    run the per-step loop — no hang, equal parameters, the single-process result."""
    monkeypatch.setenv("RAI_XDP", "1")
    _fused_dp_world2_check(dp_batch="global", inject_fail_rank=1)


def _fused_dp_world2_check(dp_batch="per-rank", inject_fail_rank=None):
    import dp_worker
    import make_golden_networks as nets
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import Batch

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.fused_dp_worker, args=(r, 2, port, q, "gloo", dp_batch, inject_fail_rank))
             for r in range(2)]
    for p in procs:
        p.start()
    res = []
    import queue
    import time

    deadline = time.time() + 240
    while len(res) < len(procs):  # fail fast when a rank dies instead of waiting out the timeout
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, s0, n0), (_, p1, s1, n1) = res
    np.testing.assert_array_equal(p0, p1)  # ranks stay bitwise in sync

    # single process: global minibatch i = rank0 rows [i*128,(i+1)*128) ++ rank1 rows [...]
    dev = torch.device("cuda", 0)
    d0, d1 = dp_worker.make_rank_data(0, dev), dp_worker.make_rank_data(1, dev)

    def interleave(f):
        a, b = getattr(d0, f), getattr(d1, f)
        return torch.cat([torch.cat([a[i * 128:(i + 1) * 128], b[i * 128:(i + 1) * 128]]) for i in range(4)])

    glob = Batch(*(interleave(f) for f in ("obs", "logprobs", "actions")), None, None,
                 *(interleave(f) for f in ("values", "advantages", "returns")))
    torch.manual_seed(0)
    policy = nets.build("cartpole").to(dev)
    algo = PPO(policy, dev, None, batch_size=256, n_epochs=2, learning_rate=3e-3, clip_range=0.2, ent_coef=0.01)
    assert algo.fused_mlp_spec() is not None

    class R:
        total_steps = 1024

        def num_minibatches(self, bs):
            return 4

        def epoch_batch(self, shuffle=True):
            return glob

    stats, norms, _ = algo.update(R())
    np.testing.assert_allclose(n0, norms, rtol=1e-4)
    np.testing.assert_allclose(s0[:, :6], stats[:, :6], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p0, algo.flat.flat.cpu().numpy(), rtol=1e-4, atol=1e-6)


def _run_world1(backend):
    import queue
    import time

    import dp_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=dp_worker.fused_dp_worker, args=(0, 1, _port(), q, backend))
    p.start()
    deadline = time.time() + 240
    while True:
        try:
            res = q.get(timeout=2)
            break
        except queue.Empty:
            assert p.exitcode in (None, 0), f"worker exited with {p.exitcode}"
            assert time.time() < deadline, "worker did not report in time"
    p.join(timeout=60)
    assert p.exitcode == 0
    return res


def test_native_rccl_epoch_loop_matches_python_loop_world1():
    """rai_mlp_ppo_epoch_dp (RCCL communicator; per step the multi-CU kernel applies the previous
    all-reduced gradient and computes the next one) against the Python-driven loop
    (rai_mlp_ppo_grads -> gloo all-reduce -> rai_clip_optim_step).  Same gradients; the two Adam
    implementations differ in the last bits (hardware sqrt/rcp vs IEEE sequences) and the norm
    in summation order, hence fp32 tolerances."""
    _, pn, sn, nn = _run_world1("nccl")
    _, pg, sg, ng = _run_world1("gloo")
    np.testing.assert_allclose(nn, ng, rtol=1e-5)
    np.testing.assert_allclose(sn[:, :6], sg[:, :6], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(pn, pg, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("dp_batch", ["global", "per-rank"])
def test_wide_mlp_dp_world2_matches_single_process_global_minibatches(dp_batch):
    """HalfCheetah-class policy on the wide-MLP kernels, 2 ranks (gloo, both on cuda:0) with the
    identity permutation: rank r's minibatch i is its time steps [4i, 4i + 4) x 16 envs, so the
    global minibatch i is time steps [4i, 4i + 4) x all 32 envs of the concatenated rollout.  The
    single-process update over that rollout (batch 128) is the reference: advantage normalisation
    over the GLOBAL minibatch, loss means over its 128 rows."""
    import queue
    import time

    import dp_worker
    from rl_algo_impls_amd.ppo import PPO

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.wide_dp_worker, args=(r, 2, port, q, dp_batch)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 240
    while len(res) < 2:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, s0, n0), (_, p1, s1, n1) = res
    np.testing.assert_array_equal(p0, p1)

    dev = torch.device("cuda", 0)
    d0, d1 = dp_worker.make_wide_rank_data(0, dev), dp_worker.make_wide_rank_data(1, dev)
    glob = {k: torch.cat([d0[k], d1[k]], dim=1 if d0[k].dim() > 1 else 0) for k in d0}
    policy, r = dp_worker.wide_policy_and_rollout(glob, dev)
    algo = PPO(policy, dev, None, batch_size=128, n_epochs=2, learning_rate=3e-4, ent_coef=0.01)
    stats, norms, _ = algo.update(r)
    np.testing.assert_allclose(n0, norms, rtol=1e-4)
    np.testing.assert_allclose(s0[:, :6], stats[:, :6], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p0, algo.flat.flat.cpu().numpy(), rtol=1e-4, atol=2e-6)


@pytest.mark.parametrize("after", [False, True], ids=["per_column", "after_scaling"])
def test_multicritic_dp_world2_matches_single_process_global_minibatches(after):
    """3-critic policy (multi_reward_weights, per-critic vf_coef, vector gamma), 2 ranks (gloo, both on
    cuda:0), identity permutation: the global minibatch's advantage moments per column (or of the
    weighted advantage under normalize_advantages_after_scaling) reach the loss kernel through
    rai_ppo_hparams.ext_moments; compared with the single-process update over the concatenated
    rollout (batch 64)."""
    import queue
    import time

    import dp_worker
    from rl_algo_impls_amd.ppo import PPO

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.mc_dp_worker, args=(r, 2, port, q, after)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 240
    while len(res) < 2:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, s0, n0), (_, p1, s1, n1) = res
    np.testing.assert_array_equal(p0, p1)

    dev = torch.device("cuda", 0)
    d0, d1 = dp_worker.make_mc_rank_data(0), dp_worker.make_mc_rank_data(1)
    glob = {k: torch.cat([d0[k], d1[k]], dim=1 if k not in ("nv", "nes") else 0) for k in d0}
    policy, r = dp_worker.mc_policy_and_rollout(glob, dev)
    algo = PPO(policy, dev, None, batch_size=64, normalize_advantages_after_scaling=after, **dp_worker.MC_KW)
    stats, norms, K = algo.update(r)
    assert K == 3
    np.testing.assert_allclose(n0, norms, rtol=1e-4)
    np.testing.assert_allclose(s0[:, :8], stats[:, :8], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p0, algo.flat.flat.cpu().numpy(), rtol=1e-4, atol=2e-6)


def test_nature_cnn_bucketed_allreduce_world1_matches_single_process():
    """C3's data-parallel step with the gradient all-reduce bucketed (fc + heads as soon as the fc
    backward has written them, overlapping the convolutions' backward; the convolutions after) on
    a side stream and captured into the step's hipGraph over our RCCL communicator (1-rank group on
    this one GPU): the same update as the whole-gradient all-reduce after each replay and as the
    single-process update (deterministic MIOpen solvers, so the three runs agree to fp32 rounding)."""
    import queue
    import time

    import dp_worker

    ctx = mp.get_context("spawn")
    out = {}
    for mode in ("buckets", "flat", "single"):
        q = ctx.Queue()
        p = ctx.Process(target=dp_worker.cnn_dp_worker, args=(0, 1, _port(), q, mode))
        p.start()
        deadline = time.time() + 240
        while True:
            try:
                res = q.get(timeout=2)
                break
            except queue.Empty:
                assert p.exitcode in (None, 0), f"{mode} worker exited with {p.exitcode}"
                assert time.time() < deadline, f"{mode} worker did not report in time"
        p.join(timeout=60)
        assert p.exitcode == 0
        out[res[0]] = res[1:]
    pb, sb, nb = out["buckets"]
    for other in ("flat", "single"):
        po, so, no = out[other]
        np.testing.assert_allclose(nb, no, rtol=1e-5)
        np.testing.assert_allclose(sb[:, :6], so[:, :6], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(pb, po, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("world", [2, 4])
def test_env_partition_split_world2_matches_single_process_c2(world):
    """bench.py's default multi-GPU rule (SURVEY.md 8(d) "global N fixed; per-GPU N = N/R" with
    8(e)'s global minibatch): `world` ranks (gloo, all on cuda:0, in-kernel exchange) each own 1/world of
    the env columns of ONE 16 x 64 CartPole-shaped rollout, compute their GAE on the device and take
    256 / world of the 256 rows of each optimizer step (world 2: the per-rank geometry, 8 CUs of 16 rows
    per network; world 4: 64 rows per rank).  Reference: the single-process update over the whole
    rollout (GAE over all 64 columns) whose epoch permutation lists, for minibatch i, rank 0's rows
    [b i, b i + b) and then rank 1's, ..., as (t, n) of the concatenated env group."""
    import queue
    import time

    import dp_worker
    import make_golden_networks as nets
    from rl_algo_impls_amd.ppo import PPO

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 240
    while len(res) < world:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(x[4] for x in res), "the in-kernel exchange was not used"
    p0, s0, n0 = res[0][1], res[0][2], res[0][3]
    for x in res[1:]:
        np.testing.assert_array_equal(p0, x[1])

    T, N = dp_worker.SPLIT_T, dp_worker.SPLIT_N
    part, b = N // world, 256 // world
    local = torch.arange(T * part)  # rank-local flat row -> (t, n) of the whole env group
    to_global = [(local // part) * N + (local % part) + r * part for r in range(world)]
    perm = torch.cat([torch.cat([to_global[r][i * b:(i + 1) * b] for r in range(world)])
                      for i in range(T * part // b)])
    dev = torch.device("cuda", 0)
    r = dp_worker.split_device_rollout(dp_worker.split_rollout_tensors(), torch.arange(N), dev, perm)
    torch.manual_seed(0)
    algo = PPO(nets.build("cartpole").to(dev), dev, None, **dp_worker.SPLIT_KW)
    stats, norms, _ = algo.update(r)
    np.testing.assert_allclose(n0, norms, rtol=1e-4)
    np.testing.assert_allclose(s0[:, :6], stats[:, :6], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p0, algo.flat.flat.cpu().numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("kind,world", [("cartpole", 2), ("cartpole", 4), ("halfcheetah", 2)])
def test_replicated_update_matches_single_process_bitwise(kind, world):
    """PPO.enable_data_parallel's automatic update mode on a dependent-chain path (the C2 fused epoch
    kernel at 256 rows; the C4 wide whole-epoch kernel at 64 rows) under bench.py's default rules (env
    split, global minibatch): `world` ranks (gloo, all on cuda:0) each own 1/world of the env columns of
    ONE rollout and compute their GAE; one all-gather assembles the whole env group's rollout and every
    rank runs the single-process update over it.  Result: BITWISE the single-process update over the
    whole rollout (same kernels, same inputs, same permutation), identical on every rank."""
    import queue
    import time

    import dp_worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.replicated_gpu_worker, args=(r, world, port, q, kind))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 240
    while len(res) < world:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dev = torch.device("cuda", 0)
    algo = dp_worker.replicated_trainer(kind, dev)
    r = dp_worker.replicated_device_rollout(dp_worker.replicated_rollout_tensors(kind), torch.arange(dp_worker.REPL_N),
                                            dev, algo.gamma, algo.gae_lambda)
    stats, norms, _ = algo.update(r)
    assert (getattr(algo, "_we_ws", None) is not None) == (kind == "halfcheetah")
    p1 = algo.flat.flat.cpu().numpy()
    for _, p, s, n, we in res:
        assert we == (kind == "halfcheetah"), "the whole-epoch kernel path on every rank"
        np.testing.assert_array_equal(p, p1)
        np.testing.assert_array_equal(n, norms)
        np.testing.assert_array_equal(s, stats)


@pytest.mark.parametrize("hidden,rows,n", [(64, 32, 512), (256, 32, 400)])
def test_wide_epoch_xdp_world2_matches_single_process_global_minibatches(hidden, rows, n):
    """The C4-class whole-epoch kernel under data parallel (rai_mlp_wide_epoch_xdp): two processes on
    this GPU, each running its `rows`-row slices of the global minibatches in one launch per epoch, the
    workgroups' owned gradients summed over the ranks inside the kernel.  Ranks stay bitwise equal; the
    result equals the single-process whole-epoch update at batch 2 x rows over the interleaved rollouts
    (fp32 tolerance: per-rank partial sums change the summation order).  n = 400: a ragged last
    minibatch (16 rows per rank)."""
    import queue
    import time

    import dp_worker
    import make_golden_networks as nets
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import Batch

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.wide_epoch_xdp_worker, args=(r, 2, port, q, hidden, rows, n)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 240
    while len(res) < len(procs):
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, s0, n0), (_, p1, s1, n1) = res
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(n0, n1)

    dev = torch.device("cuda", 0)
    d0, d1 = dp_worker.make_rank_data_wide(0, dev, n), dp_worker.make_rank_data_wide(1, dev, n)
    nmb = -(-n // rows)

    def interleave(f):
        a, b = getattr(d0, f), getattr(d1, f)
        return torch.cat([torch.cat([a[i * rows:(i + 1) * rows], b[i * rows:(i + 1) * rows]]) for i in range(nmb)])

    glob = Batch(*(interleave(f) for f in ("obs", "logprobs", "actions")), None, None,
                 *(interleave(f) for f in ("values", "advantages", "returns")))
    torch.manual_seed(0)
    policy = ActorCritic(nets.halfcheetah_env(), pi_hidden_sizes=[hidden, hidden], v_hidden_sizes=[hidden, hidden],
                         activation_fn="relu", log_std_init=-2, init_layers_orthogonal=False).to(dev)
    algo = PPO(policy, dev, None, batch_size=2 * rows, n_epochs=2, learning_rate=3e-4, clip_range=0.2, ent_coef=0.01,
               max_grad_norm=0.5)

    class R:
        total_steps = 2 * n

        def num_minibatches(self, bs):
            return -(-self.total_steps // bs)

        def epoch_batch(self, shuffle=True):
            return glob

    assert algo._wide_epoch_step(R()) is not None
    stats, norms, _ = algo.update(R())
    np.testing.assert_allclose(n0, norms, rtol=2e-4)
    np.testing.assert_allclose(s0[:, :6], stats[:, :6], rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(p0, algo.flat.flat.cpu().numpy(), rtol=2e-4, atol=2e-6)


@pytest.mark.parametrize("xdp,world", [(False, 2), (True, 2), (True, 4)],
                         ids=["host_allreduce_w2", "in_kernel_w2", "in_kernel_w4"])
def test_scaled_batch_policy_dp_world2_matches_single_process(xdp, world):
    """SURVEY 8(d)'s batch policy (b) under data parallel: `world` ranks (gloo, one GPU) run 512-row slices
    of 512 x world-row global minibatches through the large-minibatch kernels, the gradient summed over
    the ranks either by a per-step host all-reduce (grads mode) or inside each step's reduce launch
    through the IPC-mapped exchange regions (rai_mlp_ppo_epoch_xdp: no host sync, no RCCL call per
    step); ranks bitwise equal, and equal to the single process at batch 512 x world over the interleaved
    rollouts (fp32 tolerance: per-rank partial sums)."""
    import queue
    import time

    import dp_worker
    import make_golden_networks as nets
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import Batch

    rows, n = 512, 2048  # > 256 rows per rank: the large-minibatch kernels at every world size
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=dp_worker.large_dp_worker, args=(r, world, port, q, rows, n, xdp))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 240
    while len(res) < world:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"rank exited with {dead}"
            assert time.time() < deadline, "ranks did not report in time"
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, p0, s0, n0 = res[0]
    for x in res[1:]:
        np.testing.assert_array_equal(p0, x[1])
        np.testing.assert_array_equal(n0, x[3])

    dev = torch.device("cuda", 0)
    ds = [dp_worker.make_rank_data(r, dev, n) for r in range(world)]
    nmb = n // rows

    def interleave(f):
        return torch.cat([torch.cat([getattr(d, f)[i * rows:(i + 1) * rows] for d in ds]) for i in range(nmb)])

    glob = Batch(*(interleave(f) for f in ("obs", "logprobs", "actions")), None, None,
                 *(interleave(f) for f in ("values", "advantages", "returns")))
    torch.manual_seed(0)
    algo = PPO(nets.build("cartpole").to(dev), dev, None, batch_size=world * rows, n_epochs=2, learning_rate=3e-3,
               clip_range=0.2, ent_coef=0.01)

    class R:
        total_steps = world * n

        def num_minibatches(self, bs):
            return -(-self.total_steps // bs)

        def epoch_batch(self, shuffle=True):
            return glob

    stats, norms, _ = algo.update(R())
    np.testing.assert_allclose(n0, norms, rtol=2e-4)
    np.testing.assert_allclose(s0[:, :6], stats[:, :6], rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(p0, algo.flat.flat.cpu().numpy(), rtol=2e-4, atol=2e-6)
