"""Multi-process workers for the data-parallel tests (spawned by tests/test_dp*.py)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _init(rank, world, port, backend="gloo"):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)


def moments_worker(rank, world, port, q):
    """Global advantage moments across ranks == moments of the concatenated minibatches: one column,
    K=3 columns, and the multi_reward_weights-weighted advantage (normalize_advantages_after_scaling)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO

    w = np.array([0.8, 0.01, 0.19])

    class Stub(PPO):
        def __init__(self, after):
            self.batch_size, self.world, self.dp_group = 64, world, None
            self.normalize_advantage, self.standardize_advantage = True, False
            self.normalize_advantages_after_scaling = after
            self.multi_reward_weights = w if after else None

    g = torch.Generator().manual_seed(100 + rank)
    results = []
    for K, after in ((1, False), (3, False), (3, True)):
        adv = torch.randn(64 * 5 + 30, K, generator=g) * (1 + rank) + rank
        adv = adv[:, 0] if K == 1 else adv
        out = Stub(after)._global_adv_moments(adv, 6)
        allv = [torch.zeros_like(adv) for _ in range(world)]
        dist.all_gather(allv, adv)
        ref = []
        for i in range(6):
            mb = torch.cat([a[i * 64:(i + 1) * 64] for a in allv]).double().reshape(-1, K)
            if after:
                mb = (mb.float() * torch.tensor(w, dtype=torch.float32)).sum(1, keepdim=True).double()
            ref.append(torch.stack([mb.mean(0), mb.std(0) + 1e-8], -1).tolist())
        results.append((out.numpy().tolist(), ref))
    q.put((rank, results))
    dist.destroy_process_group()


def fused_dp_worker(rank, world, port, q, backend="gloo", dp_batch="per-rank", inject_fail_rank=None):
    """DP fused update on rank-local data (gloo: all ranks on cuda:0, Python-driven loop;
    nccl (world 1 on a one-GPU box): the natively driven RCCL loop, rai_mlp_ppo_epoch_dp).
    128 rows per rank per optimizer step under either minibatch rule: batch_size 128 with
    dp_batch="per-rank", batch_size 256 (the global minibatch) with dp_batch="global".
    inject_fail_rank: that rank's in-kernel exchange canary reports a failure (every rank must
    then fall back to the per-step loop together)."""
    import numpy as np
    import torch

    if inject_fail_rank is not None:
        os.environ["RAI_XDP_INJECT_FAIL_RANK"] = str(inject_fail_rank)
    _init(rank, world, port, backend)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import Batch
    import make_golden_networks as nets

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    policy = nets.build("cartpole").to(dev)
    bs = 128 * (world if dp_batch == "global" else 1)
    algo = PPO(policy, dev, None, batch_size=bs, n_epochs=2, learning_rate=3e-3, clip_range=0.2, ent_coef=0.01)
    algo.enable_data_parallel(xdp=os.environ.get("RAI_XDP", "1") != "0", dp_batch=dp_batch,
                              update_mode=os.environ.get("RAI_DP_UPDATE", "exchange"))
    assert algo.batch_size == 128 and algo.global_batch_size == 128 * world
    expect_xdp = world > 1 and os.environ.get("RAI_XDP", "1") != "0" and inject_fail_rank is None
    assert (algo._dp_comm is not None) == (backend == "nccl" and not expect_xdp)
    assert (algo._xdp is not None) == expect_xdp, "in-kernel exchange not set up"
    data = make_rank_data(rank, dev)

    class R:
        total_steps = data.obs.shape[0]

        def num_minibatches(self, bs):
            return self.total_steps // bs

        def epoch_batch(self, shuffle=True):
            return data

    stats, norms, _ = algo.update(R())
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms))
    import torch.distributed as dist

    dist.destroy_process_group()


def wide_epoch_xdp_worker(rank, world, port, q, hidden=64, rows_per_rank=32, n=512):
    """C4-class wide MLP (Gaussian head) under data parallel with the in-kernel exchange: every rank runs
    rai_mlp_wide_epoch_xdp on its own rows (rows_per_rank per optimizer step; global minibatch
    rows_per_rank x world, dp_batch="global")."""
    import torch

    _init(rank, world, port, "gloo")
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.policy import ActorCritic
    import make_golden_networks as nets

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    policy = ActorCritic(nets.halfcheetah_env(), pi_hidden_sizes=[hidden, hidden], v_hidden_sizes=[hidden, hidden],
                         activation_fn="relu", log_std_init=-2, init_layers_orthogonal=False).to(dev)
    algo = PPO(policy, dev, None, batch_size=rows_per_rank * world, n_epochs=2, learning_rate=3e-4, clip_range=0.2,
               ent_coef=0.01, max_grad_norm=0.5)
    algo.enable_data_parallel(xdp=True, dp_batch="global", update_mode="exchange")
    assert algo.batch_size == rows_per_rank
    assert algo._xdp is not None, "in-kernel exchange not set up for the wide policy"
    data = make_rank_data_wide(rank, dev, n)

    class R:
        total_steps = n

        def num_minibatches(self, bs):
            return -(-self.total_steps // bs)

        def epoch_batch(self, shuffle=True):
            return data

    assert algo._wide_epoch_step(R()) is not None, "whole-epoch kernel not selected under data parallel"
    stats, norms, _ = algo.update(R())
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms))
    import torch.distributed as dist

    dist.destroy_process_group()


def make_rank_data_wide(rank, dev, n=512):
    import torch

    from rl_algo_impls_amd.rollout import Batch

    g = torch.Generator().manual_seed(11 + rank)
    obs = torch.randn(n, 17, generator=g)
    act = torch.randn(n, 6, generator=g).clamp(-1, 1)
    logp = -4.0 + 0.3 * torch.randn(n, generator=g)
    vals = torch.randn(n, generator=g)
    adv = torch.randn(n, generator=g) * 2 + 0.3 * rank
    ret = vals + adv
    t = lambda x: x.to(dev)
    return Batch(t(obs), t(logp), t(act), None, None, t(vals), t(adv), t(ret))


def large_dp_worker(rank, world, port, q, rows_per_rank=512, n=2048, xdp=False):
    """SURVEY 8(d) batch policy (b) under data parallel: the CartPole-class policy at minibatches of
    rows_per_rank x world rows (> 256, the large-minibatch kernels), dp_batch="global" over gloo; xdp: the
    gradient summed over the ranks inside each step's reduce launch (IPC-mapped regions) instead of the
    per-step host all-reduce."""
    import torch

    _init(rank, world, port, "gloo")
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO
    import make_golden_networks as nets

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    algo = PPO(nets.build("cartpole").to(dev), dev, None, batch_size=rows_per_rank * world, n_epochs=2,
               learning_rate=3e-3, clip_range=0.2, ent_coef=0.01)
    algo.enable_data_parallel(xdp=xdp, dp_batch="global", update_mode="exchange")
    assert algo.batch_size == rows_per_rank and (algo._xdp is not None) == xdp and algo.fused_mlp_spec() is not None
    data = make_rank_data(rank, dev, n)

    class R:
        total_steps = n

        def num_minibatches(self, bs):
            return -(-self.total_steps // bs)

        def epoch_batch(self, shuffle=True):
            return data

    stats, norms, _ = algo.update(R())
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms))
    import torch.distributed as dist

    dist.destroy_process_group()


def make_rank_data(rank, dev, n=512):
    import torch

    from rl_algo_impls_amd.rollout import Batch

    g = torch.Generator().manual_seed(7 + rank)
    obs = torch.randn(n, 4, generator=g)
    act = torch.randint(0, 2, (n,), generator=g)
    logp = torch.log(torch.full((n,), 0.5)) + 0.05 * torch.randn(n, generator=g)
    vals = torch.randn(n, generator=g)
    adv = torch.randn(n, generator=g) * 2 + 0.3 * rank
    ret = vals + adv
    t = lambda x: x.to(dev)
    return Batch(t(obs), t(logp), t(act), None, None, t(vals), t(adv), t(ret))


def rms_worker(rank, world, port, q):
    """Normalize wrappers over a ragged env split with the cross-rank RunningMeanStd merge."""
    import numpy as np
    import torch.distributed as dist

    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd import wrappers
    from test_host_wrappers import FixtureEnv

    _init(rank, world, port)
    z = np.load(ROOT / "tests" / "golden" / "host_wrappers.npz", allow_pickle=False)
    n = z["env_obs"].shape[1]
    # ragged split: rank 0 owns 3 envs, rank 1 the other 5
    envs = slice(0, 3) if rank == 0 else slice(3, n)
    env = wrappers.NormalizeReward(wrappers.NormalizeObservation(FixtureEnv(z, envs), group=dist.group.WORLD),
                                   gamma=0.97, group=dist.group.WORLD)
    o, _ = env.reset()
    obs, rew = [o], []
    for _ in range(z["env_rew"].shape[0]):
        o, r, *_ = env.step(None)
        obs.append(o)
        rew.append(r)
    q.put((rank, np.stack(obs), np.stack(rew), env.env.rms.mean, env.rms.var))
    dist.destroy_process_group()


def make_wide_rank_data(rank, dev, T=16, N=16):
    """Rank-local (T, N, ...) rollout tensors for a HalfCheetah-shaped policy (17-dim obs, Box(6))."""
    import torch

    g = torch.Generator().manual_seed(31 + rank)
    return dict(obs=torch.randn(T, N, 17, generator=g), act=torch.randn(T, N, 6, generator=g).clamp(-1, 1),
                rew=torch.randn(T, N, generator=g) + 0.2 * rank, vals=torch.randn(T, N, generator=g),
                starts=(torch.rand(T, N, generator=g) < 0.05).to(torch.uint8),
                logp=-8.0 + 0.3 * torch.randn(T, N, generator=g), nv=torch.randn(N, generator=g),
                nes=torch.zeros(N, dtype=torch.uint8))


def wide_policy_and_rollout(d, dev, hidden=128):
    """(policy seeded identically everywhere, DeviceRollout with the identity permutation)."""
    import torch

    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.rollout import DeviceRollout

    torch.manual_seed(0)
    env = SyntheticVecEnv(2, "halfcheetah", seed=3)
    policy = ActorCritic(env, pi_hidden_sizes=[hidden, hidden], v_hidden_sizes=[hidden, hidden], activation_fn="relu",
                         log_std_init=-1.0, init_layers_orthogonal=False).to(dev)
    t = lambda x: x.to(dev)
    r = DeviceRollout(dev, t(d["nes"]), t(d["nv"]), t(d["obs"]), t(d["act"]), t(d["rew"]), t(d["starts"]),
                      t(d["vals"]), t(d["logp"]), None, 0.99, 0.95, perm_source=lambda n: torch.arange(n))
    return policy, r


def wide_dp_worker(rank, world, port, q, dp_batch="per-rank"):
    """Data-parallel update through the wide-MLP kernels (gloo, all ranks on cuda:0): global advantage
    moments per minibatch (rai_ppo_hparams.ext_moments), gradient all-reduce per step.  64 rows per
    rank per step: batch_size 64 per rank ("per-rank") or the global 128 ("global")."""
    import torch

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO

    dev = torch.device("cuda", 0)
    policy, r = wide_policy_and_rollout(make_wide_rank_data(rank, dev), dev)
    algo = PPO(policy, dev, None, batch_size=64 * (world if dp_batch == "global" else 1), n_epochs=2,
               learning_rate=3e-4, ent_coef=0.01)
    algo.enable_data_parallel(dp_batch=dp_batch, update_mode="exchange")
    assert algo.batch_size == 64
    stats, norms, _ = algo.update(r)
    assert algo._wide not in (None, False), "wide path not taken"
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms))
    import torch.distributed as dist

    dist.destroy_process_group()


def make_mc_rank_data(rank, T=16, N=8):
    """Rank-local rollout tensors for the 3-critic harness policy (4-dim obs, 3 actions)."""
    import torch

    g = torch.Generator().manual_seed(71 + rank)
    return dict(obs=torch.randn(T, N, 4, generator=g), act=torch.randint(0, 3, (T, N), generator=g),
                rew=torch.randn(T, N, 3, generator=g) + 0.3 * rank, vals=torch.randn(T, N, 3, generator=g),
                starts=(torch.rand(T, N, generator=g) < 0.05).to(torch.uint8),
                logp=-1.1 + 0.1 * torch.randn(T, N, generator=g), nv=torch.randn(N, 3, generator=g),
                nes=torch.zeros(N, dtype=torch.uint8))


MC_KW = dict(n_epochs=2, learning_rate=3e-4, ent_coef=0.01, clip_range_vf=0.2, multi_reward_weights=[0.8, 0.01, 0.19],
             vf_coef=[0.5, 0.1, 0.2], ppo2_vf_coef_halving=True)


def mc_policy_and_rollout(d, dev):
    import numpy as np
    import torch

    import make_golden_networks as nets
    from rl_algo_impls_amd.rollout import DeviceRollout

    torch.manual_seed(0)
    policy = nets.build("multicritic").to(dev)
    t = lambda x: x.to(dev)
    r = DeviceRollout(dev, t(d["nes"]), t(d["nv"]), t(d["obs"]), t(d["act"]), t(d["rew"]), t(d["starts"]),
                      t(d["vals"]), t(d["logp"]), None, np.array([0.99, 0.999, 0.999]), np.array([0.95, 0.99, 0.99]),
                      perm_source=lambda n: torch.arange(n))
    return policy, r


def mc_dp_worker(rank, world, port, q, after):
    """Data-parallel per-minibatch update of a 3-critic policy (gloo, all ranks on cuda:0): global
    advantage moments per column (or of the weighted advantage after scaling) through ext_moments."""
    import torch

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO

    dev = torch.device("cuda", 0)
    policy, r = mc_policy_and_rollout(make_mc_rank_data(rank), dev)
    algo = PPO(policy, dev, None, batch_size=32, normalize_advantages_after_scaling=after, **MC_KW)
    algo.enable_data_parallel(dp_batch="per-rank")
    stats, norms, _ = algo.update(r)
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms))
    import torch.distributed as dist

    dist.destroy_process_group()


def batch_rule_worker(rank, world, port, q):
    """PPO.enable_data_parallel's minibatch rules on CPU (gloo): per-rank keeps batch_size rows per
    rank (global minibatch batch_size x world); global splits the YAML batch_size over the ranks and
    rejects a batch that does not divide; weights are broadcast from rank 0."""
    import torch

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO
    import make_golden_networks as nets

    out = {}
    for rule, bs in (("per-rank", 256), ("global", 256), ("global", 255)):
        torch.manual_seed(rank)  # different init per rank: enable_data_parallel must broadcast rank 0's
        algo = PPO(nets.build("cartpole"), torch.device("cpu"), None, batch_size=bs)
        try:
            algo.enable_data_parallel(dp_batch=rule)
            out[(rule, bs)] = (algo.batch_size, algo.global_batch_size, float(algo.flat.flat.double().sum()))
        except ValueError as e:
            out[(rule, bs)] = str(e)
    # idempotent: a second call (or a switch of rule) derives from the YAML batch_size again
    algo = PPO(nets.build("cartpole"), torch.device("cpu"), None, batch_size=256)
    sizes = []
    for rule in ("global", "global", "per-rank", "global"):
        algo.enable_data_parallel(dp_batch=rule)
        sizes.append((algo.batch_size, algo.global_batch_size))
    out["repeat"] = sizes
    q.put((rank, out))
    import torch.distributed as dist

    dist.destroy_process_group()


def cnn_dp_worker(rank, world, port, q, mode):
    """NatureCNN (C3-shaped, 84x84 uint8 frames) graph-replayed update, world 1 on cuda:0.
    mode "buckets": data parallel over our RCCL communicator with the bucketed all-reduce overlapped
    with the backward and captured into the step's graph (dp_buckets.py); "flat": data parallel with
    the whole-gradient all-reduce after each replay (RAI_DP_BUCKETS=0); "single": no data parallel."""
    import numpy as np
    import torch

    if mode == "flat":
        os.environ["RAI_DP_BUCKETS"] = "0"
    if mode != "single":
        _init(rank, world, port, "nccl")
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import DeviceRollout

    torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    policy = ActorCritic(SyntheticVecEnv(2, "pong", seed=5), activation_fn="relu").to(dev)
    g = torch.Generator().manual_seed(9)
    T, N = 2, 256
    t = lambda x: x.to(dev)
    r = DeviceRollout(dev, t(torch.zeros(N, dtype=torch.uint8)), t(torch.randn(N, generator=g)),
                      t(torch.randint(0, 256, (T, N, 4, 84, 84), generator=g, dtype=torch.uint8)),
                      t(torch.randint(0, 6, (T, N), generator=g)), t(torch.randn(T, N, generator=g)),
                      t((torch.rand(T, N, generator=g) < 0.05).to(torch.uint8)), t(torch.randn(T, N, generator=g)),
                      t(-1.79 + 0.05 * torch.randn(T, N, generator=g)), None, 0.99, 0.95,
                      perm_source=lambda n: torch.randperm(n, generator=torch.Generator().manual_seed(3)))
    algo = PPO(policy, dev, None, batch_size=128, n_epochs=2, learning_rate=2.5e-4, clip_range=0.1, vf_coef=0.5,
               ent_coef=0.01)
    if mode != "single":
        algo.enable_data_parallel(dp_batch="per-rank")
        assert algo._dp_comm is not None
    stats, norms, _ = algo.update(r)
    torch.cuda.synchronize()
    assert (getattr(algo, "_buckets", None) is not None) == (mode == "buckets")
    if mode == "buckets":  # the fc + heads bucket went from inside the backward (autograd's device thread)
        assert algo._buckets.early_launches > 0
    q.put((mode, algo.flat.flat.cpu().numpy(), np.asarray(stats), np.asarray(norms)))
    if mode != "single":
        import torch.distributed as dist

        dist.destroy_process_group()


def c3_repro_worker(q, deterministic):
    """The same C3-shaped update twice from the same weights, rollout and permutations, under
    running_utils.set_device_optimizations(use_deterministic_algorithms=deterministic)."""
    import torch

    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.envs import SyntheticVecEnv
    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import SyncStepRolloutGenerator
    from rl_algo_impls_amd.running_utils import set_device_optimizations

    dev = torch.device("cuda", 0)
    set_device_optimizations(dev, use_deterministic_algorithms=deterministic)
    N, T = 64, 32
    env = SyntheticVecEnv(N, "pong", seed=3)
    torch.manual_seed(3)
    pol = ActorCritic(env, activation_fn="relu").to(dev)
    gen = SyncStepRolloutGenerator(pol, env, n_steps=T, seed=3)
    r = gen.rollout(gamma=0.99, gae_lambda=0.95)
    p0 = torch.nn.utils.parameters_to_vector(pol.parameters()).detach().clone()
    out = []
    for _ in range(2):
        torch.nn.utils.vector_to_parameters(p0, pol.parameters())
        algo = PPO(pol, dev, None, n_epochs=2, batch_size=256, learning_rate=2.5e-4, clip_range=0.1, vf_coef=0.5,
                   ent_coef=0.01)
        g = torch.Generator(device="cpu").manual_seed(11)
        r._perm_source = lambda n: torch.randperm(n, generator=g)
        stats, norms, _ = algo.update(r)
        torch.cuda.synchronize()
        out.append((algo.flat.flat.detach().cpu().numpy().copy(), norms.copy()))
    q.put(out)


SPLIT_T, SPLIT_N = 16, 64


def split_rollout_tensors(seed=21):
    """One (T, N) CartPole-shaped rollout (inputs of GAE and the update), identical wherever it is
    built: the env group of N envs that bench.py --env-partition split divides over the ranks."""
    import torch

    g = torch.Generator().manual_seed(seed)
    T, N = SPLIT_T, SPLIT_N
    return dict(obs=torch.randn(T, N, 4, generator=g), act=torch.randint(0, 2, (T, N), generator=g),
                rew=torch.randn(T, N, generator=g), starts=(torch.rand(T, N, generator=g) < 0.05).to(torch.uint8),
                vals=torch.randn(T, N, generator=g), logp=-0.69 + 0.05 * torch.randn(T, N, generator=g),
                nstarts=(torch.rand(N, generator=g) < 0.05).to(torch.uint8), nvals=torch.randn(N, generator=g))


def split_device_rollout(d, cols, dev, perm):
    """DeviceRollout (GAE on the device) over env columns `cols` of the rollout, epoch permutation
    `perm` every epoch."""
    from rl_algo_impls_amd.rollout import DeviceRollout

    t = lambda x: x[:, cols].contiguous().to(dev)
    return DeviceRollout(dev, d["nstarts"][cols].contiguous().to(dev), d["nvals"][cols].contiguous().to(dev),
                         t(d["obs"]), t(d["act"]), t(d["rew"]), t(d["starts"]), t(d["vals"]), t(d["logp"]), None,
                         0.98, 0.8, perm_source=lambda n: perm.clone())


SPLIT_KW = dict(batch_size=256, n_epochs=2, learning_rate=3e-3, clip_range=0.2, ent_coef=0.01, gamma=0.98,
                gae_lambda=0.8)


def split_worker(rank, world, port, q):
    """bench.py --env-partition split --dp-batch global on the C2 path: rank r owns env columns
    [r N/R, (r+1) N/R) of ONE env group, runs its own GAE on the device and takes batch_size / R rows
    per optimizer step through the fused epoch kernel with the in-kernel exchange (identity epoch
    permutation, so the parent can rebuild the global minibatches)."""
    import torch

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO
    import make_golden_networks as nets

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    algo = PPO(nets.build("cartpole").to(dev), dev, None, **SPLIT_KW)
    algo.enable_data_parallel(dp_batch="global", update_mode="exchange")
    assert algo.batch_size == SPLIT_KW["batch_size"] // world and algo.fused_mlp_spec() is not None
    n = SPLIT_N // world
    cols = torch.arange(rank * n, (rank + 1) * n)
    r = split_device_rollout(split_rollout_tensors(), cols, dev, torch.arange(SPLIT_T * n))
    stats, norms, _ = algo.update(r)
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms, algo._xdp is not None))
    import torch.distributed as dist

    dist.destroy_process_group()


def replicated_worker(rank, world, port, q):
    """PPO's replicated data-parallel update on CPU (gloo): the batch rule (every rank keeps the YAML
    minibatch), the rollout assembly (rank r's (T, N/R, ...) fields become env columns
    [r N/R, (r+1) N/R) of the whole group's rollout) and the shuffle keys agreed from rank 0's."""
    import torch

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    from rl_algo_impls_amd.ppo import PPO
    from rl_algo_impls_amd.rollout import DeviceRollout
    import make_golden_networks as nets

    out = {}
    torch.manual_seed(rank)
    algo = PPO(nets.build("cartpole"), torch.device("cpu"), None, batch_size=256)
    algo.enable_data_parallel(dp_batch="global", update_mode="replicated")
    out["sizes"] = (algo.batch_size, algo.global_batch_size, algo.dp_update_mode)
    out["params"] = float(algo.flat.flat.double().sum())
    try:
        algo.enable_data_parallel(dp_batch="per-rank", update_mode="replicated")
        out["per_rank"] = "accepted"
    except ValueError as e:
        out["per_rank"] = str(e)
    algo.enable_data_parallel(dp_batch="global")  # auto on a CPU trainer: the exchange rule
    out["auto_cpu"] = (algo.batch_size, algo.dp_update_mode)
    T, n = 5, 3
    g = torch.Generator().manual_seed(100 + rank)
    f = lambda *s: torch.randn((T, n) + s, generator=g)
    local = dict(obs=f(4), actions=torch.randint(0, 2, (T, n), generator=g), values=f(), advantages=f(),
                 returns=f(), logprobs=f())
    keys = iter(range(1000 * (rank + 1), 1000 * (rank + 2)))
    r = DeviceRollout.from_fields(torch.device("cpu"), local["obs"], local["actions"], local["values"],
                                  local["advantages"], local["returns"], local["logprobs"],
                                  perm_keys=lambda: next(keys))
    algo.world = world
    gr = algo._replicated_rollout(r)
    out["local"] = {k: v.numpy() for k, v in local.items()}
    out["gathered"] = {k: getattr(gr, k).numpy() for k in local}
    out["total_steps"] = gr.total_steps
    out["keys"] = [gr._perm_keys() for _ in range(3)]
    q.put((rank, out))
    import torch.distributed as dist

    dist.destroy_process_group()


REPL_T, REPL_N = 16, 64


def replicated_rollout_tensors(kind, seed=31):
    """One (T, N) rollout of the CartPole-class (C2 fused epoch kernel) or HalfCheetah-class (C4 wide
    whole-epoch kernel) shape, identical wherever it is built."""
    import torch

    g = torch.Generator().manual_seed(seed)
    T, N = REPL_T, REPL_N
    if kind == "cartpole":
        obs, act = torch.randn(T, N, 4, generator=g), torch.randint(0, 2, (T, N), generator=g)
        logp = -0.69 + 0.05 * torch.randn(T, N, generator=g)
    else:
        obs, act = torch.randn(T, N, 17, generator=g), torch.randn(T, N, 6, generator=g).clamp(-1, 1)
        logp = -1.0 + 0.1 * torch.randn(T, N, generator=g)
    return dict(obs=obs, act=act, rew=torch.randn(T, N, generator=g),
                starts=(torch.rand(T, N, generator=g) < 0.05).to(torch.uint8), vals=torch.randn(T, N, generator=g),
                logp=logp, nstarts=(torch.rand(N, generator=g) < 0.05).to(torch.uint8), nvals=torch.randn(N, generator=g),
                perm=torch.randperm(T * N, generator=g))


def replicated_trainer(kind, dev):
    """(PPO trainer seeded identically everywhere, whole-epoch path of `kind`)."""
    import torch

    from rl_algo_impls_amd.policy import ActorCritic
    from rl_algo_impls_amd.ppo import PPO
    import make_golden_networks as nets

    torch.manual_seed(0)
    if kind == "cartpole":
        return PPO(nets.build("cartpole").to(dev), dev, None, **SPLIT_KW)
    policy = ActorCritic(nets.halfcheetah_env(), pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256],
                         activation_fn="relu", log_std_init=-1.0, init_layers_orthogonal=False).to(dev)
    return PPO(policy, dev, None, batch_size=64, n_epochs=2, learning_rate=3e-4, clip_range=0.2, ent_coef=0.01,
               max_grad_norm=0.5, gamma=0.99, gae_lambda=0.95)


def replicated_device_rollout(d, cols, dev, gamma, lam):
    """DeviceRollout (GAE on the device) over env columns `cols`; the epoch permutation is the fixed
    permutation of the WHOLE env group's T x N rows (the replicated update draws it over the gathered
    rollout)."""
    from rl_algo_impls_amd.rollout import DeviceRollout

    t = lambda x: x[:, cols].contiguous().to(dev)
    perm = d["perm"]
    return DeviceRollout(dev, d["nstarts"][cols].contiguous().to(dev), d["nvals"][cols].contiguous().to(dev),
                         t(d["obs"]), t(d["act"]), t(d["rew"]), t(d["starts"]), t(d["vals"]), t(d["logp"]), None,
                         gamma, lam, perm_source=lambda n: perm.clone())


def replicated_gpu_worker(rank, world, port, q, kind):
    """bench.py's default multi-GPU rules (env split, global minibatch) with PPO's automatic update mode on
    a dependent-chain path: rank r owns env columns [r N/R, (r+1) N/R) and computes their GAE; the update
    is replicated (one all-gather of the rollout, the single-process update on every rank)."""
    import torch

    _init(rank, world, port)
    import _pkgload

    _pkgload.load()
    dev = torch.device("cuda", 0)
    algo = replicated_trainer(kind, dev)
    algo.enable_data_parallel(dp_batch="global")
    assert algo.dp_update_mode == "replicated" and algo._xdp is None and algo._dp_comm is None
    n = REPL_N // world
    r = replicated_device_rollout(replicated_rollout_tensors(kind), torch.arange(rank * n, (rank + 1) * n), dev,
                                  algo.gamma, algo.gae_lambda)
    stats, norms, _ = algo.update(r)
    assert algo.last_update_rollout.total_steps == REPL_T * REPL_N
    we = getattr(algo, "_we_ws", None) is not None
    q.put((rank, algo.flat.flat.cpu().numpy(), stats, norms, we))
    import torch.distributed as dist

    dist.destroy_process_group()
