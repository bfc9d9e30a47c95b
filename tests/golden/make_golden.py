"""Generate the golden vectors that pin the oracle and the HIP path.

Runs the REFERENCE ITSELF (read-only at /root/reference, pure Python/PyTorch) in
this container, importing it with the minimal stub packages in ./stubs
(gymnasium 0.29 API surface, stable_baselines3.common.preprocessing, a
tensorboard SummaryWriter recorder).  Only inputs and outputs are written, as
small .npz/.json fixtures next to this script; no reference source is copied.

    python tests/golden/make_golden.py

Fixtures:
  gae_cases.npz           G1  compute_advantages (rl_algo_impls/shared/gae.py:97-124)
  ppo_steps.npz           G2  PPO minibatch steps through PPO.learn_epoch
                              (rl_algo_impls/ppo/ppo.py:214-447): per-step grads,
                              grad norms, params, loss stats, optimizer state
  a2c_step.npz            G4  one A2C update (rl_algo_impls/a2c/a2c.py:76-205)
  learn_epoch_cartpole.npz G3 a full learn_epoch with SyncStepRolloutGenerator
                              (rl_algo_impls/rollout/sync_step_rollout.py) on the
                              seeded synthetic CartPole-shaped env
  policy_init.json/.npz   G5  ActorCritic state_dict keys/shapes/init checksums and
                              forward outputs for the BASELINE policy shapes
"""
from __future__ import annotations

import json
import sys
import types
from dataclasses import astuple
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REFERENCE = Path("/root/reference")


def import_reference():
    sys.path.insert(0, str(HERE / "stubs"))
    sys.path.insert(0, str(REFERENCE))
    tb = types.ModuleType("torch.utils.tensorboard")
    tbw = types.ModuleType("torch.utils.tensorboard.writer")

    class SummaryWriter:
        def __init__(self, *a, **k):
            self.scalars = []

        def add_scalar(self, tag, value, global_step=None):
            self.scalars.append((tag, float(np.asarray(value)), global_step))

        def close(self):
            pass

    tbw.SummaryWriter = SummaryWriter
    tb.SummaryWriter = SummaryWriter
    tb.writer = tbw
    sys.modules["torch.utils.tensorboard"] = tb
    sys.modules["torch.utils.tensorboard.writer"] = tbw
    return SummaryWriter


SummaryWriter = import_reference()

import gymnasium.spaces as gs  # noqa: E402  (stub)
from gymnasium.experimental.vector.vector_env import VectorEnv  # noqa: E402  (stub)
from rl_algo_impls.a2c.a2c import A2C  # noqa: E402
from rl_algo_impls.ppo import ppo as ppo_mod  # noqa: E402
from rl_algo_impls.ppo.ppo import PPO  # noqa: E402
from rl_algo_impls.rollout import sync_step_rollout as ssr_mod  # noqa: E402
from rl_algo_impls.rollout.rollout import Batch, Rollout  # noqa: E402
from rl_algo_impls.rollout.sync_step_rollout import SyncStepRolloutGenerator  # noqa: E402
from rl_algo_impls.shared.callbacks.summary_wrapper import SummaryWrapper  # noqa: E402
from rl_algo_impls.shared.gae import compute_advantages  # noqa: E402
from rl_algo_impls.shared.policy.actor_critic import ActorCritic  # noqa: E402

torch.use_deterministic_algorithms(True)


# ---------------------------------------------------------------------------
class StubVecEnv(VectorEnv):
    """Space-only env (policy construction) or the seeded synthetic env."""

    def __init__(self, num_envs, obs_space, act_space, seed=1, term_prob=1 / 200, kind="cartpole"):
        self.num_envs = num_envs
        self.single_observation_space = obs_space
        self.single_action_space = act_space
        self.rng = np.random.default_rng(seed)
        self.term_prob = term_prob
        self.kind = kind

    def _obs(self):
        shp = (self.num_envs,) + self.single_observation_space.shape
        if self.kind == "pong":
            return self.rng.integers(0, 256, size=shp, dtype=np.uint8)
        return self.rng.standard_normal(shp, dtype=np.float32)

    def reset(self, **kw):
        return self._obs(), {}

    def step(self, actions):
        obs = self._obs()
        rew = np.ones(self.num_envs, np.float32) if self.kind == "cartpole" else \
            self.rng.standard_normal(self.num_envs, dtype=np.float32)
        term = self.rng.random(self.num_envs) < self.term_prob
        return obs, rew, term, np.zeros(self.num_envs, np.bool_), {}


def cartpole_env(n=8, seed=1):
    return StubVecEnv(n, gs.Box(-np.inf, np.inf, (4,), np.float32), gs.Discrete(2), seed=seed)


def halfcheetah_env(n=1, seed=1):
    return StubVecEnv(n, gs.Box(-np.inf, np.inf, (17,), np.float32),
                      gs.Box(-1.0, 1.0, (6,), np.float32), seed=seed, kind="halfcheetah")


def pong_env(n=1, seed=1):
    return StubVecEnv(n, gs.Box(0, 255, (4, 84, 84), np.uint8), gs.Discrete(6), seed=seed, kind="pong")


def flat(ts):
    return torch.cat([t.detach().reshape(-1).float() for t in ts]).numpy().copy()


# ---------------------------------------------------------------------------
# G1: GAE
# ---------------------------------------------------------------------------
def gen_gae(out):
    rng = np.random.default_rng(1234)
    cases = []
    shapes = [(1, 1), (5, 3), (32, 8), (128, 16), (512, 4)]
    for gamma, lam in [(0.98, 0.8), (0.99, 0.95)]:
        for T, N in shapes:
            for dens in [0.0, 0.01, 0.1, 1.0]:
                cases.append(dict(T=T, N=N, K=None, gamma=gamma, lam=lam, dens=dens))
    for T, N in [(17, 5), (64, 8)]:
        for dens in [0.0, 0.1]:
            cases.append(dict(T=T, N=N, K=3, gamma=np.array([0.99, 0.999, 0.999]),
                              lam=np.array([0.95, 0.99, 0.99]), dens=dens))
    # mixed scalar/vector, and K=1 value column with vector gamma
    cases.append(dict(T=33, N=7, K=3, gamma=np.array([0.9, 0.95, 0.99]), lam=0.9, dens=0.05))
    cases.append(dict(T=33, N=7, K=3, gamma=0.97, lam=np.array([0.9, 0.8, 0.7]), dens=0.05))
    cases.append(dict(T=21, N=6, K=1, gamma=np.array([0.99]), lam=np.array([0.95]), dens=0.1))
    arrays = {}
    meta = []
    for i, c in enumerate(cases):
        T, N, K = c["T"], c["N"], c["K"]
        vs = (T, N) if K is None else (T, N, K)
        rewards = (rng.standard_normal(vs) * 3).astype(np.float32)
        values = (rng.standard_normal(vs) * 10).astype(np.float32)
        es = rng.random((T, N)) < c["dens"]
        nes = rng.random((N,)) < c["dens"]
        nv = (rng.standard_normal(vs[1:]) * 10).astype(np.float32)
        adv = compute_advantages(rewards, values, es, nes, nv, c["gamma"], c["lam"])
        assert adv.dtype == np.float32
        p = f"c{i}_"
        arrays.update({p + "rewards": rewards, p + "values": values, p + "episode_starts": es,
                       p + "next_episode_starts": nes, p + "next_values": nv, p + "adv": adv,
                       p + "returns": adv + values,
                       p + "gamma": np.atleast_1d(np.asarray(c["gamma"], np.float64)),
                       p + "lam": np.atleast_1d(np.asarray(c["lam"], np.float64))})
        meta.append(dict(gamma_is_vector=isinstance(c["gamma"], np.ndarray),
                         lam_is_vector=isinstance(c["lam"], np.ndarray)))
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(out / "gae_cases.npz", **arrays)
    print(f"gae_cases.npz: {len(cases)} cases")


# ---------------------------------------------------------------------------
# G2/G4: minibatch steps through the reference learn loop
# ---------------------------------------------------------------------------
class FixedRollout(Rollout):
    def __init__(self, batches):
        self.batches = batches

    @property
    def y_true(self):
        return torch.cat([b.returns for b in self.batches]).numpy()

    @property
    def y_pred(self):
        return torch.cat([b.values for b in self.batches]).numpy()

    @property
    def total_steps(self):
        return sum(len(b) for b in self.batches)

    def num_minibatches(self, batch_size):
        return len(self.batches)

    def minibatches(self, batch_size, shuffle=True):
        return iter(self.batches)


class FixedGen:
    vec_env = None

    def __init__(self, r):
        self.r = r

    def rollout(self, gamma, gae_lambda):
        return self.r


def make_batch(policy, n, rng, obs_shape, discrete_n=None, act_dim=None, K=1, obs_u8=False):
    if obs_u8:
        obs = torch.from_numpy(rng.integers(0, 256, size=(n,) + obs_shape, dtype=np.uint8))
    else:
        obs = torch.from_numpy(rng.standard_normal((n,) + obs_shape).astype(np.float32))
    if discrete_n is not None:
        actions = torch.from_numpy(rng.integers(0, discrete_n, size=n).astype(np.int64))
    else:
        actions = torch.from_numpy((rng.standard_normal((n, act_dim)) * 0.5).astype(np.float32))
    with torch.no_grad():
        lp, _, v = policy(obs, actions)
    logprobs = (lp + torch.from_numpy((rng.standard_normal(n) * 0.1).astype(np.float32))).float()
    vshape = (n,) if K == 1 else (n, K)
    values = (v.reshape(vshape) + torch.from_numpy((rng.standard_normal(vshape) * 0.2).astype(np.float32)))
    adv = torch.from_numpy((rng.standard_normal(vshape) * 2).astype(np.float32))
    returns = (values + adv).float()
    return Batch(obs, logprobs.detach(), actions, None, None, values.detach().float(), adv, returns)


def run_reference_update(algo_cls, policy, batches, algo_kwargs, n_epochs=1):
    writer = SummaryWriter()
    tbw = SummaryWrapper(writer)
    if algo_cls is PPO:
        algo = PPO(policy, torch.device("cpu"), tbw, n_epochs=n_epochs, **algo_kwargs)
    else:
        algo = A2C(policy, torch.device("cpu"), tbw, **algo_kwargs)
    rec = dict(grads=[], norms=[], params=[], stats=[])
    orig = algo.optimizer_step

    def optimizer_step():
        rec["grads"].append(flat([p.grad if p.grad is not None else torch.zeros_like(p)
                                  for p in policy.parameters()]))
        n = orig()
        rec["norms"].append(np.nan if n is None else n)
        rec["params"].append(flat(policy.parameters()))
        return n

    algo.optimizer_step = optimizer_step
    real_tss = ppo_mod.TrainStepStats

    def tss(*args):
        s = real_tss(*args)
        rec["stats"].append(s)
        return s

    ppo_mod.TrainStepStats = tss
    try:
        r = FixedRollout(batches)
        if algo_cls is PPO:
            algo.learn_epoch(0, r.total_steps, FixedGen(r), None)
        else:
            algo.learn(r.total_steps, FixedGen(r))
    finally:
        ppo_mod.TrainStepStats = real_tss
    opt = algo.optimizer.state_dict()
    st = [opt["state"][i] for i in sorted(opt["state"])]
    rec["opt_state1"] = flat([s["exp_avg"] if "exp_avg" in s else s["square_avg"] for s in st])
    rec["opt_state2"] = flat([s["exp_avg_sq"] for s in st]) if "exp_avg_sq" in st[0] else np.zeros(0, np.float32)
    rec["opt_step"] = float(st[0]["step"])
    rec["scalars"] = writer.scalars
    return rec


def stats_array(stats, K):
    rows = []
    for s in stats:
        vl = np.atleast_1d(np.asarray(s.v_loss, np.float64))
        row = [s.loss, s.pi_loss, s.entropy_loss, s.approx_kl, s.clipped_frac]
        vlk = np.zeros(K)
        vlk[: vl.size] = vl
        vcf = np.zeros(K)
        vc = np.atleast_1d(np.asarray(s.val_clipped_frac, np.float64))
        vcf[: vc.size] = vc
        rows.append(row + list(vlk) + list(vcf))
    return np.array(rows, np.float64)


class MultiCritic(torch.nn.Module):
    """Harness network with value_shape (K,) for the multi-critic loss cases
    (the reference's multi-critic heads live in the out-of-scope backbones)."""

    def __init__(self, K=3, n_act=3):
        super().__init__()
        self.body = torch.nn.Sequential(torch.nn.Linear(4, 16), torch.nn.Tanh())
        self.pi = torch.nn.Linear(16, n_act)
        self.v = torch.nn.Linear(16, K)

    def forward(self, obs, actions, action_masks=None):
        h = self.body(obs)
        d = torch.distributions.Categorical(logits=self.pi(h))
        return d.log_prob(actions), d.entropy(), self.v(h)

    def reset_noise(self, *a, **k):
        pass


def gen_ppo_steps(out):
    arrays = {}
    cases = {
        "cp_default": dict(policy="cartpole", n=3, B=256, kw=dict(
            learning_rate=1e-3, batch_size=256, gamma=0.98, gae_lambda=0.8, clip_range=0.2, ent_coef=0.0)),
        "cp_vclip_ent": dict(policy="cartpole", n=2, B=256, kw=dict(
            learning_rate=1e-3, batch_size=256, clip_range=0.2, clip_range_vf=0.1, ent_coef=0.01)),
        "cp_gradacc": dict(policy="cartpole", n=2, B=128, kw=dict(
            learning_rate=1e-3, batch_size=128, clip_range=0.2, gradient_accumulation=True,
            ent_coef=0.01)),
        "cp_klcut": dict(policy="cartpole", n=3, B=64, kw=dict(
            learning_rate=3e-3, batch_size=64, clip_range=0.2, kl_cutoff=1e-4)),
        "hc_gauss": dict(policy="halfcheetah", n=2, B=64, kw=dict(
            learning_rate=2.0633e-05, batch_size=64, clip_range=0.1, ent_coef=0.000401762,
            max_grad_norm=0.8, vf_coef=0.58096)),
        "mc_mrw": dict(policy="multicritic", n=2, B=96, kw=dict(
            learning_rate=1e-3, batch_size=96, clip_range=0.2, clip_range_vf=0.2, ent_coef=0.01,
            vf_coef=[0.5, 0.3, 0.2], multi_reward_weights=[1.0, 0.5, 0.25], ppo2_vf_coef_halving=True)),
        "mc_after": dict(policy="multicritic", n=2, B=96, kw=dict(
            learning_rate=1e-3, batch_size=96, clip_range=0.2, multi_reward_weights=[0.8, 0.1, 0.1],
            normalize_advantages_after_scaling=True, vf_coef=0.5)),
        "mc_huber_w": dict(policy="multicritic", n=2, B=96, kw=dict(
            learning_rate=1e-3, batch_size=96, clip_range=0.2, clip_range_vf=0.1,
            vf_loss_fn="huber_loss", vf_weights=[0.6, 0.3, 0.1], vf_coef=0.5,
            normalize_advantage=False, standardize_advantage=True,
            multi_reward_weights=[1.0, 1.0, 1.0])),
    }
    index = {}
    for name, c in cases.items():
        torch.manual_seed(7)
        rng = np.random.default_rng(11)
        if c["policy"] == "cartpole":
            policy = ActorCritic(cartpole_env())
            mk = lambda: make_batch(policy, c["B"], rng, (4,), discrete_n=2)
            K = 1
        elif c["policy"] == "halfcheetah":
            policy = ActorCritic(halfcheetah_env(), pi_hidden_sizes=[64, 64], v_hidden_sizes=[64, 64],
                                 activation_fn="relu", log_std_init=-2, init_layers_orthogonal=False)
            mk = lambda: make_batch(policy, c["B"], rng, (17,), act_dim=6)
            K = 1
        else:
            policy = MultiCritic()
            mk = lambda: make_batch(policy, c["B"], rng, (4,), discrete_n=3, K=3)
            K = 3
        init = flat(policy.parameters())
        batches = [mk() for _ in range(c["n"])]
        rec = run_reference_update(PPO, policy, batches, c["kw"])
        p = name + "/"
        for i, b in enumerate(batches):
            for f in ("obs", "logprobs", "actions", "values", "advantages", "returns"):
                arrays[f"{p}b{i}_{f}"] = getattr(b, f).numpy()
        arrays[p + "init"] = init
        arrays[p + "grads"] = rec["grads"][0]  # first step's pre-clip grads; later steps via params
        arrays[p + "norms"] = np.array(rec["norms"], np.float64)
        arrays[p + "params"] = np.stack(rec["params"])
        arrays[p + "stats"] = stats_array(rec["stats"], K)
        arrays[p + "opt_state1"] = rec["opt_state1"]
        arrays[p + "opt_state2"] = rec["opt_state2"]
        index[name] = dict(policy=c["policy"], n=c["n"], B=c["B"], K=K, kw=c["kw"],
                           opt_step=rec["opt_step"])
    arrays["index"] = np.array(json.dumps(index))
    np.savez_compressed(out / "ppo_steps.npz", **arrays)
    print(f"ppo_steps.npz: {list(cases)}")


def gen_a2c(out):
    torch.manual_seed(3)
    rng = np.random.default_rng(5)
    policy = ActorCritic(cartpole_env())
    init = flat(policy.parameters())
    b = make_batch(policy, 40, rng, (4,), discrete_n=2)
    b = Batch(b.obs, None, b.actions, None, None, b.values, b.advantages, b.returns)
    rec = run_reference_update(A2C, policy, [b], dict(learning_rate=7e-4, ent_coef=0.01))
    np.savez_compressed(out / "a2c_step.npz", init=init, obs=b.obs.numpy(), actions=b.actions.numpy(),
                        values=b.values.numpy(), advantages=b.advantages.numpy(), returns=b.returns.numpy(),
                        grads=np.stack(rec["grads"]), params=np.stack(rec["params"]),
                        opt_state1=rec["opt_state1"], opt_step=rec["opt_step"])
    print("a2c_step.npz")


# ---------------------------------------------------------------------------
# G3: a full learn_epoch with the reference's SyncStepRolloutGenerator
# ---------------------------------------------------------------------------
def gen_learn_epoch(out):
    torch.manual_seed(1)
    np.random.seed(1)
    env = cartpole_env(n=8, seed=1)
    policy = ActorCritic(env).to(torch.device("cpu"))
    init = flat(policy.parameters())
    captured = {}
    RealVecRollout = ssr_mod.VecRollout

    def vec_rollout(**kw):
        for k in ("next_episode_starts", "next_values", "obs", "actions", "rewards", "episode_starts",
                  "values", "logprobs"):
            captured[k] = np.array(kw[k], copy=True)
        r = RealVecRollout(**kw)
        captured["advantages"] = r.advantages.copy()
        captured["returns"] = r.returns.copy()
        return r

    ssr_mod.VecRollout = vec_rollout
    perms = []
    real_randperm = torch.randperm

    def randperm(n, *a, **k):
        p = real_randperm(n, *a, **k)
        perms.append(p.numpy().copy())
        return p

    torch.randperm = randperm
    try:
        gen = SyncStepRolloutGenerator(policy, env, n_steps=32)
        kw = dict(learning_rate=1e-3, batch_size=64, n_epochs=2, gamma=0.98, gae_lambda=0.8,
                  clip_range=0.2, ent_coef=0.0)
        writer = SummaryWriter()
        algo = PPO(policy, torch.device("cpu"), SummaryWrapper(writer), **kw)
        grad_norms = []
        orig = algo.optimizer_step

        def optimizer_step():
            n = orig()
            grad_norms.append(n)
            return n

        algo.optimizer_step = optimizer_step
        algo.learn_epoch(0, 256, gen, None)
    finally:
        ssr_mod.VecRollout = RealVecRollout
        torch.randperm = real_randperm
    scal = {t: v for t, v, _ in writer.scalars}
    np.savez_compressed(
        out / "learn_epoch_cartpole.npz", init=init, params=flat(policy.parameters()),
        perms=np.stack(perms), grad_norms=np.array(grad_norms),
        losses=np.array([scal[f"losses/{k}"] for k in
                         ("loss", "pi_loss", "v_loss", "entropy_loss", "approx_kl", "clipped_frac",
                          "explained_var", "grad_norm")]),
        kw=np.array(json.dumps(kw)), **captured)
    print("learn_epoch_cartpole.npz")


# ---------------------------------------------------------------------------
# G5: policy construction parity
# ---------------------------------------------------------------------------
def gen_policy_init(out):
    specs = {
        "cartpole": (cartpole_env, {}),
        "halfcheetah": (halfcheetah_env, dict(pi_hidden_sizes=[256, 256], v_hidden_sizes=[256, 256],
                                              activation_fn="relu", log_std_init=-2,
                                              init_layers_orthogonal=False)),
        "pong": (pong_env, dict(activation_fn="relu")),
    }
    meta = {}
    arrays = {}
    for name, (mk_env, kw) in specs.items():
        torch.manual_seed(1)
        env = mk_env()
        policy = ActorCritic(env, **kw)
        sd = policy.state_dict()
        meta[name] = dict(kwargs=kw, keys=[[k, list(v.shape), float(v.double().sum()),
                                            float((v.double() ** 2).sum()),
                                            [float(x) for x in v.reshape(-1)[:4]]]
                                           for k, v in sd.items()])
        rng = np.random.default_rng(2)
        obs = env._obs()[:1] if False else None
        n = 4
        shp = env.single_observation_space.shape
        if name == "pong":
            obs = rng.integers(0, 256, size=(n,) + shp, dtype=np.uint8)
        else:
            obs = rng.standard_normal((n,) + shp).astype(np.float32)
        if name == "halfcheetah":
            act = (rng.standard_normal((n, 6)) * 0.5).astype(np.float32)
        else:
            act = rng.integers(0, env.single_action_space.n, size=n).astype(np.int64)
        with torch.no_grad():
            lp, ent, v = policy(torch.from_numpy(obs), torch.from_numpy(act))
        arrays.update({f"{name}_obs": obs, f"{name}_act": act, f"{name}_logp": lp.numpy(),
                       f"{name}_entropy": ent.numpy(), f"{name}_v": v.numpy()})
    (out / "policy_init.json").write_text(json.dumps(meta, indent=1))
    np.savez_compressed(out / "policy_forward.npz", **arrays)
    print("policy_init.json, policy_forward.npz")


if __name__ == "__main__":
    assert REFERENCE.exists(), "the reference is only available in the build container"
    out = HERE
    gen_gae(out)
    gen_ppo_steps(out)
    gen_a2c(out)
    gen_learn_epoch(out)
    gen_policy_init(out)
    (out / "VERSIONS.json").write_text(json.dumps(
        dict(torch=torch.__version__, numpy=np.__version__, python=sys.version.split()[0]), indent=1))
