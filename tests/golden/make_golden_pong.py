"""Golden vectors for the C3 (Pong, NatureCNN) update path, from the REFERENCE ITSELF.

SURVEY.md §8(c) G2, Pong shape: the reference's ActorCritic for PongNoFrameskip-v4
(uint8 4x84x84 frames -> NatureCnn (rl_algo_impls/shared/encoder/nature_cnn.py:10-53,
`/range_size` prescale cnn.py:24-27) -> Categorical(6) actor, critic), stepped by the
reference's own PPO.learn_epoch (rl_algo_impls/ppo/ppo.py:214-447) over fixed
minibatches with the `_atari` hyperparameters (rl_algo_impls/hyperparams/ppo.yml:225-253:
clip_range 0.1, ent_coef 0.01, vf_coef 0.5, lr 2.5e-4, batch 32 here).

The initial weights are NOT the reference's seeded orthogonal init (its LAPACK QR is host
dependent, and 6.75 MB of init would travel with every GPU run): they are drawn from
numpy's PCG64 stream, which is bit-reproducible on every host, and written into the
reference module before its update runs.  `pong_init()` below is the recipe; the GPU test
regenerates the same bits.  Init parity of the module tree itself is pinned separately
(policy_init.json).

    python tests/golden/make_golden_pong.py      # writes pong_steps.npz
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

INIT_SEED = 20261016


def pong_init(shapes, seed: int = INIT_SEED) -> np.ndarray:
    """Flat fp32 initial parameters for the NatureCNN actor-critic, tensor by tensor in
    parameters() order: weights ~ N(0, 1) * gain / sqrt(fan_in) (gain sqrt(2) for hidden
    layers, 0.01 for the actor output, 1 for the critic output, as layer_init's orthogonal
    gains), biases ~ N(0, 1) * 0.01.  Shared by the generator and the GPU test."""
    rng = np.random.default_rng(seed)
    out = []
    weights = [s for s in shapes if len(s) > 1]
    last_w = len(weights) - 1
    wi = 0
    for s in shapes:
        z = rng.standard_normal(int(np.prod(s))).astype(np.float32)
        if len(s) > 1:
            fan_in = int(np.prod(s[1:]))
            gain = np.sqrt(2.0)
            if wi == last_w - 1:
                gain = 0.01  # actor head (pi) output layer
            elif wi == last_w:
                gain = 1.0  # critic output layer
            out.append(z * np.float32(gain / np.sqrt(fan_in)))
            wi += 1
        else:
            out.append(z * np.float32(0.01))
    return np.concatenate(out)


def main():
    import make_golden as mg  # imports the reference with its stubs

    from rl_algo_impls.ppo.ppo import PPO
    from rl_algo_impls.shared.policy.actor_critic import ActorCritic

    kw = dict(learning_rate=2.5e-4, batch_size=32, clip_range=0.1, vf_coef=0.5, ent_coef=0.01)
    n_batches, B = 3, 32
    torch.manual_seed(7)
    policy = ActorCritic(mg.pong_env(), activation_fn="relu")
    shapes = [tuple(p.shape) for p in policy.parameters()]
    init = pong_init(shapes)
    off = 0
    with torch.no_grad():
        for p in policy.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(init[off:off + n]).reshape(p.shape))
            off += n
    rng = np.random.default_rng(13)
    batches = [mg.make_batch(policy, B, rng, (4, 84, 84), discrete_n=6, obs_u8=True) for _ in range(n_batches)]
    rec = mg.run_reference_update(PPO, policy, batches, kw)
    arrays = {}
    for i, b in enumerate(batches):
        for f in ("obs", "logprobs", "actions", "values", "advantages", "returns"):
            arrays[f"b{i}_{f}"] = getattr(b, f).numpy()
    arrays["norms"] = np.array(rec["norms"], np.float64)
    arrays["stats"] = mg.stats_array(rec["stats"], 1)
    arrays["params"] = rec["params"][-1]
    # per-tensor checks of intermediate states (full vectors would be 6.75 MB each)
    sizes = [int(np.prod(s)) for s in shapes]
    cut = np.cumsum([0] + sizes)
    per = lambda v: np.array([np.sqrt(np.sum(np.square(v[cut[j]:cut[j + 1]].astype(np.float64))))
                              for j in range(len(sizes))])
    arrays["step1_param_delta_norms"] = per(rec["params"][0] - init)
    arrays["grads1_norms"] = per(rec["grads"][0])
    arrays["opt_state1_norms"] = per(rec["opt_state1"])
    arrays["opt_state2_norms"] = per(rec["opt_state2"])
    index = dict(kw=kw, n=n_batches, B=B, shapes=[list(s) for s in shapes], init_seed=INIT_SEED,
                 opt_step=rec["opt_step"], torch=torch.__version__, numpy=np.__version__,
                 policy=dict(activation_fn="relu"))
    arrays["index"] = np.array(json.dumps(index))
    np.savez_compressed(HERE / "pong_steps.npz", **arrays)
    print(f"pong_steps.npz: {n_batches} x {B} rows, P={cut[-1]}, norms={arrays['norms']}")


if __name__ == "__main__":
    main()
