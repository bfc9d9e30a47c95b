"""ACBC (rl_algo_impls/acbc/acbc.py:29-165) on the GPU against the reference's own ACBC.learn
(tests/golden/acbc_steps.npz, made by tests/golden/make_golden_acbc.py): fixed minibatches over two
epochs, with and without gradient accumulation; per-step pre-clip grad norms, the parameters after
every optimizer step, the last epoch's mean loss / pi_loss / v_loss tensorboard scalars and the
Adam state."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from rl_algo_impls_amd.acbc import ACBC
from rl_algo_impls_amd.registry import ALGOS
from rl_algo_impls_amd.rollout import Batch
import make_golden_networks as nets

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class Recorder:
    def __init__(self):
        self.scalars = {}

    def add_scalar(self, tag, value, global_step=None):
        self.scalars[tag] = float(value)


class FixedRollout:
    def __init__(self, batches):
        self.batches = batches

    @property
    def total_steps(self):
        return sum(len(b) for b in self.batches)

    def num_minibatches(self, bs):
        return len(self.batches)

    def minibatches(self, bs, shuffle=True):
        return iter(self.batches)

    def explained_variance(self):
        y = torch.cat([b.returns for b in self.batches]).double()
        p = torch.cat([b.values for b in self.batches]).double()
        return float(1 - torch.var(y - p, unbiased=False) / torch.var(y, unbiased=False))


@pytest.mark.parametrize("case", ["cp_acbc", "cp_acbc_gradacc"])
def test_acbc_steps_match_reference(case):
    assert ALGOS["acbc"] is ACBC
    z = np.load(GOLDEN / "acbc_steps.npz", allow_pickle=False)
    meta = json.loads(str(z["index"]))[case]
    p = case + "/"
    policy = nets.build("cartpole")
    nets.load_flat(policy, z[p + "init"])
    policy = policy.to(DEV)
    rec = Recorder()
    algo = ACBC(policy, DEV, rec, n_epochs=meta["epochs"], **meta["kw"])
    batches = []
    for i in range(meta["n"]):
        t = lambda k: torch.from_numpy(z[f"{p}b{i}_{k}"]).to(DEV)
        batches.append(Batch(t("obs"), None, t("actions"), None, None, t("values"), t("advantages"), t("returns")))
    r = FixedRollout(batches)

    class Gen:
        def rollout(self, gamma, gae_lambda):
            return r

    algo.learn(r.total_steps, Gen())
    torch.cuda.synchronize()
    n_opt = z[p + "params"].shape[0]
    assert algo.optimizer.step_count == n_opt == meta["opt_step"]
    norms = algo.blocks.norms[:n_opt].cpu().numpy()
    np.testing.assert_allclose(norms, z[p + "norms"], rtol=2e-5)
    np.testing.assert_allclose(algo.flat.flat.cpu().numpy(), z[p + "params"][-1], rtol=1e-4, atol=2e-6)
    m_ref = z[p + "opt_state1"]  # near-zero first moments differ by fp32 summation order: absolute floor
    np.testing.assert_allclose(algo.optimizer.state1.cpu().numpy(), m_ref, rtol=1e-3, atol=1e-6 * np.abs(m_ref).max())
    ref = dict(meta["scalars"])
    for tag in ("losses/loss", "losses/pi_loss", "losses/v_loss", "losses/explained_var"):
        assert tag in rec.scalars, tag
        np.testing.assert_allclose(rec.scalars[tag], ref[tag], rtol=1e-4, atol=1e-6)
    last = z[p + "last_epoch_stats"]
    np.testing.assert_allclose(ref["losses/loss"], last[:, 0].mean(), rtol=1e-12)
