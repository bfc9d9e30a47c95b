import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
# MIOpen records its solver choices per problem in a user database that outlives the process; the
# tests switch MIOpen to its deterministic solvers (~100x slower at the C3 shapes), so they keep a
# database of their own instead of leaving those choices to later runs on the same machine
os.environ.setdefault("MIOPEN_USER_DB_PATH", tempfile.mkdtemp(prefix="rai-miopen-tests-"))
# likewise TunableOp's GEMM picks (running_utils.set_gemm_tuning, on when deterministic mode is off)
os.environ.setdefault("RAI_TUNABLEOP_FILE", os.path.join(tempfile.mkdtemp(prefix="rai-tunableop-tests-"),
                                                         "tunableop_results%d.csv"))
sys.path.insert(0, str(ROOT / "oracle"))

import _pkgload  # noqa: E402

rai = _pkgload.load()
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _release_gpu_objects_between_tests(request):
    """Trainers own hipGraphs, RCCL communicators and HBM rollouts: collect the previous test's
    garbage and drain the device at a test boundary, not at a random allocation inside the next
    test (a cyclic GC pass once ran in the middle of a later test's forward)."""
    yield
    if "gpu" in request.keywords:
        import gc

        import torch

        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)

    return load


@pytest.fixture(scope="session")
def gae_cases(golden):
    z = golden("gae_cases.npz")
    meta = json.loads(str(z["meta"]))
    cases = []
    for i, m in enumerate(meta):
        p = f"c{i}_"
        c = {k[len(p):]: z[k] for k in z.files if k.startswith(p)}
        gamma = c["gamma"] if m["gamma_is_vector"] else float(c["gamma"][0])
        lam = c["lam"] if m["lam_is_vector"] else float(c["lam"][0])
        c.update(gamma=gamma, lam=lam, idx=i)
        cases.append(c)
    return cases
