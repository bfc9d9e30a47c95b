"""CPU checks of the run setup (rl_algo_impls/runner/running_utils.py:161-184 restated in
rl-algo-impls_amd/running_utils.py): a CPU-device run must not touch the HIP runtime."""
import torch

from rl_algo_impls_amd.running_utils import set_device_optimizations, set_gemm_tuning


def test_cpu_device_optimizations_do_not_touch_hip():
    prev = torch.are_deterministic_algorithms_enabled()
    try:
        for det in (False, True):
            set_device_optimizations(torch.device("cpu"), use_deterministic_algorithms=det)
            assert torch.are_deterministic_algorithms_enabled() == det
        assert set_gemm_tuning(torch.device("cpu"), True) is False
    finally:
        torch.use_deterministic_algorithms(prev)


def test_miopen_find_db_seeded_without_overwriting(tmp_path, monkeypatch):
    """seed_miopen_find_db copies the shipped find / perf records into the target directory (never over a
    file already there: MIOpen appends to it), points MIOPEN_USER_DB_PATH at it, and leaves a caller's
    own MIOPEN_USER_DB_PATH alone."""
    import os

    from rl_algo_impls_amd import running_utils as ru

    shipped = sorted(n for n in os.listdir(ru.MIOPEN_DB_SHIPPED) if n.endswith(".txt"))
    assert any(n.endswith(".ufdb.txt") for n in shipped), "the find database ships with the package"
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    dst = tmp_path / "db"
    dst.mkdir()
    (dst / shipped[0]).write_text("mine\n")
    assert ru.seed_miopen_find_db(str(dst)) == str(dst)
    assert os.environ["MIOPEN_USER_DB_PATH"] == str(dst)
    assert sorted(p.name for p in dst.iterdir()) == shipped
    assert (dst / shipped[0]).read_text() == "mine\n"
    assert ru.seed_miopen_find_db(str(tmp_path / "other")) is None  # the caller's setting stays
    assert os.environ["MIOPEN_USER_DB_PATH"] == str(dst)
