"""bench.py's launcher contract: `bench.py --gpus N` starts N ranks itself (one child process per GPU
with the torch.distributed.run environment) unless a launcher already did, and rank 0's JSON line is
the job's output (the metric of rl_algo_impls/ppo/ppo.py:221,422-427, summed over ranks)."""
import json
import os
import subprocess
import sys
import types

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


class _FakeProc:
    def __init__(self, argv, env):
        self.argv, self.env = argv, env
        self.signals = []

    def poll(self):
        return 0

    def send_signal(self, sig):
        self.signals.append(sig)


def test_self_launch_starts_one_rank_per_gpu(monkeypatch):
    started = []

    def fake_popen(argv, env):
        started.append(_FakeProc(argv, env))
        return started[-1]

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("MASTER_PORT", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    monkeypatch.setattr(subprocess, "Popen", fake_popen)
    rc = bench.self_launch(types.SimpleNamespace(gpus=4))
    assert rc == 0 and len(started) == 4
    ports = {p.env["MASTER_PORT"] for p in started}
    assert len(ports) == 1
    for r, p in enumerate(started):
        assert p.argv[0] == sys.executable and p.argv[1].endswith("bench.py")
        assert p.argv[2:] == ["--gpus", "4", "--steps", "2"]
        assert (p.env["RANK"], p.env["LOCAL_RANK"], p.env["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert p.env["MASTER_ADDR"] == "127.0.0.1"


def test_self_launch_is_a_no_op_under_a_launcher_or_one_gpu(monkeypatch):
    monkeypatch.setattr(subprocess, "Popen", lambda *a, **k: pytest.fail("must not spawn"))
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.self_launch(types.SimpleNamespace(gpus=1)) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(types.SimpleNamespace(gpus=2)) is None
    assert bench.self_launch(types.SimpleNamespace(gpus=1)) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.self_launch(types.SimpleNamespace(gpus=4))


def test_self_launch_propagates_a_failed_rank(monkeypatch):
    class Failing(_FakeProc):
        def poll(self):
            return 3 if self.env["RANK"] == "1" else (None if not self.signals else -15)

    started = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(subprocess, "Popen", lambda argv, env: started.append(Failing(argv, env)) or started[-1])
    assert bench.self_launch(types.SimpleNamespace(gpus=2)) == 3
    assert started[0].signals  # rank 0 was stopped, not left waiting in a collective


@pytest.mark.gpu
def test_bench_gpus_2_self_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher: two ranks (gloo for the setup collectives, both on the one
    GPU of the test box, the CartPole epoch kernels exchanging in-kernel as tests/test_gpu_dp.py does)
    and ONE JSON line with n_gpus 2 and the two ranks' env steps."""
    env = dict(os.environ, RAI_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--roofline-reps", "5"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_num_envs"] == 4096 and line["scaling"] == "strong"
    assert line["value"] > 0 and "dp_path" in line
