"""Host logic of the measurement tooling behind bench.py's `roofline.traffic`: the PMC
summary (tools/pmc_summary.py), the C3 whole-update merge (tools/c3_traffic.py) and the per-kernel counter
aggregation (tools/pmc_kernels.py), on synthetic rocprofv3 CSV / JSON inputs.  No GPU."""
import csv
import hashlib
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
TOOLS = ROOT / "tools"


def _write_counter_csv(path: Path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, k, c, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": c, "Counter_Value": v})


def _run(*args):
    r = subprocess.run([sys.executable, *map(str, args)], capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    return r


def test_pmc_summary_traffic_is_2x_fetch_plus_write_medians_and_records_the_library_hash(tmp_path):
    k = "void (anonymous namespace)::mlp_ppo_mc8_kernel<0, 16, 16>((anonymous namespace)::MlpArgs)"
    fcsv, wcsv = tmp_path / "f.csv", tmp_path / "w.csv"
    # three launches each: medians 200 KiB fetched, 30 KiB written
    _write_counter_csv(fcsv, [(1, k, "FETCH_SIZE", 100.0), (2, k, "FETCH_SIZE", 200.0), (3, k, "FETCH_SIZE", 900.0)])
    _write_counter_csv(wcsv, [(1, k, "WRITE_SIZE", 30.0), (2, k, "WRITE_SIZE", 10.0), (3, k, "WRITE_SIZE", 31.0)])
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"not a library, just bytes to hash")
    out = tmp_path / "pmc.json"
    _run(TOOLS / "pmc_summary.py", out, "ppo cartpole", fcsv, wcsv, "--lib", lib)
    doc = json.loads(out.read_text())
    e = doc["ppo cartpole"]["mlp_ppo_mc8_kernel<0, 16, 16>"]
    assert e["FETCH_SIZE_KiB_median"] == 200.0 and e["WRITE_SIZE_KiB_median"] == 30.0
    assert e["traffic_bytes_per_launch"] == 2 * 200 * 1024 + 30 * 1024
    assert e["launches"] == [3, 3]
    assert e["lib_sha256"] == hashlib.sha256(lib.read_bytes()).hexdigest()
    # a second workload merges into the same file, the first stays
    _run(TOOLS / "pmc_summary.py", out, "ppo halfcheetah", fcsv, wcsv, "--lib", lib)
    assert set(json.loads(out.read_text())) == {"ppo cartpole", "ppo halfcheetah"}


def test_pmc_kernels_aggregates_per_kernel_and_forms_the_mfma_busy_fraction(tmp_path):
    a, b = "kernel_a", "kernel_b"
    rows = [(1, a, "SQ_VALU_MFMA_BUSY_CYCLES", 1024.0), (1, a, "GRBM_GUI_ACTIVE", 8.0 * 4),
            (2, a, "SQ_VALU_MFMA_BUSY_CYCLES", 1024.0), (2, a, "GRBM_GUI_ACTIVE", 8.0 * 4),
            (3, b, "SQ_VALU_MFMA_BUSY_CYCLES", 0.0), (3, b, "GRBM_GUI_ACTIVE", 8.0)]
    c = tmp_path / "c.csv"
    _write_counter_csv(c, rows)
    out = tmp_path / "k.json"
    _run(TOOLS / "pmc_kernels.py", c, out)
    d = json.loads(out.read_text())["kernels"]
    assert d[a]["dispatches"] == 2 and d[b]["dispatches"] == 1
    # busy / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs): 2048 / (64 / 8 * 1024)
    assert d[a]["mfma_busy_frac"] == pytest.approx(2048.0 / (64.0 / 8 * 256 * 4))
    assert d[b]["mfma_busy_frac"] == 0.0


def test_c3_traffic_splits_per_step_and_per_update_bytes_and_drops_tuning_trials(tmp_path):
    steps = 2048
    conv = "conv_fwd_lds_kernel<...>"
    gather = "gather_rows_kernel"
    trial = "Cijk_Ailk_Bljk_SB_MT64x64"  # a hipBLASLt solution timed by TunableOp: fewer dispatches than steps
    gemm = "Cijk_Ailk_Bljk_SB_MT128x128"  # the tuned solution, once per step
    bw = "gae_stream_kernel<double, 4, true, 1024, true>"  # the bench's own bandwidth-regime GAE: excluded
    fetch = {"kernels": {conv: {"dispatches": steps, "FETCH_SIZE": 100.0 * steps},
                         gather: {"dispatches": 4, "FETCH_SIZE": 10.0 * 4},
                         trial: {"dispatches": 3, "FETCH_SIZE": 1e9},
                         gemm: {"dispatches": steps, "FETCH_SIZE": 50.0 * steps},
                         bw: {"dispatches": 5, "FETCH_SIZE": 1e9}}}
    write = {"kernels": {conv: {"dispatches": steps, "WRITE_SIZE": 40.0 * steps},
                         gather: {"dispatches": 4, "WRITE_SIZE": 20.0 * 4},
                         trial: {"dispatches": 3, "WRITE_SIZE": 5.0},
                         gemm: {"dispatches": steps, "WRITE_SIZE": 0.0},
                         bw: {"dispatches": 5, "WRITE_SIZE": 1e9}}}
    fj, wj, out = tmp_path / "f.json", tmp_path / "w.json", tmp_path / "t.json"
    fj.write_text(json.dumps(fetch))
    wj.write_text(json.dumps(write))
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"bytes to hash")
    _run(TOOLS / "c3_traffic.py", fj, wj, out, "--lib", lib)
    doc = json.loads(out.read_text())
    per_step = (2 * 100 + 40) * 1024 + (2 * 50 + 0) * 1024  # conv + the tuned GEMM, KiB -> bytes
    outside = (2 * 10 + 20) * 1024 * 4  # the per-epoch gathers, once per update
    assert doc["bytes_per_optimizer_step"] == per_step
    assert doc["bytes_per_update_outside_steps"] == outside
    assert doc["bytes_per_update"] == per_step * steps + outside
    assert doc["bytes_excluded_gemm_tuning_trials"] == round(2 * 1e9 * 1024 + 5 * 1024)
    assert trial not in doc["kernels"] and bw not in doc["kernels"]
    assert doc["kernels"][conv]["per_optimizer_step"] and not doc["kernels"][gather]["per_optimizer_step"]
    assert doc["lib_sha256"] == hashlib.sha256(lib.read_bytes()).hexdigest()
