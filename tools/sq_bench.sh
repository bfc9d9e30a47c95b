#!/bin/bash
# MicroRTS (C5) check: squnet tests, then the bench at 64 envs/GPU (the per-GPU share of C5's 512 envs
# over 8 GPUs) and a rocprofv3 kernel-stats run of it.  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sqb}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_squnet.py tests/test_gridnet.py -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --config microrts --num-envs 64 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu "$OUT/bench.log" | tail -4 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --config microrts --num-envs 64 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/stats.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; rm -f "$OUT/stats/run_kernel_trace.csv"
fi
exit 0
