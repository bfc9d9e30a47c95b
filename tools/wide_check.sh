#!/bin/bash
# C4 epoch-kernel iteration on the GPU box: the wide-MLP parity tests, then the per-phase stamps
# (tools/wide_stamps.py, diagnostic build) and the halfcheetah bench.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-wide}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-4}
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest tests/test_gpu_trainer.py -m gpu -x -v --timeout 200 --timeout-method thread -k "${PYTEST_K:-wide}"
TAILN=20 run stamps 200 python tools/wide_stamps.py
[[ ${BENCH:-1} == 1 ]] && run c4 600 python bench.py --config halfcheetah --num-envs 256 --steps 3 --warmup 1
exit 0
