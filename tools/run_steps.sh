#!/bin/bash
# GPU-box driver for ad-hoc measurement runs: each argument is "name|timeout|command"; every step
# runs under its own time limit with output in gpurun_out/$OUT/<name>.log, and the script stops at
# the first step that neither passes (0) nor fails tests (1).
#   OUT=r2b bash tools/run_steps.sh "kernels|300|python -m pytest tests/test_gpu_kernels.py -q" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-steps}
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($to s): $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$name.log" | tail -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
