#!/bin/bash
# One pytest -m gpu invocation on the GPU box under its own time limit, output in gpurun_out/<name>.log.
#   bash tools/gpu_pytest.sh <name> <timeout_s> <pytest args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAI_TEST_REPORT_DIR=gpurun_out/reports
name=$1 to=$2; shift 2
echo "== $name: pytest $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$to" python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
tail -3 "gpurun_out/$name.log"
# 0 pass, 1 test failures: keep going; anything else (fault, abort, timeout) stops the caller's chain
[ $rc -eq 0 ] || [ $rc -eq 1 ]
