#!/bin/bash
# GPU-box validation run: smoke -> pytest -m gpu -> short bench.  Each GPU step has
# its own time limit; the script stops at the first fault/abort/timeout (exit codes
# other than 0 = pass and 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAI_TEST_REPORT_DIR=gpurun_out/reports
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench}
[[ $STEPS == *smoke* ]] && step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
if [[ -n ${PYTEST_K:-} ]]; then KARGS=(-k "$PYTEST_K"); else KARGS=(); fi
[[ $STEPS == *pytest* ]] && step pytest_gpu 1000 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v --timeout 300 --timeout-method thread "${KARGS[@]}" ${PYTEST_ARGS:-}
[[ $STEPS == *bench* ]] && step bench 900 python bench.py ${BENCH_ARGS:-}
[[ $STEPS == *gaebench* ]] && step gaebench 300 python tools/gae_bench.py
exit 0
