#!/bin/bash
# Same-box A/B of a C3 switch (env var AB_VAR): the conv tests, the Pong parity tests with the switch on,
# then the C3 bench alternately on / off, REPS times.  Stops at the first step that does not pass.
#   TAG=r3z AB_VAR=RAI_CONV_FUSE_RELU_BWD bash tools/ab_c3.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab_c3_${TAG:-x}
mkdir -p "$OUT"
V=${AB_VAR:?AB_VAR}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$name.log" | tail -2
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run test 400 $PT tests/test_gpu_conv.py -m gpu
export "$V=1"
run pong 900 $PT tests/test_gpu_pong.py -m gpu
for i in $(seq 1 ${REPS:-2}); do
  for s in 1 0; do
    export "$V=$s"
    run "c3_${s}_$i" 400 python3 bench.py --config pong --steps 3 --warmup 1 --no-cpu-baseline
    echo "$V=$s rep $i $(grep -o '"value": [0-9.]*' "$OUT/c3_${s}_$i.log" | head -1)" | tee -a "$OUT/summary.txt"
  done
done
exit 0
