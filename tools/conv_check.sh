#!/bin/bash
# C3 convolution kernels on the GPU box: their tests, the per-layer A/B timing against MIOpen, the
# Pong parity tests through the product path, and the C3 bench with the MFMA kernels on / off.
# Each step under its own limit; stops at the first step that does not pass.
#   TAG=r3p STEPS=test,bench,pong,c3 bash tools/conv_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
OUT=gpurun_out/conv_$TAG
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$name.log" | tail -4
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
S=${STEPS:-test,bench,pong,c3}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
[[ $S == *test* ]] && run test 400 $PT tests/test_gpu_conv.py -m gpu
[[ $S == *bench* ]] && run bench 300 python3 tools/conv_bench.py --reps 30
[[ $S == *pong* ]] && run pong 900 $PT tests/test_gpu_pong.py -m gpu
[[ $S == *c3* ]] && run c3_mfma 400 python3 bench.py --config pong --steps 3 --warmup 1 --no-cpu-baseline
[[ $S == *c3* ]] && RAI_CONV_MFMA=0 run c3_miopen 400 python3 bench.py --config pong --steps 3 --warmup 1 --no-cpu-baseline
[[ $S == *prof* ]] && run c3prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3prof" -o run -- \
  python3 bench.py --config pong --steps 2 --warmup 1 --no-cpu-baseline
rm -f "$OUT"/*/run_kernel_trace.csv
exit 0
