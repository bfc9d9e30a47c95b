#!/bin/bash
# Round measurements on the GPU box: selected steps (MEASURE=c2,c2prof,c4,c4prof,gae,c3,c5) each under its own
# time limit, outputs under gpurun_out/$TAG/.  Stops at the first step that fails (non-zero exit).
#   TAG=r3a MEASURE=c2,c4,gae bash tools/measure.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$name.log" | tail -3
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
M=${MEASURE:-c2,gae}
[[ $M == *c2,* || $M == c2 || $M == *,c2 ]] && run c2 400 python3 bench.py --steps 5 --warmup 1
[[ $M == *c2prof* ]] && run c2prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c2prof" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
[[ $M == *c4,* || $M == c4 || $M == *,c4 ]] && run c4 600 python3 bench.py --config halfcheetah --num-envs 256 --steps 3 --warmup 1
[[ $M == *c4prof* ]] && run c4prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- \
  python3 bench.py --config halfcheetah --num-envs 256 --steps 2 --warmup 1
[[ $M == *gae* ]] && run gae 300 python3 tools/gae_bench.py
[[ $M == *c3* ]] && run c3 600 python3 bench.py --config pong --steps 3 --warmup 1
[[ $M == *c5* ]] && run c5 900 python3 bench.py --config microrts --num-envs 64 --steps 2 --warmup 1
rm -f "$OUT"/*/run_kernel_trace.csv
exit 0
