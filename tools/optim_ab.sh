#!/bin/bash
# A/B of the one-launch clip + Adam against the two-launch form (RAI_OPTIM_FUSED=0) on the
# graph-replayed configs, then rocprof kernel stats of the one-launch form.  Each GPU step runs
# under its own time limit; the script stops at the first step that does not exit 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/optim_ab
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -1 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
for c in ${CONFIGS:-halfcheetah pong}; do
  RAI_OPTIM_FUSED=0 run "${c}_two" 400 python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline
  RAI_OPTIM_FUSED=1 run "${c}_one" 400 python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline
done
if [ -n "${STATS:-}" ]; then
  run stats 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$STATS" -o run -- \
      python3 bench.py --config "$STATS" --steps 2 --warmup 1 --no-cpu-baseline
  rm -f "$OUT/stats_$STATS/run_kernel_trace.csv"
fi
exit 0
