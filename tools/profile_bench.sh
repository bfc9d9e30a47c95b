#!/bin/bash
# GPU-box profiling run for the bench workload(s): rocprofv3 kernel-trace stats of bench.py, then one
# PMC pass per TCC counter (FETCH_SIZE and WRITE_SIZE cannot share a pass), each step under its own
# time limit; stops at the first step that does not exit 0.  Output: gpurun_out/prof_<tag>/...
#   TAG=r1b CONFIGS="cartpole pong" bash tools/profile_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
CONFIGS=${CONFIGS:-cartpole}
OUT=gpurun_out/prof_$TAG
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
for c in $CONFIGS; do
  extra=${EXTRA:-}
  run "stats_$c" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$c" -o run -- \
      python3 bench.py --config "$c" --steps 2 --warmup 1 --no-cpu-baseline $extra
  rm -f "$OUT/stats_$c/run_kernel_trace.csv"  # traces run to 100s of MB (gpurun returns <= 64 MiB); stats stay
  if [ "${PMC:-1}" = 1 ]; then
    run "fetch_$c" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$c" -o run -- \
        python3 bench.py --config "$c" --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 $extra
    run "write_$c" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$c" -o run -- \
        python3 bench.py --config "$c" --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 $extra
    # per-kernel medians + the library's sha256 (bench.py reports traffic only for the same binary)
    wl=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['config']['workload'])" "$OUT/write_$c.log")
    fcsv=$(find "$OUT/fetch_$c" -name "*counter_collection.csv" | head -1)
    wcsv=$(find "$OUT/write_$c" -name "*counter_collection.csv" | head -1)
    python3 tools/pmc_summary.py "$OUT/pmc.json" "$wl" "$fcsv" "$wcsv" > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc_summary failed"; exit 1; }
    find "$OUT" -name "*counter_collection.csv" -size +20M -delete
  fi
  if [ -n "${MFMA_PMC:-}" ]; then
    run "mfma_$c" 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
        --output-format csv -d "$OUT/mfma_$c" -o run -- \
        python3 bench.py --config "$c" --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 $extra
  fi
done
exit 0
