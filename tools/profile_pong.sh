#!/bin/bash
# C3 (Pong NatureCNN, 1024 envs x 128 steps) profile on the GPU box:
#   1. kernel-trace stats of the bench run as shipped (graph-replayed update and rollout);
#   2. the MFMA-busy PMC pass of ONE update at the same shape, with the update and rollout forwards
#      run eagerly (RAI_GRAPHS=0 RAI_ROLLOUT_GRAPH=0: the same kernels, launched one by one) and the
#      counters restricted to the contraction and epilogue kernels (--kernel-include-regex).
#      Over the whole update rocprofv3 crashed: SIGSEGV in its counter callback during graph replay
#      (round 1), HSA_STATUS_ERROR_INVALID_PACKET_FORMAT on a torch copy kernel eagerly (r2a).
#      FETCH_SIZE / WRITE_SIZE still segfault restricted (inside MIOpen's convolution dispatch,
#      profiles/r2o_pong_fetch_pmc_crash.txt): PASSES=fetch / write only to re-check that.
# Each step has its own time limit; the script stops at the first step that does not exit 0.
#   TAG=r2a bash tools/profile_pong.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2}
OUT=gpurun_out/prof_pong_$TAG
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$name.log" | grep -v "^    @" | tail -4
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
B="python3 bench.py --config pong --no-cpu-baseline --roofline-reps 20"
# PRETUNE=1: one un-profiled bench run first tunes the fc GEMMs (TunableOp) into a results file the
# profiled runs then reuse, so their traces hold no tuning dispatches (a steady-state profile)
if [ "${PRETUNE:-0}" = 1 ]; then
  export RAI_TUNABLEOP_FILE=/tmp/rai_c3_pretuned%d.csv
  run pretune 300 $B --steps 1 --warmup 0
fi
# DIAG=1: bench.py dumps /proc/self/maps at each stage and Python stacks on a fatal signal into
# $OUT/diag (RAI_DIAG_DIR), so a native crash's PCs map to a library and offset (tools/map_pcs.py)
[ "${DIAG:-0}" = 1 ] && export RAI_DIAG_DIR="$OUT/diag"
if [ "${STATS:-1}" = 1 ]; then
  run stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- $B --steps 2 --warmup 1
  rm -f "$OUT/stats/run_kernel_trace.csv"
fi
export RAI_GRAPHS=0 RAI_ROLLOUT_GRAPH=0
# a PMC pass serialises every dispatch (~125k in one update) and prints nothing for minutes: report
# the growth of its counter CSV every 30 s (progress, not a keep-alive: each step keeps its own limit)
( while sleep 30; do echo "$(date +%T) $(du -sb "$OUT" 2>/dev/null | cut -f1) bytes under $OUT" >> "$OUT/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
REGEX=${REGEX:-"conv_|igemm|Cijk|bias_relu|heads|gather_minibatch"}
for pass in ${PASSES:-mfma}; do
  case $pass in
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    mfma) ctr="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  esac
  run "$pass" 420 rocprofv3 --pmc $ctr --kernel-include-regex "$REGEX" --output-format csv -d "$OUT/$pass" -o run -- \
      $B --steps 1 --warmup 0
  f=$(ls "$OUT/$pass"/*counter_collection.csv | head -1)
  run "${pass}_agg" 300 python3 tools/pmc_kernels.py "$f" "$OUT/${pass}_kernels.json" --delete
done
exit 0
