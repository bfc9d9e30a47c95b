#!/bin/bash
# C3 FETCH_SIZE crash diagnosis.  ONE crashing step per GPU call at most:
#   WHAT=repro  NatureCNN's three convolutions alone (tools/miopen_pmc_repro.py, no code of ours)
#   WHAT=bench  the C3 bench update, as profiles/r2o_pong_fetch_pmc_crash.txt
# under `rocprofv3 --pmc FETCH_SIZE`, with /proc/self/maps and Python stacks dumped to
# $OUT/diag so the crash's PCs map to libraries (tools/map_pcs.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
OUT=gpurun_out/pmcdiag_$TAG
mkdir -p "$OUT/diag"
export RAI_DIAG_DIR="$OUT/diag"
case ${WHAT:-repro} in
  repro) cmd=(python3 tools/miopen_pmc_repro.py --iters 3) ;;
  repro_nofind) cmd=(python3 tools/miopen_pmc_repro.py --iters 3 --no-find) ;;
  bench) cmd=(python3 bench.py --config pong --no-cpu-baseline --roofline-reps 5 --steps 1 --warmup 0) ;;
esac
echo "== ${WHAT:-repro}: rocprofv3 --pmc FETCH_SIZE -- ${cmd[*]}" | tee "$OUT/steps.log"
RAI_GRAPHS=0 RAI_ROLLOUT_GRAPH=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
  -d "$OUT/pmc" -o run -- "${cmd[@]}" > "$OUT/run.log" 2>&1
rc=$?
echo "== rc=$rc" | tee -a "$OUT/steps.log"
grep -v amdgpu.ids "$OUT/run.log" | tail -40
crash="$OUT/run.log"
for m in "$OUT"/diag/*maps*.txt; do
  [ -f "$m" ] && python3 tools/map_pcs.py "$crash" "$m" > "$m.mapped" 2>&1
done
ls -la "$OUT/diag"
find "$OUT/pmc" -name "*counter_collection.csv" -size +10M -delete 2>/dev/null
exit 0
