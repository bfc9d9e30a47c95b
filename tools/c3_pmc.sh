#!/bin/bash
# C3 (NatureCNN, 1024 envs x 128 steps) HBM-traffic counters for one whole update.  rocprofv3's
# counter collection segfaults on graph-replayed dispatches (profiles/r3c_pong_fetch_pmc_crash_mapped.txt),
# so the product's graphed step body runs eagerly (GRAPHS=1 GRAPH_EAGER=1: same kernels, no capture).
# Two rocprofv3 passes (FETCH_SIZE and WRITE_SIZE cannot share a pass: 3 + 2 TCC
# counters), each aggregated per kernel ON the box (tools/pmc_kernels.py) so the per-dispatch CSV
# never travels.  Each pass has its own time limit; the script stops at the first failure.
# AUTOGRAD_MT=0: the backward on the calling thread (every dispatch from one host thread).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
OUT=gpurun_out/c3pmc_$TAG
mkdir -p "$OUT/diag"
export RAI_DIAG_DIR="$OUT/diag"   # bench.py dumps /proc/self/maps (start, setup, update0) + faulthandler
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== $C" | tee -a "$OUT/steps.log"
  RAI_AUTOGRAD_MT=${AUTOGRAD_MT:-1} RAI_GRAPHS=${GRAPHS:-0} RAI_ROLLOUT_GRAPH=${GRAPHS:-0} RAI_GRAPH_EAGER=${GRAPH_EAGER:-0} timeout -s KILL 400 rocprofv3 --pmc $C ${KREGEX:+--kernel-include-regex "$KREGEX"} --output-format csv -d "$OUT/$C" -o run -- \
    python3 bench.py --config pong --no-cpu-baseline --roofline-reps 1 --steps 1 --warmup 0 > "$OUT/$C.log" 2>&1
  rc=$?
  sha256sum rl-algo-impls_amd/lib/librai_amd.so > "$OUT/lib_sha256.txt"  # the binary the crash frames map to
  echo "== $C rc=$rc" | tee -a "$OUT/steps.log"
  grep -v amdgpu.ids "$OUT/$C.log" | tail -3
  if [ $rc -ne 0 ]; then  # map the crash's PCs with the newest maps dump of that process
    m=$(ls -t "$OUT"/diag/maps_*.txt 2>/dev/null | head -1)
    [ -n "$m" ] && python3 tools/map_pcs.py "$OUT/$C.log" "$m" > "$OUT/$C.crash_mapped.txt" 2>&1
    exit $rc
  fi
  f=$(find "$OUT/$C" -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_kernels.py "$f" "$OUT/$C.json" --delete || exit 1
done
exit 0
