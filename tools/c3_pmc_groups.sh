#!/bin/bash
# C3 whole-update HBM traffic assembled from kernel-GROUP-restricted counter passes (the unrestricted
# whole-update pass aborts inside rocprofiler-sdk: profiles/r3c/r3zd/r3ze/r4b_*_crash_mapped.txt).
# Groups: ours (this repo's HIP kernels), gemm (hipBLASLt / rocBLAS), rest (everything else: torch
# elementwise, copies, MIOpen if any).  Per group a FETCH_SIZE and a WRITE_SIZE pass over one eager C3
# update (the product's graphed step body launched eagerly, RAI_GRAPH_EAGER=1), aggregated per kernel on
# the box (tools/pmc_kernels.py); tools/c3_traffic.py then merges them.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r4}
CONFIG=${CONFIG:-pong}  # round 6: any bench config (microrts for C5); GROUPS_=all: one unrestricted pass per counter
# (COUNTERS restricts the passes to a subset of FETCH_SIZE WRITE_SIZE)
OUT=gpurun_out/c3grp_$TAG
mkdir -p "$OUT"
# round 5: "ours" split into the convolutions and the rest of this repo's kernels (the round-5 run of the
# combined group aborted inside rocprofiler-sdk at a conv_wrw_kernel launch: profiles/r5y_c3_ours_fetch_crash.txt)
CONV='conv_'
OURS='rai_|gather|bias_relu|heads|pg_loss|loss_|clip_optim|grad_sumsq|gae|sample|policy|minibatch'
GEMM='Cijk|gemm|Gemm|GEMM'
sha256sum rl-algo-impls_amd/lib/librai_amd.so > "$OUT/lib_sha256.txt"
for grp in ${GROUPS_:-conv ours gemm rest}; do
  case $grp in
    conv) sel=(--kernel-include-regex "$CONV") ;;
    ours) sel=(--kernel-include-regex "$OURS") ;;
    gemm) sel=(--kernel-include-regex "$GEMM") ;;
    rest) sel=(--kernel-exclude-regex "$CONV|$OURS|$GEMM") ;;
    # "rest" split in two (round 6: a C5 rest WRITE_SIZE pass ended in a SIGSEGV inside the profiler's
    # dispatch path at a torch reduction launch, profiles/r6z_c5_rest_write_crash.txt)
    restat) sel=(--kernel-include-regex "at::native") ;;
    restx) sel=(--kernel-exclude-regex "$CONV|$OURS|$GEMM|at::native") ;;
    all) sel=() ;;
  esac
  for C in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
    echo "== $grp $C" | tee -a "$OUT/steps.log"
    RAI_GRAPHS=1 RAI_GRAPH_EAGER=1 timeout -s KILL 400 rocprofv3 --pmc $C "${sel[@]}" --output-format csv \
      -d "$OUT/${grp}_$C" -o run -- python3 bench.py --config "$CONFIG" --no-cpu-baseline --roofline-reps 1 --steps 1 \
      --warmup 0 ${BENCH_EXTRA:-} > "$OUT/${grp}_$C.log" 2>&1
    rc=$?
    echo "== $grp $C rc=$rc" | tee -a "$OUT/steps.log"
    [ $rc -eq 0 ] || { grep -v amdgpu.ids "$OUT/${grp}_$C.log" | tail -20; exit $rc; }
    f=$(find "$OUT/${grp}_$C" -name "*counter_collection.csv" | head -1)
    python3 tools/pmc_kernels.py "$f" "$OUT/${grp}_$C.json" --delete || exit 1
  done
done
python3 - "$OUT" ${GROUPS_:-conv ours gemm rest} <<'PY'
import json, sys
out = sys.argv[1]
import os
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    merged = {"kernels": {}}
    for g in sys.argv[2:]:
        if os.path.exists(f"{out}/{g}_{c}.json"):  # COUNTERS may restrict a run to one counter
            merged["kernels"].update(json.load(open(f"{out}/{g}_{c}.json"))["kernels"])
    json.dump(merged, open(f"{out}/{c}.json", "w"), indent=1)
PY
exit 0
