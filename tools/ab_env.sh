#!/bin/bash
# A/B an environment switch in ONE GPU call (box-to-box drift cancels): bench.py alternately without and
# with "$AB_ENV" (e.g. AB_ENV="RAI_CONV_MFMA_DGRAD=1"), REPS times each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab_${TAG:-x}
mkdir -p "$OUT"
for i in $(seq 1 ${REPS:-3}); do
  for v in base alt; do
    if [ $v = alt ]; then envs=(env $AB_ENV); else envs=(env); fi
    timeout -k 10 400 "${envs[@]}" python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > "$OUT/${v}_$i.log" 2>&1 || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' "$OUT/${v}_$i.log" | head -1) $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${v}_$i.log" | head -1)" | tee -a "$OUT/summary.txt"
  done
done
