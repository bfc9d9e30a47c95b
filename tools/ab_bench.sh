#!/bin/bash
# A/B a kernel variant in ONE GPU call (box-to-box drift cancels): the C4 bench alternately on the
# shipped library and on lib/librai_amd_alt.so (build.py alt, RAI_ALT_FLAGS), REPS times each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_${TAG:-x}
mkdir -p "$OUT"
for i in $(seq 1 ${REPS:-3}); do
  for v in base alt; do
    if [ $v = alt ]; then export RAI_AMD_LIB=rl-algo-impls_amd/lib/librai_amd_alt.so; else unset RAI_AMD_LIB; fi
    timeout -k 10 300 python3 bench.py ${BENCH_ARGS:---config halfcheetah --num-envs 256 --steps 2 --warmup 1} > "$OUT/${v}_$i.log" 2>&1 || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' "$OUT/${v}_$i.log" | head -1) $(grep -o '"avg_ms": [0-9.]*' "$OUT/${v}_$i.log" | head -1)" | tee -a "$OUT/summary.txt"
  done
done
