#!/bin/bash
# MFMA-busy of the dominant kernel of C2 (default and scaled batch policy) and C4 on the current library:
# one SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE counter pass each, restricted to that kernel
# (tools/pmc_kernels.py: busy / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs)).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r5zq}
OUT=gpurun_out/mfma_$T
mkdir -p "$OUT"
sha256sum rl-algo-impls_amd/lib/librai_amd.so > "$OUT/lib_sha256.txt"
run() {  # name regex bench-args...
  local name=$1 rx=$2; shift 2
  timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$rx" \
    --output-format csv -d "$OUT/$name" -o run -- python3 bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline \
    --roofline-reps 5 > "$OUT/$name.log" 2>&1 || { tail -20 "$OUT/$name.log"; exit 1; }
  local f
  f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_kernels.py "$f" "$OUT/$name.json" --delete || exit 1
}
run c2 mlp_ppo_mc8 --config cartpole &&
run c2_scaled lb_grads --config cartpole --batch-policy scaled &&
run c4 mlp_wide_epoch --config halfcheetah &&
python3 - "$OUT" <<'PY'
import json, sys
for n in ("c2", "c2_scaled", "c4"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))["kernels"]
    for k, e in d.items():
        print(f"{n:10s} {e.get('mfma_busy_frac', 0):7.4f}  {e['dispatches']:5d}  {k[:90]}")
PY
