#!/bin/bash
# C3 convolution kernels' MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE, tools/pmc_kernels.py)
# from one counter pass restricted to the convolution kernels over one eager C3 update (B = 256 minibatches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r5}
OUT=gpurun_out/c3mfma_$TAG
mkdir -p "$OUT"
sha256sum rl-algo-impls_amd/lib/librai_amd.so > "$OUT/lib_sha256.txt"
RAI_GRAPHS=1 RAI_GRAPH_EAGER=1 timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex conv_ --output-format csv -d "$OUT/mfma" -o run -- python3 bench.py --config pong \
  --no-cpu-baseline --roofline-reps 1 --steps 1 --warmup 0 > "$OUT/mfma.log" 2>&1 || { tail -20 "$OUT/mfma.log"; exit 1; }
f=$(find "$OUT/mfma" -name "*counter_collection.csv" | head -1)
python3 tools/pmc_kernels.py "$f" "$OUT/conv_mfma.json" --delete || exit 1
python3 - "$OUT/conv_mfma.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, e in sorted(d.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
    print(f"{e.get('mfma_busy_frac', 0):6.3f}  {e['dispatches']:6d}  {k[:110]}")
PY
