#!/bin/bash
# Final-library measurements, part A: C2 (default and scaled batch policy) and C4 -- rocprofv3 kernel stats and
# the FETCH / WRITE passes (same library sha256), then the bench lines with that PMC summary in place (so
# their roofline.traffic is filled) and the CPU baseline.  Output under gpurun_out/; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r5y}
OUT=gpurun_out/prof_$T
TAG=$T CONFIGS="cartpole halfcheetah" bash tools/profile_bench.sh || exit 1
mv "$OUT/stats_cartpole" "$OUT/stats_cartpole_yaml"
TAG=$T CONFIGS=cartpole EXTRA="--batch-policy scaled" bash tools/profile_bench.sh || exit 1
mv "$OUT/stats_cartpole" "$OUT/stats_cartpole_scaled"
cp "$OUT/pmc.json" "profiles/${T}_pmc.json"
timeout -k 10 400 python bench.py > "gpurun_out/${T}_c2_bench.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py --batch-policy scaled > "gpurun_out/${T}_c2_scaled_bench.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py --config halfcheetah > "gpurun_out/${T}_c4_bench.log" 2>&1 || exit 1
exit 0
