#!/bin/bash
# Final-library extras: the C2 default line at --gpus 2 rehearsed on one GPU (gloo setup, both ranks'
# in-kernel exchange on the one device, per-rank geometry) and the C5 bench line (its first update runs
# MIOpen's find-mode tuning for minutes; bench.py prints a heartbeat meanwhile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r5zq}
RAI_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > "gpurun_out/${T}_c2_gpus2_gloo_onegpu.log" 2>&1 || exit 1
timeout -k 10 1000 python -u bench.py --config microrts --steps 1 --warmup 1 --no-cpu-baseline \
  > "gpurun_out/${T}_c5_bench.log" 2>&1 || exit 1
