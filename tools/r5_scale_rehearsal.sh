#!/bin/bash
# Multi-rank rehearsals of the C2 default line on ONE GPU (gloo setup; every rank's in-kernel exchange runs
# on the one device, so these bound the exchange cost, not xGMI): N = 4 under the default rules (split env
# partition, global minibatch: 64 rows per rank), and N = 2 under the weak-scaling rules (4096 envs and 256
# rows per rank).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r5zq}
RAI_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 1 --warmup 1 --no-cpu-baseline \
  > "gpurun_out/${T}_c2_gpus4_gloo_onegpu.log" 2>&1 || exit 1
RAI_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline \
  --env-partition per-rank --dp-batch per-rank > "gpurun_out/${T}_c2_gpus2_weak_gloo_onegpu.log" 2>&1 || exit 1
