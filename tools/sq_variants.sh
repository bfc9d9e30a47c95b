#!/bin/bash
# MicroRTS (C5) memory-format experiment: the bench at 64 envs with NCHW activations, NHWC
# activations, and NHWC with MIOpen's NHWC suggestion; each run under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sqv
run() { local name=$1; shift; echo "== $name"; env "$@" timeout -k 10 400 python -u bench.py --config microrts --num-envs 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sqv/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu gpurun_out/sqv/$name.log | tail -3 | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run nchw RAI_SQUNET_NHWC=0
run nhwc RAI_SQUNET_NHWC=1
run nhwc_suggest RAI_SQUNET_NHWC=1 PYTORCH_MIOPEN_SUGGEST_NHWC=1
