#!/bin/bash
# Round-5 A/B, both epoch kernels: hand-off slots published with plain stores when a network's CUs share
# one XCC (default build) against write-through always (alt build: -DRAI_M8_NO_XCC_LOCAL
# -DRAI_WE_NO_XCC_LOCAL).  Parity tests on the default library, stamps, then C2 and C4 bench lines
# alternating the two libraries (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5ze}
ALT=$PWD/rl-algo-impls_amd/lib/librai_amd_alt.so
mkdir -p gpurun_out
bash tools/gpu_pytest.sh ${T}_c2tests 500 tests/test_gpu_trainer.py -k "fused or c2_horizon or learns or reference_steps or wide" &&
bash tools/gpu_pytest.sh ${T}_dptests 500 tests/test_gpu_dp.py -k "fused_dp or env_partition or wide_epoch_xdp" &&
timeout -k 10 200 python tools/mlp_stamps.py > gpurun_out/${T}_stamps.txt 2>&1 &&
timeout -k 10 200 python tools/wide_stamps.py > gpurun_out/${T}_wide_stamps.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/${T}_c2_xcc_$i.log 2>&1 &&
  RAI_AMD_LIB=$ALT timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/${T}_c2_wt_$i.log 2>&1 &&
  timeout -k 10 300 python bench.py --config halfcheetah --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4_xcc_$i.log 2>&1 &&
  RAI_AMD_LIB=$ALT timeout -k 10 300 python bench.py --config halfcheetah --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4_wt_$i.log 2>&1 || exit 1
  for c in c2 c4; do
    echo "pair $i $c: xcc $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${c}_xcc_$i.log | head -1) wt $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${c}_wt_$i.log | head -1)"
  done
done
