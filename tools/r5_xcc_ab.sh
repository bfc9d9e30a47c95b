#!/bin/bash
# Round-5 A/B: the C2 epoch kernel publishing its gradient slots with plain stores when the network's CUs
# share one XCC (default build) against write-through always (alt build, -DRAI_M8_NO_XCC_LOCAL): parity
# tests on the default library, stamps, then C2 bench lines alternating the two libraries (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5za}
ALT=$PWD/rl-algo-impls_amd/lib/librai_amd_alt.so
mkdir -p gpurun_out
bash tools/gpu_pytest.sh ${T}_c2tests 500 tests/test_gpu_trainer.py -k "fused or c2_horizon or learns or reference_steps" &&
bash tools/gpu_pytest.sh ${T}_dptests 400 tests/test_gpu_dp.py -k "fused_dp or env_partition" &&
timeout -k 10 200 python tools/mlp_stamps.py > gpurun_out/${T}_stamps.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/${T}_c2_xcc_$i.log 2>&1 &&
  RAI_AMD_LIB=$ALT timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/${T}_c2_wt_$i.log 2>&1 || exit 1
  echo "pair $i: xcc $(grep -o '"value": [0-9.]*' gpurun_out/${T}_c2_xcc_$i.log | head -1) wt $(grep -o '"value": [0-9.]*' gpurun_out/${T}_c2_wt_$i.log | head -1)"
done
