#!/bin/bash
# Round-5 A/B of the C4 whole-epoch kernel: the current library (new) against lib/librai_amd_alt.so (base: the
# previous commit's build, or an -D variant), after the C4 parity and data-parallel tests on the current
# library; stamps of the current stamps build; then alternating bench lines (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5zg}
ALT=$PWD/rl-algo-impls_amd/lib/librai_amd_alt.so
mkdir -p gpurun_out
bash tools/gpu_pytest.sh ${T}_c2tests 500 tests/test_gpu_trainer.py -k "wide" &&
bash tools/gpu_pytest.sh ${T}_dptests 400 tests/test_gpu_dp.py -k "wide_epoch_xdp or wide_mlp_dp" &&
timeout -k 10 200 python tools/wide_stamps.py > gpurun_out/${T}_wide_stamps.txt 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config halfcheetah --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4_new_$i.log 2>&1 &&
  RAI_AMD_LIB=$ALT timeout -k 10 300 python bench.py --config halfcheetah --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4_base_$i.log 2>&1 || exit 1
  for v in new base; do
    echo "$i $v $(grep -o '"value": [0-9.]*' gpurun_out/${T}_c4_${v}_$i.log | head -1) $(grep -o '"roofline_latency": {[^}]*"achieved": [0-9.]*' gpurun_out/${T}_c4_${v}_$i.log | grep -o 'achieved": [0-9.]*') us/step" | tee -a gpurun_out/${T}_ab.txt
  done
done
