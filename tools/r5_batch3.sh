#!/bin/bash
# Round-5: parity tests of both epoch kernels on the current library, then same-box A/B lines: C2 new/base,
# C4 new/base/alt2 (alt2: a timing-only variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5zi}
L=$PWD/rl-algo-impls_amd/lib
mkdir -p gpurun_out
bash tools/gpu_pytest.sh ${T}_tests 600 tests/test_gpu_trainer.py -k "fused or c2_horizon or learns or reference_steps or wide" &&
bash tools/gpu_pytest.sh ${T}_dptests 400 tests/test_gpu_dp.py -k "fused_dp or env_partition or wide_epoch_xdp" &&
timeout -k 10 200 python tools/mlp_stamps.py > gpurun_out/${T}_stamps.txt 2>&1 && timeout -k 10 200 python tools/wide_stamps.py > gpurun_out/${T}_wide_stamps.txt 2>&1 &&
for i in 1 2; do
  for cfg in c2 c4; do
    for v in new base; do
      [ $cfg = c2 ] && [ $v = alt2 ] && continue
      case $v in new) lib=$L/librai_amd.so;; base) lib=$L/librai_amd_alt.so;; alt2) lib=$L/librai_amd_alt2.so;; esac
      if [ $cfg = c2 ]; then args="--steps 2"; else args="--config halfcheetah --steps 1 --warmup 1"; fi
      RAI_AMD_LIB=$lib timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/${T}_${cfg}_${v}_$i.log 2>&1 || exit 1
      echo "$i $cfg $v $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${cfg}_${v}_$i.log | head -1) $(grep -o '"roofline_latency": {[^}]*"achieved": [0-9.]*' gpurun_out/${T}_${cfg}_${v}_$i.log | grep -o 'achieved": [0-9.]*') us/step" | tee -a gpurun_out/${T}_ab.txt
    done
  done
done
