#!/bin/bash
# Round-5 A/B/C of one config's bench line across libraries (same box, alternating): the current library
# (new), lib/librai_amd_alt.so (base) and lib/librai_amd_alt2.so (a timing-only variant), after the
# config's parity tests on the current library.
#   TAG=... CFG="--config halfcheetah --steps 1 --warmup 1" TESTS="tests/test_gpu_trainer.py -k wide" bash tools/r5_ab3.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5zh}
L=$PWD/rl-algo-impls_amd/lib
mkdir -p gpurun_out
bash tools/gpu_pytest.sh ${T}_tests 500 ${TESTS} &&
for i in 1 2 3; do
  for v in new base alt2; do
    case $v in new) lib=$L/librai_amd.so;; base) lib=$L/librai_amd_alt.so;; alt2) lib=$L/librai_amd_alt2.so;; esac
    RAI_AMD_LIB=$lib timeout -k 10 300 python bench.py ${CFG} --no-cpu-baseline > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    echo "$i $v $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${v}_$i.log | head -1) $(grep -o '"roofline_latency": {[^}]*"achieved": [0-9.]*' gpurun_out/${T}_${v}_$i.log | grep -o 'achieved": [0-9.]*') us/step" | tee -a gpurun_out/${T}_ab.txt
  done
done
