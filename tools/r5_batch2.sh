#!/bin/bash
# Round-5 A/B: the C2 epoch kernel with the fast actor loss (alt build, -DRAI_M8_FAST_LOSS) against the
# default build: parity tests under the alt library, then default bench lines with each (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ALT=$PWD/rl-algo-impls_amd/lib/librai_amd_alt.so
RAI_AMD_LIB=$ALT bash tools/gpu_pytest.sh r5m_alt 400 tests/test_gpu_trainer.py -k "fused or c2_horizon or learns" &&
timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/r5m_c2_default.log 2>&1 &&
RAI_AMD_LIB=$ALT timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/r5m_c2_alt.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/r5m_c2_default2.log 2>&1
