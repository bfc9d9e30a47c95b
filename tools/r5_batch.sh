#!/bin/bash
# Round-5 GPU batch: split-K conv tests, rollout / policy-step tests, conv forward A/B, C2 rollout timing,
# scaled C2 bench.  Stops at the first step that fails (each under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_pytest.sh r5l_conv 300 tests/test_gpu_conv.py -k "splitk or fwd_matches or nature" &&
bash tools/gpu_pytest.sh r5k_t 400 tests/test_gpu_scaled.py tests/test_gpu_trainer.py tests/test_gpu_returns.py tests/test_gpu_kernels.py \
  -k "staging or c2 or scaled or learns or rollout or policy_step or sample" &&
timeout -k 10 200 python tools/conv_bench.py --batches 256,1024 --variants 0 > gpurun_out/r5l_conv_bench_splitk.txt 2>&1 &&
RAI_CONV_FWD_SPLITK=0 timeout -k 10 200 python tools/conv_bench.py --batches 256 --variants 0 \
  > gpurun_out/r5l_conv_bench_nosplit.txt 2>&1 &&
RAI_CONV_FWD_WPC=1 timeout -k 10 200 python tools/conv_bench.py --batches 256,1024 --variants 0 \
  > gpurun_out/r5l_conv_bench_wpc1.txt 2>&1 &&
timeout -k 10 120 python tools/large_bench.py --epochs 10 > gpurun_out/r5k_lb.txt 2>&1 &&
timeout -k 10 200 python tools/c2_rollout_timing.py > gpurun_out/r5k_c2_rollout.txt 2>&1 &&
timeout -k 10 300 python bench.py --batch-policy scaled --no-cpu-baseline > gpurun_out/r5k_scaled.log 2>&1
