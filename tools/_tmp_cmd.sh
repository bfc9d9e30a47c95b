R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_trainer.py -q -k "learns_cartpole" --durations=3 > gpurun_out/pytest_learn.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pytest_learn.log | grep -E "passed|failed|assert|reached|s call" | head -10; exit $rc
