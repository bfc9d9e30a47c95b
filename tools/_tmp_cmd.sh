R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -q -x > gpurun_out/pytest_v2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_v2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mlp_stamps.py > gpurun_out/stamps_v2.log 2>&1; rc=$?; cat gpurun_out/stamps_v2.log | grep -v amdgpu.ids; exit $rc
