cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_dp.log | grep -v "^$" | tail -25
exit $rc
