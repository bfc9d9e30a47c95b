R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_dp.py -q -x > gpurun_out/pytest_dp.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_dp.log; exit $rc
