R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; exit $rc
