R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -q -x > gpurun_out/pytest_v4.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_v4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mlp_stamps.py > gpurun_out/stamps_v4.log 2>&1; rc=$?; cat gpurun_out/stamps_v4.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_v4.log 2>&1; rc=$?; grep '^{' gpurun_out/bench_v4.log | cut -c1-400; exit $rc
