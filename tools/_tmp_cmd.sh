R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 300 python tools/mlp_dp_stamps.py > gpurun_out/dp_stamps.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/dp_stamps.log | tail -16; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m pytest tests/test_gpu_dp.py tests/test_gpu_trainer.py -q -x > gpurun_out/pytest_dp.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_dp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --dp-rehearsal > gpurun_out/bench_dp1.log 2>&1; rc=$?; grep '^{' gpurun_out/bench_dp1.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1.log 2>&1; rc=$?; grep '^{' gpurun_out/bench_1.log | cut -c1-200; exit $rc
