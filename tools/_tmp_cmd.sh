cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_dp.log | grep -v "^$" | tail -25
[ $rc -eq 0 ] || exit 3
timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/hcw_stats -o run -- python3 -u bench.py --config halfcheetah --num-envs 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/exp/hcw_stats.log 2>&1; echo "rc=$?"
rm -f gpurun_out/exp/hcw_stats/run_kernel_trace.csv
timeout -k 10 200 python -u bench.py --config halfcheetah --num-envs 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp/b_hc256w.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/exp/b_hc256w.log | cut -c1-220
