R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r1f -o bench -- python $R/bench.py > $R/gpurun_out/prof_r1f_bench.log 2>&1; rc=$?; grep '^{' $R/gpurun_out/prof_r1f_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mlp_ppo_mc|gae_kernel" --output-format csv -d $R/gpurun_out/pmc_fetch_f -o fetch -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 > $R/gpurun_out/pmc_fetch_f.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mlp_ppo_mc|gae_kernel" --output-format csv -d $R/gpurun_out/pmc_write_f -o write -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 > $R/gpurun_out/pmc_write_f.log 2>&1; rc=$?; exit $rc
