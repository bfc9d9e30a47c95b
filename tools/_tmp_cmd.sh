R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/_diag/xchg_diag > $R/gpurun_out/xchg_diag.log 2>&1; rc=$?; cat $R/gpurun_out/xchg_diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/bench_r1b.log 2>&1; rc=$?; grep '^{' $R/gpurun_out/bench_r1b.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex mlp_ppo_epoch --output-format csv -d $R/gpurun_out/pmc_fetch_mlp -o fetch -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 > $R/gpurun_out/pmc_fetch_mlp.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex mlp_ppo_epoch --output-format csv -d $R/gpurun_out/pmc_write_mlp -o write -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 20 > $R/gpurun_out/pmc_write_mlp.log 2>&1; rc=$?; exit $rc
