set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/gm4
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py -q -k "graphed or wide" --timeout 300 --timeout-method thread > gpurun_out/gm4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/gm4/pytest.log; [ $rc -le 1 ] || exit $rc
for cfg in halfcheetah pong; do
  extra=""; [ $cfg = halfcheetah ] && extra="--num-envs 256"
  timeout -k 10 400 python3 bench.py --config $cfg $extra --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gm4/$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; grep "timed update 1\|\"value\"" gpurun_out/gm4/$cfg.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gm4/hc -o run -- python3 bench.py --config halfcheetah --num-envs 256 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/gm4/hcprof.log 2>&1; rc=$?
rm -f gpurun_out/gm4/hc/run_kernel_trace.csv; echo "prof rc=$rc"
