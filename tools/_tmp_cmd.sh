set -u
mkdir -p gpurun_out/gm5
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainer.py -q -k "gather or graphed or wide" --timeout 200 --timeout-method thread > gpurun_out/gm5/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/gm5/pytest.log; [ $rc -le 1 ] || exit $rc
for cfg in halfcheetah pong; do
  extra=""; [ $cfg = halfcheetah ] && extra="--num-envs 256"
  timeout -k 10 400 python3 bench.py --config $cfg $extra --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gm5/$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; grep "timed update 1" gpurun_out/gm5/$cfg.log; [ $rc -eq 0 ] || exit $rc
done
