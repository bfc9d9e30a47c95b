set -u
mkdir -p gpurun_out/hl
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/hl/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/hl/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --config halfcheetah --num-envs 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/hl/hc.log 2>&1; rc=$?
echo "hc rc=$rc"; grep "timed update 1" gpurun_out/hl/hc.log; exit $rc
