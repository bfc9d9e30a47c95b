set -u
mkdir -p gpurun_out/cat
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/cat/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/cat/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config pong --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cat/pong.log 2>&1; rc=$?
echo "pong rc=$rc"; grep "timed update 1\|\"value\"" gpurun_out/cat/pong.log | cut -c1-120; exit $rc
