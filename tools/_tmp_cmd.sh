set -u
mkdir -p gpurun_out/bg
timeout -k 10 400 python -u -m pytest tests/test_squnet.py tests/test_gridnet.py -q --timeout 300 --timeout-method thread > gpurun_out/bg/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/bg/pytest.log; grep -E "FAILED|Error" gpurun_out/bg/pytest.log | head -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --config microrts --num-envs 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bg/mr.log 2>&1; rc=$?
echo "microrts rc=$rc"; grep "timed update" gpurun_out/bg/mr.log; exit $rc
