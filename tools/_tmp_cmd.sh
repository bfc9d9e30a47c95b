set -u
mkdir -p gpurun_out/xdp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -v --timeout 300 --timeout-method thread > gpurun_out/xdp/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL" gpurun_out/xdp/pytest.log | cut -c1-120; exit $rc
