set -u
mkdir -p gpurun_out/final2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final2/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final2/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/final2/pytest.log; exit $rc
