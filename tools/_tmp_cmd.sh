set -u
mkdir -p gpurun_out/final3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final3/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/final3/pytest.log; grep FAILED gpurun_out/final3/pytest.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config pong --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/final3/pong.log 2>&1; rc=$?; echo "pong rc=$rc"; grep "timed update 1" gpurun_out/final3/pong.log; exit $rc
