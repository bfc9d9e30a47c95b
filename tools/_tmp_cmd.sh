set -u
mkdir -p gpurun_out/tp2
timeout -k 10 300 python -u -m pytest tests/test_gridnet.py tests/test_squnet.py -q --timeout 200 --timeout-method thread > gpurun_out/tp2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/tp2/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u tools/torch_prof.py --config microrts --num-envs 64 --rows 40 > gpurun_out/tp2/microrts.txt 2>&1; rc=$?; echo "prof rc=$rc"; exit $rc
