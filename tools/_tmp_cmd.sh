R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_dp.py -q -x > gpurun_out/pytest_xdp.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pytest_xdp.log | grep -E "passed|failed|Error|error|assert|Mismatch|Max|rank" | head -30; exit $rc
