R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | grep -E "passed|failed|Error|assert|Mismatch|Max" | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1.log 2>&1; rc=$?; grep '^{' gpurun_out/bench_1.log | cut -c1-200; exit $rc
