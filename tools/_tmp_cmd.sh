cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 3; }
tail -2 gpurun_out/pytest_gpu.log
TAG=r1b CONFIGS=cartpole bash tools/profile_bench.sh || exit $?
timeout -k 10 300 python bench.py --config pong --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pong.log 2>&1 || { tail gpurun_out/pong.log; exit 3; }
tail -1 gpurun_out/pong.log
timeout -k 10 300 python bench.py --config halfcheetah --num-envs 256 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/hc.log 2>&1 || { tail gpurun_out/hc.log; exit 3; }
tail -1 gpurun_out/hc.log
