cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py -m gpu -x -q --timeout 120 --timeout-method thread -k "graphed or learn_epoch or synthetic" > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --config halfcheetah --num-envs 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/hc.log 2>&1 || { tail gpurun_out/hc.log; exit 3; }
tail -1 gpurun_out/hc.log | cut -c1-300
timeout -k 10 300 python bench.py --config pong --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pong.log 2>&1 || { tail gpurun_out/pong.log; exit 3; }
tail -1 gpurun_out/pong.log | cut -c1-300
