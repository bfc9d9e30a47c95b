cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_dp.py -q -x > gpurun_out/pytest_dp.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_dp.log; [ $rc -eq 0 ] || exit $rc
RAI_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 0 --num-envs 256 --no-cpu-baseline > gpurun_out/bench2_gloo.log 2>&1; rc=$?; tail -1 gpurun_out/bench2_gloo.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
