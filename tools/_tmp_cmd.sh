cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && export TMPDIR=/tmp
for c in 8 16 32; do
  RAI_GAE_COLS=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gae" > gpurun_out/exp/pytest_gae_$c.log 2>&1 || { tail -20 gpurun_out/exp/pytest_gae_$c.log; exit 3; }
  for cfg in cartpole halfcheetah; do
    RAI_GAE_COLS=$c timeout -k 10 300 python -u bench.py --config $cfg --num-envs $([ $cfg = cartpole ] && echo 4096 || echo 2048) --steps 1 --warmup 0 --no-cpu-baseline --roofline-reps 400 > gpurun_out/exp/bench_gae_$c.log 2>&1 || exit 3
    echo "cols=$c $cfg $(tail -1 gpurun_out/exp/bench_gae_$c.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['roofline_gae']['avg_us'], d['roofline_gae']['frac'])")"
  done
done
