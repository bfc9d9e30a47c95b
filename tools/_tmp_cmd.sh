cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && export TMPDIR=/tmp
( while sleep 45; do echo "tick $(date +%T)"; done ) & TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
tail -2 gpurun_out/pytest_gpu.log
for c in cartpole pong halfcheetah; do
  timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp/b_$c.log 2>&1 || { tail gpurun_out/exp/b_$c.log; exit 3; }
  echo "$c $(tail -1 gpurun_out/exp/b_$c.log | cut -c80-200)"
done
