cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && export TMPDIR=/tmp
( while sleep 45; do echo "tick $(date +%T)"; done ) & TICK=$!
trap "kill $TICK" EXIT
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config pong --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp/pong_$tag.log 2>&1 || { tail gpurun_out/exp/pong_$tag.log; exit 3; }
  echo "$tag $(tail -1 gpurun_out/exp/pong_$tag.log | cut -c80-200)"
}
run base RAI_X=0
run bench RAI_CUDNN_BENCHMARK=1
run cl RAI_CHANNELS_LAST=1
run cl_bench RAI_CHANNELS_LAST=1 RAI_CUDNN_BENCHMARK=1
timeout -k 10 300 python -u -m pytest tests/test_evaluation.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_eval.log 2>&1 || { tail -40 gpurun_out/pytest_eval.log; exit 3; }
tail -2 gpurun_out/pytest_eval.log
