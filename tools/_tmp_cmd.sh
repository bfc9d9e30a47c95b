set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r1g
timeout -k 10 600 python bench.py > gpurun_out/r1g/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -v amdgpu gpurun_out/r1g/bench.log | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc
TAG=r1g CONFIGS=cartpole bash tools/profile_bench.sh > gpurun_out/r1g/prof_steps.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for cfg in pong halfcheetah microrts; do
  extra=""; [ $cfg = halfcheetah ] && extra="--num-envs 256"; [ $cfg = microrts ] && extra="--num-envs 64"
  timeout -k 10 400 python3 bench.py --config $cfg $extra --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1g/$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; grep "timed update 1" gpurun_out/r1g/$cfg.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1g/mr -o run -- python3 bench.py --config microrts --num-envs 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r1g/mrprof.log 2>&1; rc=$?; rm -f gpurun_out/r1g/mr/run_kernel_trace.csv; echo "mrprof rc=$rc"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1g/pong -o run -- python3 bench.py --config pong --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r1g/pongprof.log 2>&1; rc=$?; rm -f gpurun_out/r1g/pong/run_kernel_trace.csv; echo "pongprof rc=$rc"
