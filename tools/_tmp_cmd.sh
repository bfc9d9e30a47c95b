set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r1f
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1f/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r1f/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r1f/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -v amdgpu gpurun_out/r1f/bench.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
TAG=r1f CONFIGS=cartpole bash tools/profile_bench.sh > gpurun_out/r1f/prof_steps.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for cfg in pong halfcheetah microrts; do
  extra=""; [ $cfg = halfcheetah ] && extra="--num-envs 256"; [ $cfg = microrts ] && extra="--num-envs 64"
  timeout -k 10 400 python3 bench.py --config $cfg $extra --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1f/$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; grep "timed update 1" gpurun_out/r1f/$cfg.log; [ $rc -eq 0 ] || exit $rc
done
