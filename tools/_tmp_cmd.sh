cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
( while sleep 45; do echo "tick $(date +%T)"; done ) & TICK=$!
trap "kill $TICK" EXIT
TAG=r1c CONFIGS=cartpole bash tools/profile_bench.sh || exit $?
python tools/pmc_summary.py gpurun_out/prof_r1c/pmc.json "ppo cartpole num_envs=4096/rank n_steps=128" gpurun_out/prof_r1c/fetch_cartpole/run_counter_collection.csv gpurun_out/prof_r1c/write_cartpole/run_counter_collection.csv > /dev/null
rm -f gpurun_out/prof_r1c/*/run_counter_collection.csv
timeout -k 10 400 python -u bench.py > gpurun_out/prof_r1c/bench_default.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/prof_r1c/bench_default.log | cut -c1-300
