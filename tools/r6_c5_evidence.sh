#!/bin/bash
# C5 (MicroRTS squeeze-U-Net GridNet, 512 envs x 512 steps on one GPU) evidence on one library: a bench
# line (the shipped MIOpen find database seeded by running_utils), a rocprofv3 kernel trace of one update,
# then FETCH_SIZE and WRITE_SIZE passes over one update (tools/c3_pmc_groups.sh, GROUPS_=all) merged by
# tools/c3_traffic.py into profiles-ready JSON.  Each GPU step has its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r6c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
sha256sum rl-algo-impls_amd/lib/librai_amd.so > "$OUT/lib_sha256.txt"
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_BENCH:-}" ]; then
  step bench 400 bash -c "python bench.py --config microrts --steps 2 --warmup 1 > $OUT/c5_bench.json 2> $OUT/c5_bench.err"
  du -sh ~/.cache/miopen 2>&1 | tee -a "$OUT/steps.log"  # MIOpen's compiled-kernel cache (later runs reuse it)
fi
# graph replay under rocprofv3 aborts inside rocprofiler-sdk (profiles/r6c_c5_trace_crash.txt, r3c): the
# rollout forward and the update's step bodies run eagerly in the profiled runs (same kernels, no capture)
export RAI_ROLLOUT_GRAPH=0 RAI_GRAPH_EAGER=1
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py \
  --config microrts --no-cpu-baseline --roofline-reps 1 --steps 1 --warmup 1
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/c5_kernel_stats.csv"
rm -rf "$OUT/trace"
step pmc 700 env TAG=${TAG}_c5 CONFIG=microrts GROUPS_=all bash tools/c3_pmc_groups.sh
TRAFFIC_STEPS=86 C3_WORKLOAD="ppo microrts num_envs=512/rank n_steps=512 (eager graph bodies, RAI_GRAPH_EAGER=1)" \
  python3 tools/c3_traffic.py gpurun_out/c3grp_${TAG}_c5/FETCH_SIZE.json gpurun_out/c3grp_${TAG}_c5/WRITE_SIZE.json \
  "$OUT/c5_traffic.json"
exit 0
