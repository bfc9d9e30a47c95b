#!/bin/bash
# C5 (MicroRTS squeeze-U-Net GridNet, 512 envs x 512 steps on one GPU) evidence on one library:
#   1. a rocprofv3 kernel trace of one update after a warm-up update (rollout forward and step bodies
#      eager: graph replay under rocprofv3 aborts inside rocprofiler-sdk, profiles/r6c_c5_trace_crash.txt);
#   2. FETCH_SIZE and WRITE_SIZE passes per kernel group (tools/c3_pmc_groups.sh: the unrestricted pass
#      aborts too, profiles/r6c_c5_all_fetch_crash.txt), merged by tools/c3_traffic.py into
#      profiles/<tag>_microrts_traffic.json (copied to gpurun_out/ for the host);
#   3. the bench line, which reads that summary (same library sha256) for roofline.traffic.
# MIOpen runs immediate mode over the shipped find database (bench.py's C5 default).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r6z}
OUT=gpurun_out/${TAG}_c5
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
export RAI_ROLLOUT_GRAPH=0 RAI_GRAPH_EAGER=1
if [ -z "${SKIP_TRACE:-}" ]; then
  step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py \
    --config microrts --no-cpu-baseline --roofline-reps 1 --steps 1 --warmup 1
  f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/c5_kernel_stats.csv"
  rm -rf "$OUT/trace"
fi
if [ -z "${SKIP_PMC:-}" ]; then
  step pmc 1000 env TAG=${TAG}_c5grp CONFIG=microrts bash tools/c3_pmc_groups.sh
  TRAFFIC_STEPS=86 C3_WORKLOAD="ppo microrts num_envs=512/rank n_steps=512 (eager graph bodies and rollout forward)" \
    python3 tools/c3_traffic.py gpurun_out/c3grp_${TAG}_c5grp/FETCH_SIZE.json gpurun_out/c3grp_${TAG}_c5grp/WRITE_SIZE.json \
    "profiles/${TAG}_microrts_traffic.json" || exit 1
  cp "profiles/${TAG}_microrts_traffic.json" "$OUT/"
fi
unset RAI_ROLLOUT_GRAPH RAI_GRAPH_EAGER
step bench 400 bash -c "python bench.py --config microrts --steps 2 --warmup 1 > $OUT/c5_bench.json 2> $OUT/c5_bench.err"
exit 0
