#!/bin/bash
# Final-library measurements, part B: C3 whole-update traffic from kernel-group-restricted counter passes
# (tools/c3_pmc_groups.sh), merged (tools/c3_traffic.py) into profiles/<tag>_pong_traffic.json, then the
# C3 bench line (which reads it: same library sha256).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r5y}
TAG=$T bash tools/c3_pmc_groups.sh || exit 1
python3 tools/c3_traffic.py "gpurun_out/c3grp_$T/FETCH_SIZE.json" "gpurun_out/c3grp_$T/WRITE_SIZE.json" \
  "profiles/${T}_pong_traffic.json" || exit 1
cp "profiles/${T}_pong_traffic.json" gpurun_out/  # profiles/ on the box does not travel back
timeout -k 10 600 python -u bench.py --config pong > "gpurun_out/${T}_c3_bench.log" 2>&1 || exit 1
exit 0
