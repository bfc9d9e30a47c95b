R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 300 python tools/mlp_stamps.py > gpurun_out/stamps_v4.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamps_v4.log; exit $rc
