R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out && cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_trainer.py -q -k "fused_epoch_matches_generic" > gpurun_out/pytest_fg.log 2>&1; rc=$?; grep -E "passed|failed|Error|assert|Mismatch|Max" gpurun_out/pytest_fg.log | head -40; exit $rc
