set -u
export TMPDIR=/tmp
timeout -k 10 120 python tools/large_stamps.py > gpurun_out/r5o_stamps.txt 2>&1; cat gpurun_out/r5o_stamps.txt
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --kernel-include-regex lb_grads --output-format csv -d gpurun_out/r5o_sq -o run -- python3 tools/large_bench.py --epochs 3 > gpurun_out/r5o_sq.log 2>&1 && echo sq-ok
