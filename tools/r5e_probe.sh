set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/large_bench.py > gpurun_out/r5e_large_base.txt 2>&1 && cat gpurun_out/r5e_large_base.txt | tail -1 &&
RAI_AMD_LIB=$PWD/rl-algo-impls_amd/lib/librai_amd_alt.so timeout -k 10 120 python tools/large_bench.py > gpurun_out/r5e_large_nofence.txt 2>&1 && tail -1 gpurun_out/r5e_large_nofence.txt &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex lb_grads --output-format csv -d gpurun_out/r5e_sq -o run -- python3 tools/large_bench.py --epochs 3 > gpurun_out/r5e_sq.log 2>&1 && echo sq-ok &&
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex lb_grads --output-format csv -d gpurun_out/r5e_sq2 -o run -- python3 tools/large_bench.py --epochs 3 > gpurun_out/r5e_sq2.log 2>&1 && echo sq2-ok
