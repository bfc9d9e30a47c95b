set -u
mkdir -p gpurun_out/pcl
run() { local name=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --config pong --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pcl/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep "timed update 1\|\"value\"" gpurun_out/pcl/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run cl RAI_CHANNELS_LAST=1
run cl_suggest RAI_CHANNELS_LAST=1 PYTORCH_MIOPEN_SUGGEST_NHWC=1
run nchw_find RAI_CUDNN_BENCHMARK=1
