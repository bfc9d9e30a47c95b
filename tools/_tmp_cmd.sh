set -u
mkdir -p gpurun_out/pc
for tree in _oldtree .; do
  name=$( [ $tree = . ] && echo new || echo old )
  (cd $tree && timeout -k 10 300 python -u bench.py --config pong --steps 2 --warmup 1 --no-cpu-baseline > /root/repo/gpurun_out/pc/pong_$name.log 2>&1); rc=$?
  echo "$name rc=$rc"; grep "timed update\|\"value\"" gpurun_out/pc/pong_$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
