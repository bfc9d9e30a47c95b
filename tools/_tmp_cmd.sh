cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && export TMPDIR=/tmp
timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/hcw_stats -o run -- python3 -u bench.py --config halfcheetah --num-envs 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/exp/hcw_stats.log 2>&1; echo "rc=$?"
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/exp/hcw_stats/run_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
# take a window in the middle of the timed update
mid=len(rows)//2
w=rows[mid:mid+60]
t0=int(w[0]['Start_Timestamp'])
for r in w:
    s,e=int(r['Start_Timestamp'])-t0,int(r['End_Timestamp'])-t0
    print(f"{s/1000:9.2f} {e/1000:9.2f} {(e-s)/1000:7.2f} {r['Kernel_Name'][:70]}")
PY
rm -f gpurun_out/exp/hcw_stats/run_kernel_trace.csv
