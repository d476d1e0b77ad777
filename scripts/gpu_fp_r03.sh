# configs[4] FixedPoint bench on the current sources (+ kernel trace of the ping-pong)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fp}
mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_fixedpoint.py --skip cpu > $OUT/fp.json 2> $OUT/fp.err || { echo FP_FAIL; tail -20 $OUT/fp.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/fp.json'))
print('pingpong', d.get('value'), d.get('role_ms_per_step'), 'pipelined', d.get('pipelined',{}).get('reports_per_s'))
print('roles_alone', d.get('roles_alone'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 tools/bench_fixedpoint.py --skip cpu,pipelined,helper,leader --steps 1 --warmup 1 > $OUT/fp_trace.json 2> $OUT/fp_trace.err || { echo TRACE_FAIL; tail -5 $OUT/fp_trace.err; exit 1; }
python3 - $OUT/trace/run_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), "ms")
PY
