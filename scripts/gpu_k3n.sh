# MFMA K3 iteration: GPU suite, kernel trace of a one-launch bench, short bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k3n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|ERROR|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
BENCH="bench.py --steps 2 --warmup 1 --reports-per-gpu 262144 --pool 1024 --no-cpu-baseline --no-dist"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/b.json 2> $OUT/b.err || { echo TRACE_FAIL; tail -5 $OUT/b.err; exit 1; }
python3 - $OUT/trace/run_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]:
    print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), "ms")
PY
timeout -k 10 300 python -u bench.py --no-cpu-baseline --pool 4096 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'])"
