# MFMA K3 iteration: parity (SumVec/FixedPoint/leader), kernel trace of a one-launch bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k3e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fixedpoint.py tests/test_gpu_leader.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
BENCH="bench.py --steps 2 --warmup 1 --reports-per-gpu 262144 --pool 1024 --no-cpu-baseline --no-dist"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/b.json 2> $OUT/b.err || { echo TRACE_FAIL; tail -5 $OUT/b.err; exit 1; }
python3 - $OUT/trace/run_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:4]:
    print("  ", r['Name'][:60], round(float(r['AverageNs'])/1e6,3), "ms")
PY
