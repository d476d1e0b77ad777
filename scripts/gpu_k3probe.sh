# MFMA K3 variants: 3 groups x 4 calls per step at one workgroup per CU (0) vs 2 groups x 2 calls at two (2)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k3probe}
mkdir -p $OUT
JX_MF_PROBE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "k3_ring or golden" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
BENCH="bench.py --steps 2 --warmup 1 --reports-per-gpu 262144 --pool 1024 --no-cpu-baseline --no-dist"
for pr in 0 2; do
  JX_MF_PROBE=$pr timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$pr -o run -- python3 $BENCH > $OUT/b$pr.json 2> $OUT/b$pr.err || true
  python3 - $OUT/trace$pr/run_kernel_stats.csv $pr <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]:
    if 'mfma' in r['Name']: print("  probe=%s"%sys.argv[2], r['Name'][:50], round(float(r['AverageNs'])/1e6,3), "ms")
PY
done
