# K1 with non-temporal meas-share stores: parity subset + bench twice.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ntst
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "golden or k1_split" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo BENCH_FAIL; tail -20 $OUT/bench$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench$i.json'));print('nt', d['value'], d['ms_per_step'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['verified'])"
done
