# K3 ring variants (JX_K3V: 0 four-wave workgroups + barrier, 1/2 one wave per workgroup with ring depth 3/4)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k3v
mkdir -p $OUT
for v in 1 2; do
  JX_K3V=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest$v.log 2>&1 || { echo PYTEST_FAIL $v; tail -30 $OUT/pytest$v.log; exit 1; }
  tail -1 $OUT/pytest$v.log
done
for v in 0 1 2 0; do
  JX_K3V=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --pool 4096 > $OUT/bench$v.json 2> $OUT/bench$v.err || { echo BENCH_FAIL; tail -20 $OUT/bench$v.err; exit 1; }
  echo "v=$v $(tail -1 $OUT/bench$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'])")"
done
