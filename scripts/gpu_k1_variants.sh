# K1 fused vs split variants on the headline bench (same tree, env switch), plus their parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "k1_split" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k1.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_k1.log; exit 1; }
tail -1 gpurun_out/pytest_k1.log
for v in 0 1 2; do
  JX_K1_SPLIT=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k1_$v.json 2> gpurun_out/bench_k1_$v.err || { echo BENCH_FAIL $v; tail -5 gpurun_out/bench_k1_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_k1_$v.json'));print('split=$v', d['value'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['kernels']['reports_per_launch'], d['verified'])"
done
