# K3 (ParallelSum FLP part) load-pipeline variants on the headline bench, plus their parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k3_pipeline" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k3.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_k3.log; exit 1; }
tail -1 gpurun_out/pytest_k3.log
for v in 1 2 12 13; do
  JX_K3_PF=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k3_$v.json 2> gpurun_out/bench_k3_$v.err || { echo BENCH_FAIL $v; tail -5 gpurun_out/bench_k3_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_k3_$v.json'));print('pf=$v', d['value'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['kernels']['reports_per_launch'], d['verified'])"
done
