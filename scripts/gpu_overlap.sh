# Two-stream overlapped fused path: the GPU suite (incl. the multi-launch overlap parity test), then
# the default bench with the overlap on and off, and its kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ovl
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 1 0 1; do
  JX_OVERLAP=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench$v.json 2> $OUT/bench$v.err || { echo BENCH_FAIL $v; tail -20 $OUT/bench$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench$v.json'));print('overlap=$v', d['value'], d['ms_per_step'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['verified'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo TRACE_FAIL; tail -20 $OUT/trace_bench.err; exit 1; }
echo TRACE_OK
