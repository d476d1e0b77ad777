# Round-end style GPU session: GPU tests, default bench (with CPU baseline), kernel-trace of
# the default bench, and the PMC passes of a one-launch bench for the traffic numbers.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo TRACE_FAIL; tail -20 $OUT/trace_bench.err; exit 1; }
echo TRACE_OK
