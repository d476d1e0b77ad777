# Round 3, first GPU pass after the batch-handle engine: the whole -m gpu suite, then the default
# bench with the RCCL world-1 combine timed (--dist) and without.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest.log | head -20
tail -1 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo PYTEST_ABORT $rc; tail -40 $OUT/pytest.log; exit 1; fi
timeout -k 10 400 python -u bench.py --dist --no-cpu-baseline > $OUT/bench_dist.json 2> $OUT/bench_dist.err || { echo BENCH_DIST_FAIL; tail -20 $OUT/bench_dist.err; exit 1; }
cat $OUT/bench_dist.json
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
