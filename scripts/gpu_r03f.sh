# lane-pair helper K1: the GPU suite (small batches run it by default), then configs[4] with it
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|ERROR|Error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u tools/bench_fixedpoint.py --skip cpu,leader > $OUT/fp.json 2> $OUT/fp.err || { echo FP_FAIL; tail -20 $OUT/fp.err; exit 1; }
cat $OUT/fp.json
