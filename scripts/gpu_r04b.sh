# Round 4: the ordering tests, then the rest of the GPU suite from where r04a stopped, then the driver's bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ordering.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_order.log 2>&1 || { echo ORDER_FAIL; tail -40 $OUT/pytest_order.log; exit 1; }
tail -1 $OUT/pytest_order.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
tail -c 3000 $OUT/bench.json
timeout -k 10 400 bash tools/k3_probe.sh gpurun_out/r04b/k3probe || { echo PROBE_FAIL; exit 1; }
