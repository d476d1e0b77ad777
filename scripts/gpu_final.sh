# Final check on the committed tree: the whole GPU suite, the driver's bench command (CPU baseline included;
# the committed PMC summary fills roofline.traffic when the kernel sources match it), and rocprofv3 kernel
# stats of the same command (the per-kernel averages the bench's HIP-event times must agree with).
# usage: bash scripts/gpu_final.sh <name>   (outputs under gpurun_out/<name>/)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo TRACE_FAIL; tail -20 $OUT/trace_bench.err; exit 1; }
echo TRACE_OK
