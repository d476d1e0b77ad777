# GPU session: GPU tests, kernel-trace stats and PMC passes of a one-launch bench, and the
# VALU microbenchmark under the same counters (calibrates thread-cycles per instruction).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH="bench.py --steps 1 --warmup 0 --reports-per-gpu 312500 --pool 512 --no-cpu-baseline"
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo TRACE_FAIL; tail -20 $OUT/trace_bench.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc_sq -o run -- python3 $BENCH > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || { echo PMC_SQ_FAIL; tail -5 $OUT/pmc_sq.err; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python3 $BENCH > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo PMC_FETCH_FAIL; tail -5 $OUT/pmc_fetch.err; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python3 $BENCH > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo PMC_WRITE_FAIL; tail -5 $OUT/pmc_write.err; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $OUT/pmc_mb -o run -- ./tools/bin/microbench_valu 16384 > $OUT/pmc_mb.jsonl 2> $OUT/pmc_mb.err || { echo PMC_MB_FAIL; tail -5 $OUT/pmc_mb.err; }
python3 tools/prof_summary.py $OUT --reports-per-launch 312500 > $OUT/summary.json && echo SUMMARY_OK
