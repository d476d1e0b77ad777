# GPU session: VALU microbench, GPU tests, kernel-trace stats and PMC passes of the bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
OUT=gpurun_out
BENCH="bench.py --steps 1 --warmup 0 --reports-per-gpu 312500 --pool 512 --no-cpu-baseline"
timeout -k 10 120 ./tools/bin/microbench_valu 4096 > $OUT/microbench_valu.jsonl 2>&1 || { echo MB_FAIL; cat $OUT/microbench_valu.jsonl; exit 1; }
cat $OUT/microbench_valu.jsonl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof/trace -o run -- python3 $BENCH > $OUT/prof/trace_bench.json 2> $OUT/prof/trace_bench.err || { echo TRACE_FAIL; tail -20 $OUT/prof/trace_bench.err; exit 1; }
timeout -k 10 60 rocprofv3 -L > $OUT/prof/counters_list.txt 2>&1 || echo LIST_FAIL
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $OUT/prof/pmc_sq -o run -- python3 $BENCH > $OUT/prof/pmc_sq.json 2> $OUT/prof/pmc_sq.err || { echo PMC_SQ_FAIL; tail -5 $OUT/prof/pmc_sq.err; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/prof/pmc_fetch -o run -- python3 $BENCH > $OUT/prof/pmc_fetch.json 2> $OUT/prof/pmc_fetch.err || { echo PMC_FETCH_FAIL; tail -5 $OUT/prof/pmc_fetch.err; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/prof/pmc_write -o run -- python3 $BENCH > $OUT/prof/pmc_write.json 2> $OUT/prof/pmc_write.err || { echo PMC_WRITE_FAIL; tail -5 $OUT/prof/pmc_write.err; }
find $OUT/prof -name "*.csv" | head -20
