# Round-end measurement on the current sources: the whole GPU suite; PMC passes over uniform 262,144-report
# launches (-> profiles/<name>_pmc_summary.json, which bench.py's roofline reads for `traffic`); the default
# bench with the CPU baseline and its rocprofv3 kernel stats; configs 0-2; configs[4] with its kernel trace.
# usage: bash scripts/gpu_round.sh <name>   (outputs under gpurun_out/<name>/)
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/pmc/trace_raw -o run -- python3 $ONE > $OUT/one.json 2> $OUT/one.err || { echo ONE_TRACE_FAIL; tail -20 $OUT/one.err; exit 1; }
mkdir -p $OUT/pmc/trace && cp $OUT/pmc/trace_raw/run_kernel_stats.csv $OUT/pmc/trace/
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc/pmc_fetch -o run -- python3 $ONE > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo PMC_FETCH_FAIL; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc/pmc_write -o run -- python3 $ONE > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo PMC_WRITE_FAIL; tail -5 $OUT/pmc_write.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc/pmc_sq -o run -- python3 $ONE > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || { echo PMC_SQ_FAIL; tail -5 $OUT/pmc_sq.err; exit 1; }
python3 tools/prof_summary.py $OUT/pmc --reports-per-launch 262144 --command "python3 $ONE" > $OUT/${N}_pmc_summary.json && echo SUMMARY_OK
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo TRACE_FAIL; tail -20 $OUT/trace_bench.err; exit 1; }
echo TRACE_OK
timeout -k 10 400 python -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
echo CONFIGS_OK
timeout -k 10 600 python -u tools/bench_fixedpoint.py > $OUT/fp.json 2> $OUT/fp.err || { echo FP_FAIL; tail -20 $OUT/fp.err; exit 1; }
echo FP_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/fp_trace -o run -- python3 tools/bench_fixedpoint.py --skip cpu,pipelined,helper,leader --steps 1 --warmup 1 > $OUT/fp_trace.json 2> $OUT/fp_trace.err || { echo FP_TRACE_FAIL; tail -5 $OUT/fp_trace.err; exit 1; }
echo FP_TRACE_OK
