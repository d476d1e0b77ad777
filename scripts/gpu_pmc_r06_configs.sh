# Round 6: PMC passes for configs[1] (Prio3Sum bits=32, 1M reports) and configs[2] (Prio3Histogram 256/16, 1M):
# a kernel trace and separate --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ) over tools/bench_configs.py steps of each
# config -> <name>_sum32_pmc_summary.json, <name>_hist_pmc_summary.json (bench.py CONFIG_PMC_SUMMARIES).
# usage: bash scripts/gpu_pmc_r06_configs.sh <name> [sum32,hist]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
CFGS=${2:-sum32,hist}
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
for C in ${CFGS//,/ }; do
  OUT=gpurun_out/$N/$C
  mkdir -p $OUT/pmc
  CMD="tools/bench_configs.py --only $C --steps 3 --warmup 1 --cpu-seconds 0.2"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/pmc/trace_raw -o run -- python3 $CMD > $OUT/trace.json 2> $OUT/trace.err || { echo TRACE_FAIL $C; tail -20 $OUT/trace.err; exit 1; }
  mkdir -p $OUT/pmc/trace && cp $OUT/pmc/trace_raw/run_kernel_stats.csv $OUT/pmc/trace/
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc/pmc_fetch -o run -- python3 $CMD > $OUT/fetch.json 2> $OUT/fetch.err || { echo FETCH_FAIL $C; tail -5 $OUT/fetch.err; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc/pmc_write -o run -- python3 $CMD > $OUT/write.json 2> $OUT/write.err || { echo WRITE_FAIL $C; tail -5 $OUT/write.err; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc/pmc_sq -o run -- python3 $CMD > $OUT/sq.json 2> $OUT/sq.err || { echo SQ_FAIL $C; tail -5 $OUT/sq.err; exit 1; }
  RPL=$(python3 -c "import json; print(json.loads(open('$OUT/trace.json').read().strip().splitlines()[-1])['kernels']['reports_per_launch'])")
  python3 tools/prof_summary.py $OUT/pmc --reports-per-launch $RPL --command "python3 $CMD ($RPL reports per launch)" > gpurun_out/$N/${N}_${C}_pmc_summary.json && echo SUMMARY_OK $C
done
