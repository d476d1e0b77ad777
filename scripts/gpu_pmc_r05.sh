# Round-5 PMC passes on the final sources (each pass its own rocprofv3 run):
#  * SumVec: the bench step on ONE stream (the same launches as roofline.alone: 4 x 262,144 + 201,424 reports),
#    one warm-up step + 3 steps -> <name>_pmc_summary.json (bench.py's PMC_SUMMARY: K1 instructions per report,
#    clock, traffic) and the kernel-trace stats of the same command;
#  * configs[4]: one serial step of 40,960 FixedPoint 16 x 10000 reports (leader rows padded to 128 B)
#    -> <name>_fixedpoint_pmc_summary.json.
# usage: bash scripts/gpu_pmc_r05.sh <name> [sumvec]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT/pmc $OUT/fp/pmc
ONE="bench.py --steps 3 --warmup 1 --pipes 1 --pool 4096 --no-cpu-baseline --no-secondary --no-dist"
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/pmc/trace_raw -o run -- python3 $ONE > $OUT/one.json 2> $OUT/one.err || { echo ONE_TRACE_FAIL; tail -20 $OUT/one.err; exit 1; }
mkdir -p $OUT/pmc/trace && cp $OUT/pmc/trace_raw/run_kernel_stats.csv $OUT/pmc/trace/
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc/pmc_fetch -o run -- python3 $ONE > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo PMC_FETCH_FAIL; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc/pmc_write -o run -- python3 $ONE > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo PMC_WRITE_FAIL; tail -5 $OUT/pmc_write.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc/pmc_sq -o run -- python3 $ONE > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || { echo PMC_SQ_FAIL; tail -5 $OUT/pmc_sq.err; exit 1; }
python3 tools/prof_summary.py $OUT/pmc --reports-per-launch 250000 --command "python3 $ONE (4 x 262,144 + 201,424-report launches per step; per-launch averages over 20 launches)" > $OUT/${N}_pmc_summary.json && echo SUMMARY_OK
[ "$2" = "sumvec" ] && exit 0
FP="tools/bench_fixedpoint.py --skip cpu,pipelined,helper,leader --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/fp/pmc/trace_raw -o run -- python3 $FP > $OUT/fp/trace.json 2> $OUT/fp/trace.err || { echo FP_TRACE_FAIL; tail -20 $OUT/fp/trace.err; exit 1; }
mkdir -p $OUT/fp/pmc/trace && cp $OUT/fp/pmc/trace_raw/run_kernel_stats.csv $OUT/fp/pmc/trace/
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fp/pmc/pmc_fetch -o run -- python3 $FP > $OUT/fp/pmc_fetch.json 2> $OUT/fp/pmc_fetch.err || { echo FP_FETCH_FAIL; tail -5 $OUT/fp/pmc_fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/fp/pmc/pmc_write -o run -- python3 $FP > $OUT/fp/pmc_write.json 2> $OUT/fp/pmc_write.err || { echo FP_WRITE_FAIL; tail -5 $OUT/fp/pmc_write.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/fp/pmc/pmc_sq -o run -- python3 $FP > $OUT/fp/pmc_sq.json 2> $OUT/fp/pmc_sq.err || { echo FP_SQ_FAIL; tail -5 $OUT/fp/pmc_sq.err; exit 1; }
python3 tools/prof_summary.py $OUT/fp/pmc --reports-per-launch 40960 --command "python3 $FP" > $OUT/${N}_fixedpoint_pmc_summary.json && echo FP_SUMMARY_OK
