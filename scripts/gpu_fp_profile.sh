# configs[4] profile: kernel-trace stats and separate PMC passes over one serial ping-pong step of 40,960
# FixedPoint 16 x 10000 reports (leader K1 + K3, helper K1 + K3), summarised by tools/prof_summary.py
# usage: bash scripts/gpu_fp_profile.sh <name>   (outputs under gpurun_out/<name>/)
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT/pmc
FP="tools/bench_fixedpoint.py --skip cpu,pipelined,helper,leader --steps 1 --warmup 0"
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/pmc/trace_raw -o run -- python3 $FP > $OUT/trace.json 2> $OUT/trace.err || { echo TRACE_FAIL; tail -20 $OUT/trace.err; exit 1; }
mkdir -p $OUT/pmc/trace && cp $OUT/pmc/trace_raw/run_kernel_stats.csv $OUT/pmc/trace/
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc/pmc_fetch -o run -- python3 $FP > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo PMC_FETCH_FAIL; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc/pmc_write -o run -- python3 $FP > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo PMC_WRITE_FAIL; tail -5 $OUT/pmc_write.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc/pmc_sq -o run -- python3 $FP > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || { echo PMC_SQ_FAIL; tail -5 $OUT/pmc_sq.err; exit 1; }
python3 tools/prof_summary.py $OUT/pmc --reports-per-launch 40960 --command "python3 $FP" > $OUT/${N}_pmc_summary.json && echo SUMMARY_OK
