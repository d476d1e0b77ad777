# Round 5: K1's clock attribution: K1 as built, with its staging stores replaced by a register sink,
# and with no per-block emission; K3 with and without its group finish. HIP events, then PMC passes (each its own
# rocprofv3 run) for clock and VALU utilisation of every variant.
# usage: bash scripts/gpu_r05_probe.sh <name>
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N/probe
mkdir -p $OUT
P="tools/bin/kernel_probe 262144 5"
timeout -k 10 120 $P > $OUT/events.json 2> $OUT/events.err || { echo PROBE_FAIL; tail -5 $OUT/events.err; exit 1; }
cat $OUT/events.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_raw -o run -- $P > $OUT/trace.json 2> $OUT/trace.err || { echo TRACE_FAIL; tail -5 $OUT/trace.err; exit 1; }
mkdir -p $OUT/trace && cp $OUT/trace_raw/run_kernel_stats.csv $OUT/trace/
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc_sq -o run -- $P > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || { echo PMC_SQ_FAIL; tail -5 $OUT/pmc_sq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- $P > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo PMC_FETCH_FAIL; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- $P > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo PMC_WRITE_FAIL; tail -5 $OUT/pmc_write.err; exit 1; }
python3 tools/prof_summary.py $OUT --reports-per-launch 262144 --command "$P" > $OUT/../k1_probe_summary.json && echo PROBE_OK
