# PMC passes of the multiproof bench (tools/bench_mp.py): kernel trace + SQ counters, one pass each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_mp
mkdir -p $OUT
B="tools/bench_mp.py --steps 1 --warmup 0 --reports 262144 --pool 256"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.json 2> $OUT/trace.err || { echo TRACE_FAIL; tail -5 $OUT/trace.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -f csv -d $OUT/pmc1 -o run -- python3 $B > $OUT/pmc1.json 2> $OUT/pmc1.err || { echo PMC1_FAIL; tail -5 $OUT/pmc1.err; }
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -f csv -d $OUT/pmc2 -o run -- python3 $B > $OUT/pmc2.json 2> $OUT/pmc2.err || { echo PMC2_FAIL; tail -5 $OUT/pmc2.err; }
echo DONE
