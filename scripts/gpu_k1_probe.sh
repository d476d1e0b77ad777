# K1 issue-efficiency probe: kernel-trace stats + SQ counters of the fused K1 and of the split
# (squeeze-only at 4 waves/SIMD + absorb-only) variant over one 262,144-report launch.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k1probe
mkdir -p $OUT
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
for v in 0 1; do
  JX_K1_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$v -o run -- python3 $ONE > $OUT/one$v.json 2> $OUT/one$v.err || { echo TRACE_FAIL $v; tail -20 $OUT/one$v.err; exit 1; }
  JX_K1_SPLIT=$v timeout -s KILL 150 rocprofv3 --pmc $SQ -f csv -d $OUT/sq$v -o run -- python3 $ONE > $OUT/sq$v.json 2> $OUT/sq$v.err || { echo PMC_FAIL $v; tail -5 $OUT/sq$v.err; exit 1; }
  echo DONE $v
done
