# Why the lane-pair K1 does not beat the lane-split K1 at 32,768 FixedPoint reports: issue / wait /
# instruction-cache counters per kernel (one PMC pass each, counters within the per-block limits)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03g
mkdir -p $OUT
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -i -E "SQC_|ICACHE|INST_LEVEL|SQ_IFETCH" $OUT/avail.txt | head -40 > $OUT/avail_ic.txt || true
ONE="tools/bench_fixedpoint.py --skip pingpong,pipelined,leader,cpu --role-reports 32768 --steps 1 --warmup 0"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in 3 6; do
  JX_K1_SPLIT=$v timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/sq$v -o run -- python3 $ONE > $OUT/sq$v.json 2> $OUT/sq$v.err || { echo PMC_FAIL $v; tail -5 $OUT/sq$v.err; exit 1; }
done
IC=$(grep -o -E "SQC_ICACHE_[A-Z_]+|SQ_IFETCH[A-Z_]*" $OUT/avail.txt | sort -u | head -4 | tr '\n' ' ')
echo "IC counters: $IC"
if [ -n "$IC" ]; then
  for v in 3 6; do
    JX_K1_SPLIT=$v timeout -s KILL 200 rocprofv3 --pmc $IC -f csv -d $OUT/ic$v -o run -- python3 $ONE > $OUT/ic$v.json 2> $OUT/ic$v.err || { echo IC_FAIL $v; tail -5 $OUT/ic$v.err; exit 1; }
  done
fi
echo DONE
