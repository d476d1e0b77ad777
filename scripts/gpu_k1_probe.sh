# K1 issue-efficiency probe: parity of the K1 variants, then kernel-trace stats + SQ counters of the
# fused K1 (0), the split launches (1: squeeze-only at 4 waves/SIMD + absorb-only), the lane-split
# kernel (3) and the sequential-permutation fused kernel (4) over one 262,144-report launch.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k1probe
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k1_split" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
SQ="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-0 1 3 4}; do
  JX_K1_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$v -o run -- python3 $ONE > $OUT/one$v.json 2> $OUT/one$v.err || { echo TRACE_FAIL $v; tail -20 $OUT/one$v.err; exit 1; }
  JX_K1_SPLIT=$v timeout -s KILL 150 rocprofv3 --pmc $SQ -f csv -d $OUT/sq$v -o run -- python3 $ONE > $OUT/sq$v.json 2> $OUT/sq$v.err || { echo PMC_FAIL $v; tail -5 $OUT/sq$v.err; exit 1; }
  echo DONE $v
done
