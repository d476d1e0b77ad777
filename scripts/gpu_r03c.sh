# configs[4]: in-place vs staged leader, pipelined ping-pong (two jobs in flight, both roles on one GPU)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 500 python -u tools/bench_fixedpoint.py --skip cpu,helper --role-reports 32768 > $OUT/fp_inplace.json 2> $OUT/fp_inplace.err || { echo FP_FAIL; tail -20 $OUT/fp_inplace.err; exit 1; }
cat $OUT/fp_inplace.json
timeout -k 10 500 python -u tools/bench_fixedpoint.py --skip cpu,helper --reports 24576 --role-reports 32768 > $OUT/fp_inplace24.json 2> $OUT/fp_inplace24.err || { echo FP24_FAIL; tail -20 $OUT/fp_inplace24.err; exit 1; }
cat $OUT/fp_inplace24.json
timeout -k 10 500 python -u tools/bench_fixedpoint.py --skip cpu,helper --reports 24576 --role-reports 32768 --leader-staged > $OUT/fp_staged24.json 2> $OUT/fp_staged24.err || { echo FP2_FAIL; tail -20 $OUT/fp_staged24.err; exit 1; }
cat $OUT/fp_staged24.json
