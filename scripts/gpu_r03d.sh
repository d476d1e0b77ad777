# configs[4]: pipelined two-role ping-pong at larger jobs (helper staging budget raised so a job is one launch)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 500 python -u tools/bench_fixedpoint.py --skip cpu,helper,leader,pingpong --reports 36864 --helper-staging-gb 106 > $OUT/fp_pipe36.json 2> $OUT/fp_pipe36.err || { echo FP36_FAIL; tail -20 $OUT/fp_pipe36.err; exit 1; }
cat $OUT/fp_pipe36.json
timeout -k 10 500 python -u tools/bench_fixedpoint.py --skip cpu,helper,leader,pingpong --reports 40960 --helper-staging-gb 118 > $OUT/fp_pipe40.json 2> $OUT/fp_pipe40.err || { echo FP40_FAIL; tail -20 $OUT/fp_pipe40.err; exit 1; }
cat $OUT/fp_pipe40.json
