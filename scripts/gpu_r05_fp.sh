# Round 5: configs[4] (FixedPointBoundedL2VecSum 16 x 10000) A/B of the helper lane-split K1 placement and the
# leader's padded input rows; ping-pong one job at a time and two jobs in flight, 40,960 reports per job.
# usage: bash scripts/gpu_r05_fp.sh <name> [variant flags...]
set -o pipefail
N=${1:?name}
shift
OUT=gpurun_out/$N
mkdir -p $OUT
FP="tools/bench_fixedpoint.py --skip helper,leader,cpu --steps 3 --warmup 1"
i=0
for V in "" "--lanes-cap 0" "--packed-lis" "--helper-k1 5"; do
  i=$((i+1))
  timeout -k 10 300 python -u $FP $V > $OUT/fp_$i.json 2> $OUT/fp_$i.err || { echo FP_FAIL $i; tail -5 $OUT/fp_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/fp_$i.json')); print('$V', d['pipelined']['reports_per_s'], d['pipelined']['kernels'], d['value'] if 'value' in d else d.get('pingpong', ''), d['verified'])"
done
echo FP_OK
