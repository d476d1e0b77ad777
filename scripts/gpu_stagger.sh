# Pipelines: pipeline 1 starting with a half launch (JX_PIPE_STAGGER=1) against the default, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
for v in 0 1 0 1; do
  JX_PIPE_STAGGER=$v timeout -k 10 300 python -u bench.py $ARGS > $OUT/s$v.json 2> $OUT/s$v.err || { echo BENCH_FAIL $v; tail -5 $OUT/s$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/s$v.json').read().strip().splitlines()[-1])
print('stagger=$v', d['value'], d['ms_per_step'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['roofline']['kernel_concurrency'], d['verified'])"
done
