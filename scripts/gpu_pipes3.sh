# Pipelines, round 3: launch size sweep at 2 pipelines (1.25M reports per step: 6 / 4 / 3 equal launches
# against the default 4 x 262,144 + 201,424).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
for c in 0 208384 312512 416704 0; do
  if [ "$c" = "0" ]; then
    timeout -k 10 300 python -u bench.py $ARGS > $OUT/c$c.json 2> $OUT/c$c.err || { echo BENCH_FAIL $c; tail -5 $OUT/c$c.err; exit 1; }
  else
    JX_CHUNK_REPORTS=$c timeout -k 10 300 python -u bench.py $ARGS > $OUT/c$c.json 2> $OUT/c$c.err || { echo BENCH_FAIL $c; tail -5 $OUT/c$c.err; exit 1; }
  fi
  python3 -c "
import json; d=json.loads(open('$OUT/c$c.json').read().strip().splitlines()[-1])
print('chunk=$c', d['value'], d['ms_per_step'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['kernels']['reports_per_launch'], d['roofline']['kernel_concurrency'], d['verified'])"
done
