# Pipelines with a low-priority K1 stream per pipeline (JX_PIPE_PRIO=1): the pipes test, then the bench
# against the default pipelines, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
JX_PIPE_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_pipes.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
for v in 0 1 0 1; do
  JX_PIPE_PRIO=$v timeout -k 10 300 python -u bench.py $ARGS > $OUT/prio$v.json 2> $OUT/prio$v.err || { echo BENCH_FAIL $v; tail -5 $OUT/prio$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/prio$v.json').read().strip().splitlines()[-1])
print('prio=$v', d['value'], d['ms_per_step'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['kernels']['k4_acc_ms_per_launch'], d['roofline']['kernel_concurrency'], d['verified'])"
done
