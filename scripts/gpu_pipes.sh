# Engine pipelines: the GPU pipes test, then the headline bench with 1 / 2 / 3 pipelines (default launch
# size: 262,144) and with 2 / 3 pipelines at one-round launches (131,072).
# usage: bash scripts/gpu_pipes.sh <name>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipes.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
for cfg in "1 0" "2 0" "3 0" "2 131072" "3 131072"; do
  set -- $cfg
  if [ "$2" = "0" ]; then
    JX_PIPES=$1 timeout -k 10 300 python -u bench.py $ARGS > $OUT/p$1_c$2.json 2> $OUT/p$1_c$2.err || { echo BENCH_FAIL $cfg; tail -5 $OUT/p$1_c$2.err; exit 1; }
  else
    JX_PIPES=$1 JX_CHUNK_REPORTS=$2 timeout -k 10 300 python -u bench.py $ARGS > $OUT/p$1_c$2.json 2> $OUT/p$1_c$2.err || { echo BENCH_FAIL $cfg; tail -5 $OUT/p$1_c$2.err; exit 1; }
  fi
  python3 -c "
import json,sys; d=json.loads(open('$OUT/p$1_c$2.json').read().strip().splitlines()[-1])
print('pipes=$1 chunk=$2', d['value'], d['ms_per_step'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['kernels']['reports_per_launch'], d['verified'])"
done
