# Round 5: the mixed helper K1 launch (lane-split + lane pairs on two streams): parity, then configs[4] two jobs.
# usage: bash scripts/gpu_r05_mixed.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "mixed or k1_split" -x -v --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo PARITY_FAIL; tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 400 python -u tools/bench_fixedpoint.py --skip cpu,helper,leader --steps 3 --warmup 1 > $OUT/fp.json 2> $OUT/fp.err || { echo FP_FAIL; tail -5 $OUT/fp.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/fp.json').read().strip().splitlines()[-1])
print('serial', d['value'], d['kernels']); p=d['pipelined']; print('two jobs', p['reports_per_s'], p['ms_per_step'], p['kernels'], p['verified'], d['verified'])"
echo MIXED_OK
