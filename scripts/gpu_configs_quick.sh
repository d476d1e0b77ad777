# GPU tests, then the other BASELINE configs and the headline bench (no profiler).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/q
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'): d=json.loads(l); print(d['config']['workload'], d['value'], d['verified'], d['kernels'])
d=json.load(open('$OUT/bench.json')); print('SUMVEC', d['value'], d['verified'], d['kernels']['k4_acc_ms_per_launch'])
"
