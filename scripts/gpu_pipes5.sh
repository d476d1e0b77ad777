# Small VDAFs at 1M reports: four whole-round launches over two pipelines (default now) against one
# stream (JX_PIPES=1, one launch), alternating; then the pipes test.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipes.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
CF="tools/bench_configs.py --only sum32,hist --cpu-seconds 0.5 --steps 5"
for v in 0 1 0 1; do
  JX_PIPES=$v timeout -k 10 300 python -u $CF > $OUT/p$v.jsonl 2> $OUT/p$v.err || { echo CFG_FAIL; tail -5 $OUT/p$v.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/p$v.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('pipes=$v', d['config']['workload'][:24], d['value'], d['kernels']['launches_per_step'], d['verified'])"
done
