# GPU suite + a short SumVec bench (small pool, no CPU leg): the kernel iteration loop
# usage: bash scripts/gpu_quick.sh <name>   (outputs under gpurun_out/<name>/)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|ERROR|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --pool 4096 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels'])"
