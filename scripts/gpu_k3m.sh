# MFMA K3: lane-map probe, GPU suite, short bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k3m}
mkdir -p $OUT
timeout -k 10 60 ./tools/bin/mfma_i8_probe > $OUT/probe.txt 2>&1; cat $OUT/probe.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|ERROR|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --pool 4096 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels'])"
