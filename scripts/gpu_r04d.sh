# Round 4 (d): GPU suite, the driver's bench, K3 probe (ring only), K3 group finish as its own kernel,
# configs[4] helper-priority experiment. Outputs under gpurun_out/r04d/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; grep -v rank0 $OUT/bench.err | tail -20; exit 1; }
tail -c 600 $OUT/bench.json
timeout -k 10 400 bash tools/k3_probe.sh $OUT/k3probe || { echo PROBE_FAIL; exit 1; }
JX_K3_SPLIT=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary --no-dist > $OUT/k3split.json 2> $OUT/k3split.err || { echo SPLIT_FAIL; tail -5 $OUT/k3split.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/k3split.json').read().strip().splitlines()[-1]); print('k3split', d['value'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'], d['verified'])"
timeout -k 10 500 bash scripts/gpu_fp_prio.sh r04d/fpprio || { echo FPPRIO_FAIL; exit 1; }
