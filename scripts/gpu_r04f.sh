# Round 4: the GPU suite, the driver's bench, the K3 ring-only probe and the K1 non-temporal-staging A/B.
# usage: bash scripts/gpu_r04f.sh <name>   (build the k3probe and nt variants first)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; grep -v rank0 $OUT/bench.err | tail -20; exit 1; }
tail -c 400 $OUT/bench.json
timeout -k 10 400 bash tools/k3_probe.sh $OUT/k3probe || { echo PROBE_FAIL; exit 1; }
timeout -k 10 600 bash tools/variant_ab.sh $OUT/nt nt || { echo AB_FAIL; exit 1; }
