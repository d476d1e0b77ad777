# K1 tail split: the K1 split-variant and FixedPoint GPU tests, then configs[4] (serial + two jobs in flight)
# with the engine's automatic helper K1 and with the lane-pair kernel forced (JX_K1_SPLIT=6).
# usage: bash scripts/gpu_k1split.sh <name>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fixedpoint.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
FP="tools/bench_fixedpoint.py --skip cpu,helper,leader --steps 3 --warmup 1"
timeout -k 10 400 python -u $FP > $OUT/fp_auto.json 2> $OUT/fp_auto.err || { echo FP_AUTO_FAIL; tail -20 $OUT/fp_auto.err; exit 1; }
JX_K1_SPLIT=6 timeout -k 10 400 python -u $FP > $OUT/fp_pairs.json 2> $OUT/fp_pairs.err || { echo FP_PAIRS_FAIL; tail -20 $OUT/fp_pairs.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for k in ("fp_auto", "fp_pairs"):
    d = json.loads(open(f"{o}/{k}.json").read().strip().splitlines()[-1])
    print(k, "serial", d["value"], d["kernels"], "two-jobs", d["pipelined"]["reports_per_s"], d["pipelined"]["kernels"], d["verified"], d["pipelined"]["verified"])
PY
