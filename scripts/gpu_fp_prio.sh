# configs[4] two-jobs shape with and without issue priority for the helper's sponge waves (measurement
# build JX_HELPER_PRIO=2), after the leader K3 fix. usage: bash scripts/gpu_fp_prio.sh <name>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
FP="tools/bench_fixedpoint.py --skip cpu,helper,leader --steps 3 --warmup 1"
timeout -k 10 400 python -u $FP > $OUT/fp_base.json 2> $OUT/fp_base.err || { echo BASE_FAIL; tail -5 $OUT/fp_base.err; exit 1; }
JX_LIB_VARIANT=hprio timeout -k 10 400 python -u $FP > $OUT/fp_prio.json 2> $OUT/fp_prio.err || { echo PRIO_FAIL; tail -5 $OUT/fp_prio.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for k in ("base", "prio"):
    d = json.loads(open(f"{o}/fp_{k}.json").read().strip().splitlines()[-1])
    print(k, "serial", d["value"], d["kernels"], "two-jobs", d["pipelined"]["reports_per_s"], d["pipelined"]["kernels"],
          d["verified"])
PY
