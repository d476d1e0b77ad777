# A/B of the main library against a measurement build lib/libjanus_prio3_<variant>.so on the headline
# bench (per-launch HIP-event times of K1 / K3 / K4, verification on).
# usage: bash tools/variant_ab.sh <outdir> <variant>   (build first: python -c "from janus_amd import build;
#        build.build(variant='<variant>', defines=('<MACRO>=1',))")
set -o pipefail
OUT=${1:?outdir}
VAR=${2:?variant}
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-dist"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/main.json 2> $OUT/main.err || { echo MAIN_FAIL; tail -5 $OUT/main.err; exit 1; }
JX_LIB_VARIANT=$VAR timeout -k 10 300 python -u bench.py $ARGS > $OUT/$VAR.json 2> $OUT/$VAR.err || { echo VAR_FAIL; tail -5 $OUT/$VAR.err; exit 1; }
timeout -k 10 300 python -u bench.py $ARGS > $OUT/main2.json 2> $OUT/main2.err || { echo MAIN2_FAIL; tail -5 $OUT/main2.err; exit 1; }
python3 - $OUT $VAR <<'PY'
import json, sys
o, var = sys.argv[1:]
for k in ("main", var, "main2"):
    d = json.loads(open(f"{o}/{k}.json").read().strip().splitlines()[-1])
    print(k, d["value"], d["kernels"]["k1_xof_ms_per_launch"], d["kernels"]["k3_flp_ms_per_launch"],
          d["kernels"]["k4_acc_ms_per_launch"], d["verified"])
PY
