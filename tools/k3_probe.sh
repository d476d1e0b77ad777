# K3 with and without its per-group finish (measurement build JX_K3_PROBE=1: the ring loop only; results
# are wrong by design, verification off). Per-launch HIP-event times of K1 / K3 / K4 for both.
# usage: bash tools/k3_probe.sh <outdir>     (build first: python -c "from janus_amd import build;
#        build.build(variant='k3probe', defines=('JX_K3_PROBE=1',))")
set -o pipefail
OUT=${1:?outdir}
mkdir -p $OUT
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-secondary --no-dist"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/full.json 2> $OUT/full.err || { echo FULL_FAIL; tail -5 $OUT/full.err; exit 1; }
JX_LIB_VARIANT=k3probe timeout -k 10 300 python -u bench.py $ARGS > $OUT/probe.json 2> $OUT/probe.err || { echo PROBE_FAIL; tail -5 $OUT/probe.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for k in ("full", "probe"):
    d = json.loads(open(f"{o}/{k}.json").read().strip().splitlines()[-1])
    print(k, d["value"], d["kernels"]["k1_xof_ms_per_launch"], d["kernels"]["k3_flp_ms_per_launch"],
          d["kernels"]["k4_acc_ms_per_launch"], d["verified"])
PY
