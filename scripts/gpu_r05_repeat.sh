# Round 5: headline repeatability on one box (the driver's bench command without the secondary legs), three runs.
# usage: bash scripts/gpu_r05_repeat.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { echo BENCH_FAIL $k; tail -5 $OUT/bench_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$k.json').read().strip().splitlines()[-1]); print($k, d['value'], d['verified'], d['roofline']['frac'], d['roofline']['frac_pmc_run'])"
done
echo REPEAT_OK
