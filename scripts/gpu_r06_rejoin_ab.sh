# Round 6: adaptive rejoin window A/B (JX_COAL_REJOIN_FRAC percent of the role's launch latency, 0 = the fixed 1 ms):
# mixed roles (32 helper + 32 leader threads) and helper-only 64 / 10 threads, 100-report SumVec jobs.
# usage: bash scripts/gpu_r06_rejoin_ab.sh <name> [fractions]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
FR=${2:-0,30}
OUT=gpurun_out/$N
mkdir -p $OUT
for F in ${FR//,/ }; do
  JX_COAL_REJOIN_FRAC=$F timeout -k 10 400 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 32 --leader-threads 32 --seconds 2 --pool 1024 --out $OUT/mixed_$F.jsonl > $OUT/mixed_$F.log 2>&1 || { echo MIXED_FAIL $F; tail -5 $OUT/mixed_$F.log; exit 1; }
  JX_COAL_REJOIN_FRAC=$F timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 64,10 --seconds 2 --out $OUT/plain_$F.jsonl > $OUT/plain_$F.log 2>&1 || { echo PLAIN_FAIL $F; tail -5 $OUT/plain_$F.log; exit 1; }
  python3 -c "
import json
for f in ('$OUT/mixed_$F.jsonl', '$OUT/plain_$F.jsonl'):
    for l in open(f):
        d = json.loads(l); print('frac=$F', f.split('/')[-1], d['threads'], d.get('leader_threads'), d.get('reports_per_s'), d.get('helper_jobs_per_launch'), d.get('leader_reports_per_s'), d.get('leader_jobs_per_launch'), d.get('verified'))
"
done
echo REJOIN_OK
