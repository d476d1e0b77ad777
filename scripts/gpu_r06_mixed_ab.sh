# Round 6: mixed-role coalescing (32 helper threads and 32 leader prepare_init threads of another task on ONE
# Prio3 instance, SumVec 8x1000/88, 100-report jobs) with 4 (default) and 6 lanes (JX_COAL_LANES): jobs per launch
# per role against each role alone.
# usage: bash scripts/gpu_r06_mixed_ab.sh <name> [lane counts]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
LANES=${2:-4,6}
OUT=gpurun_out/$N
mkdir -p $OUT
for L in ${LANES//,/ }; do
  JX_COAL_LANES=$L timeout -k 10 400 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 32,0 --leader-threads 0,32 --seconds 2 --pool 1024 --out $OUT/mixed_$L.jsonl > $OUT/mixed_$L.log 2>&1 || { echo MIXED_FAIL $L; tail -5 $OUT/mixed_$L.log; exit 1; }
  python3 -c "
import json
for l in open('$OUT/mixed_$L.jsonl'):
    d = json.loads(l); print('lanes=$L', d['threads'], d.get('leader_threads'), d.get('reports_per_s'), d.get('helper_jobs_per_launch'), d.get('leader_reports_per_s'), d.get('leader_jobs_per_launch'), d.get('verified'))
"
done
echo MIXED_OK
