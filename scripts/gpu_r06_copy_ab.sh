# Round 6: copy-kernel grid cap A/B (JX_COPY_WGS) at 64 threads, SumVec 100 / 1,000 / 10,000-report jobs and Count
# 10,000 (native driver, 2 s per case, every job verified).
# usage: bash scripts/gpu_r06_copy_ab.sh <name> [caps]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
CAPS=${2:-64,512}
OUT=gpurun_out/$N
mkdir -p $OUT
for W in ${CAPS//,/ }; do
  JX_COPY_WGS=$W timeout -k 10 400 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100,1000,10000 --threads 64,10 --seconds 2 --out $OUT/copy_$W.jsonl > $OUT/copy_$W.log 2>&1 || { echo COPY_FAIL $W; tail -5 $OUT/copy_$W.log; exit 1; }
  python3 -c "
import json
for l in open('$OUT/copy_$W.jsonl'):
    d = json.loads(l); print('wgs=$W', d['reports_per_job'], d['threads'], round(d['reports_per_s']), d['prep_ms_p50'], d['jobs_per_launch'], d.get('device_ms'), d['verified'])
"
done
echo COPY_OK
