# Round 6: group merging A/B (JX_COAL_MERGE=0 off, 1 on = the default) at 64 and 10 threads, plain and HPKE-sealed 100-report SumVec jobs
# (tools/bench_jobs.py: every job and the aggregate verified), 2 s per case.
# usage: bash scripts/gpu_r06_merge_ab.sh <name>
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
for M in 0 1; do
  JX_COAL_MERGE=$M timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 64,10 --seconds 2 --out $OUT/plain_$M.jsonl > $OUT/plain_$M.log 2>&1 || { echo PLAIN_FAIL $M; tail -5 $OUT/plain_$M.log; exit 1; }
  JX_COAL_MERGE=$M timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 64,10 --seconds 2 --encrypted --pool 1024 --out $OUT/enc_$M.jsonl > $OUT/enc_$M.log 2>&1 || { echo ENC_FAIL $M; tail -5 $OUT/enc_$M.log; exit 1; }
  python3 -c "
import json
for f in ('$OUT/plain_$M.jsonl', '$OUT/enc_$M.jsonl'):
    for l in open(f):
        d = json.loads(l); print('merge=$M', f.split('/')[-1], d['threads'], d['reports_per_s'], d['prep_ms_p50'], d['jobs_per_launch'], d.get('device_ms'), d.get('gather_ms'), d['verified'])
"
done
echo MERGE_OK
