# Round 6: the job-size matrix on the final tree (native driver, coalesced, 2 s per case, every job and the
# aggregate verified): SumVec 8x1000/88 and Count, 10 / 100 / 1,000 / 10,000-report jobs, 1 / 8 / 64 threads.
# usage: bash scripts/gpu_r06_matrix.sh <name>
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec,count --sizes 10,100,1000,10000 --threads 1,8,64 --seconds 2 --out $OUT/matrix.jsonl > $OUT/matrix.log 2>&1 || { echo MATRIX_FAIL; tail -5 $OUT/matrix.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/matrix.jsonl'):
    d = json.loads(l); print(d['vdaf'][:12], d['reports_per_job'], d['threads'], round(d['reports_per_s']), d['prep_ms_p50'], d['jobs_per_launch'], d['verified'])
"
echo MATRIX_OK
