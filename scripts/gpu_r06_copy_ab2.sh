set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06cp2
mkdir -p $OUT
for W in 64 16 64 16; do
  JX_COPY_WGS=$W timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 1000 --threads 64 --seconds 3 --out $OUT/c_$W.jsonl > $OUT/c_$W.log 2>&1 || { echo FAIL; exit 1; }
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/c_*.jsonl')):
    for l in open(f):
        d=json.loads(l); print(f, d['reports_per_job'], d['threads'], round(d['reports_per_s']), d['prep_ms_p50'], d['jobs_per_launch'], d.get('device_ms'), d['verified'])
"
