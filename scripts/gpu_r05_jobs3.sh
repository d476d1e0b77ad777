# Round 5: arena / coalescer tests, the job matrix (SumVec + Count, 10..1,000 reports x 1, 8, 64 threads, coalesced and
# direct) on the current tree, and configs[4] with the lane-pair helper K1 forced (A/B against the lane-split default).
# usage: bash scripts/gpu_r05_jobs3.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_coalesce.py tests/test_gpu_accumulate.py tests/test_gpu_pipes.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec,count --sizes 10,100,1000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_coalesce_cpp.jsonl > $OUT/jobs_c.log 2>&1 || { echo JOBS_C_FAIL; tail -5 $OUT/jobs_c.log; exit 1; }
timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode direct --vdafs sumvec,count --sizes 10,100,1000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_direct_cpp.jsonl > $OUT/jobs_d.log 2>&1 || { echo JOBS_D_FAIL; tail -5 $OUT/jobs_d.log; exit 1; }
timeout -k 10 400 python -u tools/bench_fixedpoint.py --skip cpu,helper,leader --steps 3 --warmup 1 --helper-k1 6 > $OUT/fp_pairs.json 2> $OUT/fp_pairs.err || { echo FP_FAIL; tail -5 $OUT/fp_pairs.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/fp_pairs.json').read().strip().splitlines()[-1])
print('serial', d['value'], d['kernels']['helper']); p=d['pipelined']; print('two jobs', p['reports_per_s'], p['ms_per_step'], p['kernels'], p['verified'], d['verified'])"
echo JOBS3_OK
