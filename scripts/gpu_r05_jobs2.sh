# Round 5: GPU suite, then the SumVec job-granularity matrix (native driver, coalesced and direct) on the current tree.
# usage: bash scripts/gpu_r05_jobs2.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec,count --sizes 10,100,1000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_coalesce_cpp.jsonl > $OUT/jobs_c.log 2>&1 || { echo JOBS_C_FAIL; tail -5 $OUT/jobs_c.log; exit 1; }
timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode direct --vdafs sumvec,count --sizes 10,100,1000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_direct_cpp.jsonl > $OUT/jobs_d.log 2>&1 || { echo JOBS_D_FAIL; tail -5 $OUT/jobs_d.log; exit 1; }
echo JOBS2_OK
