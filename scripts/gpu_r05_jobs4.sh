# Round 5: coalescer tests and the 10..1,000-report job matrix (coalesced) on the current tree.
# usage: bash scripts/gpu_r05_jobs4.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_coalesce.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec,count --sizes 10,100,1000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_coalesce_cpp.jsonl > $OUT/jobs_c.log 2>&1 || { echo JOBS_C_FAIL; tail -5 $OUT/jobs_c.log; exit 1; }
echo JOBS4_OK
