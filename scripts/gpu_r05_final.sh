# Round 5, final tree: the GPU suite, the job-granularity matrix (coalesced and direct) and the driver's bench command.
# usage: bash scripts/gpu_r05_final.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/gpu_r05_jobs.sh $N || exit 1
