# GPU session: the given pytest selection (default: the whole -m gpu suite) under a time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -60
tail -40 gpurun_out/pytest_gpu.log | grep -v PASSED
exit $rc
