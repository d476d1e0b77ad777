# Round 6: GPU tests (a failure or fault ends the script). usage: bash scripts/gpu_r06_tests.sh <name> <test files / -k ...>
set -o pipefail
N=${1:?name}
shift
OUT=gpurun_out/$N
mkdir -p $OUT
X=-x; [ -n "$NOX" ] && X=
timeout -k 10 1000 python -u -m pytest "$@" $X -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -60
exit $rc
