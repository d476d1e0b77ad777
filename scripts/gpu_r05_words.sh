# Round 5: the word-per-lane small-launch K1 and the one-kernel small accumulate: parity first (a failure or
# fault ends the script), then the pairs-vs-words launch-size sweep (tools/kernel_probe sweep).
# usage: bash scripts/gpu_r05_words.sh <name> [pytest -k expression]
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
K=${2:-k1_split or accumulate or coalesce}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accumulate.py tests/test_gpu_coalesce.py -k "$K" -x -v --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { echo PARITY_FAIL; tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
timeout -k 10 120 tools/bin/kernel_probe sweep > $OUT/sweep.jsonl 2> $OUT/sweep.err || { echo SWEEP_FAIL; tail -5 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
echo WORDS_OK
