# BASELINE configs 0-2 with the C++ CPU engine baseline (1 thread and the box's thread budget)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
