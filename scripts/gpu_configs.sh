# Other BASELINE configs (Count, Sum32, Histogram) + the round bench with kernel-trace stats.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
bash scripts/gpu_bench_round.sh
