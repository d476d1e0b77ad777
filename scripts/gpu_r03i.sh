# K3 stream without arithmetic (ring vs flat sweep) and the Keccak loop at steady-state clock
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 120 ./tools/bin/microbench_stream 262144 > $OUT/stream.jsonl 2> $OUT/stream.err || { echo STREAM_FAIL; tail -5 $OUT/stream.err; exit 1; }
cat $OUT/stream.jsonl
timeout -k 10 200 ./tools/bin/microbench_keccak 8000 > $OUT/keccak_long.jsonl 2> $OUT/keccak_long.err || { echo MB_FAIL; tail -5 $OUT/keccak_long.err; exit 1; }
cat $OUT/keccak_long.jsonl
