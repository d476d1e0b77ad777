set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/stream2
mkdir -p $OUT
timeout -k 10 200 ./tools/bin/microbench_stream 262144 > $OUT/stream.jsonl 2> $OUT/stream.err || { echo STREAM_FAIL; tail -5 $OUT/stream.err; exit 1; }
cat $OUT/stream.jsonl
