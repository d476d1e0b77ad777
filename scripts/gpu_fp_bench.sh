set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_fixedpoint.py "$@" > gpurun_out/fp_bench.json 2> gpurun_out/fp_bench.err || { echo FP_BENCH_FAIL; tail -20 gpurun_out/fp_bench.err; exit 1; }
cat gpurun_out/fp_bench.json
