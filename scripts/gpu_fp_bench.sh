# configs[4] (FixedPoint 16 x 10000) bench; extra arguments go to tools/bench_fixedpoint.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_fixedpoint.py "$@" > gpurun_out/fp_bench.json 2> gpurun_out/fp_bench.err || { echo FP_BENCH_FAIL; tail -20 gpurun_out/fp_bench.err; exit 1; }
cat gpurun_out/fp_bench.json
