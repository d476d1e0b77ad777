# K3 ring with 8 slot groups per workgroup (26) vs 4 (21): parity + one-launch traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k3w8
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "k3_pipeline" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
for v in 21 26 21 26; do
  JX_K3_PF=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$v -o run -- python3 $ONE > $OUT/one$v.json 2> $OUT/one$v.err || { echo TRACE_FAIL $v; tail -20 $OUT/one$v.err; exit 1; }
  grep -h "flp_psum_part" $OUT/trace$v/run_kernel_stats.csv | cut -c1-140
done
