# K3 LDS-DMA ring variants (k3_pf 20 / 21) and the lane-split helper K1 on FixedPoint: parity, one-launch
# kernel traces, FixedPoint helper bench with the fused and the lane-split K1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k3glds
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "k3_pipeline or k1_split" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
for v in 1 20 21; do
  JX_K3_PF=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$v -o run -- python3 $ONE > $OUT/one$v.json 2> $OUT/one$v.err || { echo TRACE_FAIL $v; tail -20 $OUT/one$v.err; exit 1; }
  grep -h "flp_psum_part" $OUT/trace$v/run_kernel_stats.csv | cut -c1-140
done
for v in 0 3; do
  JX_K1_SPLIT=$v timeout -k 10 400 python -u tools/bench_fixedpoint.py --reports 24576 > $OUT/fp$v.json 2> $OUT/fp$v.err || { echo FP_FAIL $v; tail -20 $OUT/fp$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/fp$v.json'));print('fp k1split=$v', d['value'], d['helper_reports_per_s'], d['kernels'], d['verified'])"
done
