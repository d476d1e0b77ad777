# Lean leader K1: leader / FixedPoint / ping-pong parity, FixedPoint bench; K3 timing probes
# (22: loads + barriers only, 23: limb products only) against the default ring (21).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/lk3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_leader.py tests/test_gpu_fixedpoint.py tests/test_gpu_accumulate.py tests/test_gpu_multiproof.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u tools/bench_fixedpoint.py --reports 24576 > $OUT/fp.json 2> $OUT/fp.err || { echo FP_FAIL; tail -20 $OUT/fp.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/fp.json'));print('fp', d['value'], d['helper_reports_per_s'], d['kernels'], d['verified'])"
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
for v in 21 22 23; do
  JX_K3_PF=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$v -o run -- python3 $ONE > $OUT/one$v.json 2> $OUT/one$v.err || { echo TRACE_FAIL $v; tail -20 $OUT/one$v.err; exit 1; }
  grep -h "flp_psum_part" $OUT/trace$v/run_kernel_stats.csv | cut -c1-140
done
