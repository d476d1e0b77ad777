# K3 loader probes: load-only with the staging's call stride (22) vs one contiguous stream per
# workgroup (25), twice each, one 262,144-report launch.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k3stream
mkdir -p $OUT
ONE="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 4096 --no-cpu-baseline"
for v in 22 25 22 25; do
  JX_K3_PF=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$v -o run -- python3 $ONE > $OUT/one$v.json 2> $OUT/one$v.err || { echo TRACE_FAIL $v; tail -20 $OUT/one$v.err; exit 1; }
  grep -h "flp_psum_part" $OUT/trace$v/run_kernel_stats.csv | cut -c1-140
done
