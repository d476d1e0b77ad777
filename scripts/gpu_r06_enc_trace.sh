# Round 6: kernel trace of HPKE-sealed 100-report SumVec jobs (native driver, 64 and 10 threads): the open's share of
# a coalesced launch (tools/launch_anatomy.py, kernel stats).
# usage: bash scripts/gpu_r06_enc_trace.sh <name>
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT /tmp/jpe
timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --encrypted --pool 1024 --keep-pool /tmp/jpe > $OUT/prep.log 2>&1 || { echo PREP_FAIL; tail -5 $OUT/prep.log; exit 1; }
P=$(ls /tmp/jpe/pool_2_1024_enc.bin)
for T in 64 10; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$T -o run -- tools/bin/jobs_driver $P /tmp/jpe/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f 100 $T 1 1 0 1 > $OUT/driver_$T.json 2> $OUT/driver_$T.err || { echo TRACE_FAIL $T; tail -5 $OUT/driver_$T.err; exit 1; }
  f=$(ls $OUT/trace_$T/*/run_kernel_trace.csv $OUT/trace_$T/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/launch_anatomy.py $f > $OUT/anatomy_$T.json || true
  grep -i "hpke\|xof_pairs\|xof_words" $OUT/trace_$T/run_kernel_stats.csv | cut -c1-200
  cat $OUT/driver_$T.json
done
echo ENC_TRACE_OK
