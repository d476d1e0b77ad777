# Round 5: per-kernel device time of small (Janus-sized) SumVec jobs, one thread, direct path: which kernel
# holds the latency floor of a 100-report launch.
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT /tmp/jp
timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode direct --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --keep-pool /tmp/jp > $OUT/prep.log 2>&1 || { echo PREP_FAIL; exit 1; }
export TMPDIR=/tmp
for n in ${2:-10 100 1000}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/n$n -o run -- tools/bin/jobs_driver /tmp/jp/pool_2_2048.bin /tmp/jp/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f $n 1 1 0 0 1 > $OUT/n$n.json 2> $OUT/n$n.err || { echo PROF_FAIL $n; tail -5 $OUT/n$n.err; exit 1; }
  cat $OUT/n$n.json
done
echo LAT_OK
