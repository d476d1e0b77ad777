# Round 5: kernel timeline of the coalesced job path (native driver, SumVec 8x1000/88, 100-report jobs, 64 threads).
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT /tmp/jp
timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --keep-pool /tmp/jp > $OUT/prep.log 2>&1 || { echo PREP_FAIL; tail -5 $OUT/prep.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- tools/bin/jobs_driver /tmp/jp/pool_2_2048.bin /tmp/jp/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f ${2:-100} ${3:-64} 1 1 0 1 > $OUT/driver.json 2> $OUT/driver.err || { echo TRACE_FAIL; tail -5 $OUT/driver.err; exit 1; }
f=$(ls $OUT/trace/*/run_kernel_trace.csv $OUT/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_overlap.py $f > $OUT/overlap.json && cat $OUT/driver.json && echo TRACE_OK
