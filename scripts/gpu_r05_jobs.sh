# Round 5: job-granularity throughput/latency (native driver), coalesced vs direct, then the driver's bench command.
# usage: bash scripts/gpu_r05_jobs.sh <name>
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec,count --sizes 10,100,1000,10000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_coalesce_cpp.jsonl > $OUT/jobs_c.log 2>&1 || { echo JOBS_C_FAIL; tail -5 $OUT/jobs_c.log; exit 1; }
timeout -k 10 400 python -u tools/bench_jobs.py --driver cpp --mode direct --vdafs sumvec,count --sizes 10,100,1000,10000 --threads 1,8,64 --seconds 2 --out $OUT/jobs_direct_cpp.jsonl > $OUT/jobs_d.log 2>&1 || { echo JOBS_D_FAIL; tail -5 $OUT/jobs_d.log; exit 1; }
[ "$2" = "jobs" ] && exit 0
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
echo ALL_OK
