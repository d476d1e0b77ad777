# Round 6: coalescer A/B at Janus's job size (native driver, SumVec 8x1000/88, 100-report jobs, 2 s per case):
# hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) x launches of a role in flight before a gather
# waits (JX_COAL_MAX_RUNNING, default 2), at 64 and 10 threads.
# usage: bash scripts/gpu_r06_ab.sh <name> [hwq list] [max-running list]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
HWQS=${2:-4,8}
MRS=${3:-2,3}
OUT=gpurun_out/$N
mkdir -p $OUT /tmp/jp
timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --keep-pool /tmp/jp > $OUT/prep.log 2>&1 || { echo PREP_FAIL; tail -5 $OUT/prep.log; exit 1; }
for Q in ${HWQS//,/ }; do for M in ${MRS//,/ }; do for T in 64 10; do
  GPU_MAX_HW_QUEUES=$Q JX_COAL_MAX_RUNNING=$M timeout -k 10 60 tools/bin/jobs_driver /tmp/jp/pool_2_2048.bin /tmp/jp/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f 100 $T 2 1 0 1 > $OUT/ab_${Q}_${M}_$T.json 2> $OUT/ab_${Q}_${M}_$T.err || { echo AB_FAIL $Q $M $T; tail -3 $OUT/ab_${Q}_${M}_$T.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_${Q}_${M}_$T.json'))
print('hwq=$Q maxrun=$M T=$T', d['reports_per_s'], 'p50', d['prep_ms_p50'], 'jpl', d['jobs_per_launch'], 'gather', d['gather_ms'], 'dev', d['device_ms'])"
done; done; done
echo AB_OK
