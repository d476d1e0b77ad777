# Round 6: Janus job granularity on the final coalescer (native driver, SumVec 8x1000/88, 100-report jobs):
#  1. 64 and 10 threads, prepare-only and from HPKE-encrypted report shares (coalesced);
#  2. mixed roles: 32 helper threads alone, 32 leader threads alone, both together (jobs per launch per role);
#  3. kernel traces of 64 x 100 and 10 x 100 (device busy fraction, tools/trace_overlap.py).
# usage: bash scripts/gpu_r06_jobs.sh <name> [steps: matrix,mixed,trace]
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
STEPS=${2:-matrix,mixed,trace}
OUT=gpurun_out/$N
mkdir -p $OUT /tmp/jp
if [[ $STEPS == *matrix* ]]; then
  timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 64,10 --seconds 2 --out $OUT/plain.jsonl > $OUT/plain.log 2>&1 || { echo PLAIN_FAIL; tail -5 $OUT/plain.log; exit 1; }
  timeout -k 10 300 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 64,10 --seconds 2 --encrypted --pool 1024 --out $OUT/enc.jsonl > $OUT/enc.log 2>&1 || { echo ENC_FAIL; tail -5 $OUT/enc.log; exit 1; }
  python3 -c "
import json
for f in ('$OUT/plain.jsonl', '$OUT/enc.jsonl'):
    for l in open(f):
        d = json.loads(l); print(f.split('/')[-1], d['threads'], d['reports_per_s'], d['prep_ms_p50'], d['jobs_per_launch'], d.get('device_ms'), d.get('gather_ms'), d['verified'])
"
fi
if [[ $STEPS == *mixed* ]]; then
  timeout -k 10 400 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 100 --threads 32,0 --leader-threads 0,32 --seconds 2 --pool 1024 --out $OUT/mixed.jsonl > $OUT/mixed.log 2>&1 || { echo MIXED_FAIL; tail -5 $OUT/mixed.log; exit 1; }
  python3 -c "
import json
for l in open('$OUT/mixed.jsonl'):
    d = json.loads(l); print('mixed', d['threads'], d.get('leader_threads'), d.get('reports_per_s'), d.get('helper_jobs_per_launch'), d.get('leader_reports_per_s'), d.get('leader_jobs_per_launch'), d.get('verified'))
"
fi
if [[ $STEPS == *trace* ]]; then
  timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --keep-pool /tmp/jp > $OUT/prep.log 2>&1 || { echo PREP_FAIL; tail -5 $OUT/prep.log; exit 1; }
  for T in 64 10; do
    timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $OUT/trace_$T -o run -- tools/bin/jobs_driver /tmp/jp/pool_2_2048.bin /tmp/jp/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f 100 $T 1 1 0 1 > $OUT/driver_$T.json 2> $OUT/driver_$T.err || { echo TRACE_FAIL $T; tail -5 $OUT/driver_$T.err; exit 1; }
    f=$(ls $OUT/trace_$T/*/run_kernel_trace.csv $OUT/trace_$T/run_kernel_trace.csv 2>/dev/null | head -1)
    c=$(ls $OUT/trace_$T/*/run_memory_copy_trace.csv $OUT/trace_$T/run_memory_copy_trace.csv 2>/dev/null | head -1)
    python3 tools/launch_anatomy.py $f ${c:+--copies $c} > $OUT/anatomy_$T.json || true
    python3 tools/trace_overlap.py $f > $OUT/overlap_$T.json && python3 -c "import json; d=json.load(open('$OUT/overlap_$T.json')); print('trace', $T, round(d['device_busy_frac'],3), d['span_ms'])" && cat $OUT/driver_$T.json
  done
fi
if [[ $STEPS == *noacc* ]]; then
  [ -f /tmp/jp/pool_2_2048.bin ] || timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --keep-pool /tmp/jp > $OUT/prep.log 2>&1 || { echo PREP_FAIL; exit 1; }
  # accumulate per job deferred (default) / at once (JX_JOBS_DEFER=0) / not at all (batches released)
  for T in 64 10; do for A in 1 0 2; do
    D=1; ACC=$A; [ $A = 0 ] && D=0 && ACC=1; [ $A = 2 ] && ACC=0
    JX_JOBS_DEFER=$D timeout -k 10 60 tools/bin/jobs_driver /tmp/jp/pool_2_2048.bin /tmp/jp/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f 100 $T 2 1 0 1 $ACC > $OUT/acc_${T}_$A.json 2> $OUT/acc_${T}_$A.err || { echo ACC_FAIL; cat $OUT/acc_${T}_$A.err | tail -3; exit 1; }
    echo "acc_mode=$A(1 deferred,0 at once,2 none) T=$T $(cat $OUT/acc_${T}_$A.json)"
  done; done
fi
echo JOBS_OK
