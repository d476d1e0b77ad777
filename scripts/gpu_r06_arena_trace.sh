# Round 6: kernel trace of two engines under a small arena budget (tests/arena_trim_worker.py, JX_ARENA_GB=6:
# the arena keeps trimming one engine's idle staging for the other's check-outs) -> per-stream gaps
# (tools/stream_gaps.py): no gap on one engine's stream should come from the other engine's trim.
# usage: bash scripts/gpu_r06_arena_trace.sh <name>
set -o pipefail
export TMPDIR=/tmp
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT
rm -f /tmp/jx_trims.log; JX_ARENA_TRIM_LOG=/tmp/jx_trims.log JX_ARENA_GB=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/arena_trace -o run -- python3 -u tests/arena_trim_worker.py > $OUT/arena_worker.json 2> $OUT/arena_worker.err || { echo ARENA_TRACE_FAIL; tail -20 $OUT/arena_worker.err; exit 1; }
cat $OUT/arena_worker.json
f=$(ls $OUT/arena_trace/*/run_kernel_trace.csv $OUT/arena_trace/run_kernel_trace.csv 2>/dev/null | head -1)
cp /tmp/jx_trims.log $OUT/arena_trims.log; python3 tools/stream_gaps.py $f --trims /tmp/jx_trims.log > $OUT/arena_stream_gaps.json && python3 -c "
import json; d=json.load(open('$OUT/arena_stream_gaps.json'))
for q, s in d['streams'].items(): print('stream', q, s['kernels'], 'max_gap_ms', s['max_gap_ms'], 'over_1ms', s['gaps_over_1ms'], 'over_1ms_on_trim', s.get('gaps_over_1ms_overlapping_a_trim'))"
echo ARENA_OK
