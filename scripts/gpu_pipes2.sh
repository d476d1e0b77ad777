# Pipelines, round 2: the driver's bench command with the default 2 pipelines (+ single-stream `alone`
# steps), then configs 1-2 at 1M reports in one launch vs two / four launches over 2 pipelines.
# usage: bash scripts/gpu_pipes2.sh <name>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], d['verified'], d.get('verified_all_configs'), r['frac'], r['pipelines'], r['kernel_concurrency'], r['device_step'], r['alone'])
print({k: v['value'] for k, v in d['secondary'].items()})"
CF="tools/bench_configs.py --only sum32,hist --cpu-seconds 0.5"
timeout -k 10 300 python -u $CF > $OUT/cfg_default.jsonl 2> $OUT/cfg_default.err || { echo CFG_FAIL; tail -5 $OUT/cfg_default.err; exit 1; }
JX_CHUNK_REPORTS=524288 JX_PIPES=2 timeout -k 10 300 python -u $CF > $OUT/cfg_c512k_p2.jsonl 2> $OUT/cfg_c512k_p2.err || { echo CFG2_FAIL; tail -5 $OUT/cfg_c512k_p2.err; exit 1; }
JX_CHUNK_REPORTS=262144 JX_PIPES=2 timeout -k 10 300 python -u $CF > $OUT/cfg_c256k_p2.jsonl 2> $OUT/cfg_c256k_p2.err || { echo CFG3_FAIL; tail -5 $OUT/cfg_c256k_p2.err; exit 1; }
for f in cfg_default cfg_c512k_p2 cfg_c256k_p2; do python3 -c "
import json
for l in open('$OUT/$f.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['config']['workload'][:30], d['value'], d['kernels'], d['verified'])"; done
