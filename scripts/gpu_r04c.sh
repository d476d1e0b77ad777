# Round 4: the driver's bench (with the secondary configs), the K3 probe, the configs[4] priority experiment
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; grep -v rank0 $OUT/bench.err | tail -20; exit 1; }
tail -c 1500 $OUT/bench.json
timeout -k 10 400 bash tools/k3_probe.sh $OUT/k3probe || { echo PROBE_FAIL; exit 1; }
timeout -k 10 500 bash scripts/gpu_fp_prio.sh r04c/fpprio || { echo FPPRIO_FAIL; exit 1; }
