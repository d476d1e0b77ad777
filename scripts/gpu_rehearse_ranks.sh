# The N>1 bench path rehearsed on one GPU (--share-gpu: every rank on cuda:0, shard records over gloo):
# world 2 and world 4, each rank a different global report range, every rank's aggregate and the merged
# record verified against the pool's block aggregates. Not a scaling measurement (the ranks share one GPU).
# usage: bash scripts/gpu_rehearse_ranks.sh <name>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?name}
mkdir -p $OUT
for W in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$W --master-addr 127.0.0.1 --master-port $((29500 + W)) \
    bench.py --gpus $W --share-gpu --reports-per-gpu 262144 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary \
    > $OUT/world$W.json 2> $OUT/world$W.err || { echo WORLD${W}_FAIL; grep -v "^\[rank" $OUT/world$W.err | tail -20; exit 1; }
  tail -c 300 $OUT/world$W.json
done
