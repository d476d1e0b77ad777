# Keccak permutation rate vs waves/SIMD and states/lane (tools/microbench_keccak.hip), and where K1's
# issue cycles go: SQ stall counters over a one-launch SumVec bench and over the microbenchmark.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03h
mkdir -p $OUT
timeout -k 10 120 ./tools/bin/microbench_keccak 400 > $OUT/keccak.jsonl 2> $OUT/keccak.err || { echo MB_FAIL; tail -5 $OUT/keccak.err; exit 1; }
cat $OUT/keccak.jsonl
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
BENCH="bench.py --steps 1 --warmup 0 --reports-per-gpu 262144 --pool 512 --no-cpu-baseline --no-dist"
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc_k1 -o run -- python3 $BENCH > $OUT/pmc_k1.json 2> $OUT/pmc_k1.err || { echo PMC_K1_FAIL; tail -5 $OUT/pmc_k1.err; exit 1; }
timeout -s KILL 100 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc_mb -o run -- ./tools/bin/microbench_keccak 200 > $OUT/pmc_mb.jsonl 2> $OUT/pmc_mb.err || { echo PMC_MB_FAIL; tail -5 $OUT/pmc_mb.err; exit 1; }
echo DONE
