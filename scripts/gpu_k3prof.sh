# Kernel-level times of the two K3 paths (MFMA wire sums vs VALU ring) on a one-launch SumVec bench,
# plus SQ counters for the MFMA kernel
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k3prof}
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --reports-per-gpu 262144 --pool 1024 --no-cpu-baseline --no-dist"
for m in 1 0; do
  JX_K3_MFMA=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$m -o run -- python3 $BENCH > $OUT/b$m.json 2> $OUT/b$m.err || { echo TRACE_FAIL $m; tail -5 $OUT/b$m.err; exit 1; }
  python3 - $OUT/trace$m/run_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), "ms")
PY
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc -o run -- python3 $BENCH > $OUT/pmc.json 2> $OUT/pmc.err || { echo PMC_FAIL; tail -5 $OUT/pmc.err; exit 1; }
echo DONE
