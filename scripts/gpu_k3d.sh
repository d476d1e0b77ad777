# MFMA K3 ring depth 3/4/6 kernel times + SQ counters at depth 6
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k3d}
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --reports-per-gpu 262144 --pool 1024 --no-cpu-baseline --no-dist"
for d in 3 4 6; do
  JX_MF_D=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace$d -o run -- python3 $BENCH > $OUT/b$d.json 2> $OUT/b$d.err || { echo TRACE_FAIL; tail -5 $OUT/b$d.err; exit 1; }
  python3 - $OUT/trace$d/run_kernel_stats.csv $d <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]:
    if 'mfma' in r['Name'] or 'wires' in r['Name']: print("  D=%s"%sys.argv[2], r['Name'][:50], round(float(r['AverageNs'])/1e6,3), "ms")
PY
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
JX_MF_D=6 timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $OUT/pmc -o run -- python3 $BENCH > $OUT/pmc.json 2> $OUT/pmc.err || { echo PMC_FAIL; tail -5 $OUT/pmc.err; exit 1; }
SQ2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
JX_MF_D=6 timeout -s KILL 200 rocprofv3 --pmc $SQ2 -f csv -d $OUT/pmc2 -o run -- python3 $BENCH > $OUT/pmc2.json 2> $OUT/pmc2.err || { echo PMC2_FAIL; tail -5 $OUT/pmc2.err; }
echo DONE
