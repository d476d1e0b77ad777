# Round 5: host CPU usage of the coalesced job path (native driver, 100-report SumVec jobs, 64 threads) and the
# box's cgroup CPU throttling counters around it.
set -o pipefail
N=${1:?name}
OUT=gpurun_out/$N
mkdir -p $OUT /tmp/jp
timeout -k 10 200 python -u tools/bench_jobs.py --driver cpp --mode coalesce --vdafs sumvec --sizes 10 --threads 1 --seconds 0.2 --keep-pool /tmp/jp > $OUT/prep.log 2>&1 || { echo PREP_FAIL; exit 1; }
cat /sys/fs/cgroup/cpu.stat > $OUT/cpustat_before.txt 2>/dev/null; cat /sys/fs/cgroup/cpu.max > $OUT/cpumax.txt 2>/dev/null
python3 -c "
import resource, subprocess, sys, time
t = time.time()
r = subprocess.run(sys.argv[1:], stdout=open('$OUT/driver_cpu.json', 'w'), timeout=100)
u = resource.getrusage(resource.RUSAGE_CHILDREN)
print('wall %.2f s user %.2f s sys %.2f s vol_cs %d invol_cs %d rc %d' % (time.time() - t, u.ru_utime, u.ru_stime, u.ru_nvcsw, u.ru_nivcsw, r.returncode))
sys.exit(r.returncode)" tools/bin/jobs_driver /tmp/jp/pool_2_2048.bin /tmp/jp/out.bin 2 8 1000 88 1 000102030405060708090a0b0c0d0e0f ${2:-100} ${3:-64} 2 1 0 1 > $OUT/driver_time.txt 2>&1 || { echo DRIVER_FAIL; tail -5 $OUT/driver_time.txt; exit 1; }
cat /sys/fs/cgroup/cpu.stat > $OUT/cpustat_after.txt 2>/dev/null
cat $OUT/driver_cpu.json; cat $OUT/driver_time.txt; paste $OUT/cpustat_before.txt $OUT/cpustat_after.txt; cat $OUT/cpumax.txt
echo CPU_OK
