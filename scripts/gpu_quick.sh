# GPU session: parity tests + bench variants (FLP group width) with kernel times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for ppw in ${PPW_LIST:-4 2 1}; do
  JX_PPW=$ppw timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ppw$ppw.json 2> gpurun_out/bench_ppw$ppw.err || { echo BENCH_FAIL $ppw; tail -20 gpurun_out/bench_ppw$ppw.err; exit 1; }
  echo "ppw=$ppw"; python3 -c "import json;d=json.load(open('gpurun_out/bench_ppw$ppw.json'));print(d['value'], d['verified'], d['kernels']['k1_xof_ms_per_launch'], d['kernels']['k3_flp_ms_per_launch'])"
done
