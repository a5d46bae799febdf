set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-v14}
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "PROF FAILED"; exit 1; }
timeout -k 10 300 python bench.py --linear-dtype mx8 --lora-r 32 --no-cpu-baseline > gpurun_out/${TAG}_bench_mx8_r32.json 2>/dev/null || { echo "MX8 FAILED"; exit 1; }
timeout -k 10 300 python bench.py --linear-dtype mx8 --no-cpu-baseline > gpurun_out/${TAG}_bench_mx8_r16.json 2>/dev/null || { echo "MX8 FAILED"; exit 1; }
for f in bench prof bench_mx8_r32 bench_mx8_r16; do python -c "import json;d=json.load(open('gpurun_out/${TAG}_$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['avg_launch_us'],d.get('cpu_baseline',{}).get('value'))"; done
