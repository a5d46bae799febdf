# full round check: GPU suite (parity log), smoke, bench (with CPU baseline), rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r}
export OSPO_PARITY_LOG=gpurun_out/${TAG}_parity.jsonl
rm -f $OSPO_PARITY_LOG
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -rf -s --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'], 'cpu', d.get('cpu_baseline', {}).get('value'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "ROCPROF FAILED"; tail -3 gpurun_out/${TAG}_prof.err; exit 1; }
echo done
