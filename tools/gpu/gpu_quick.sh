# focused GPU check: selected tests, attention microbench, short bench (args: TAG, PYTEST_K)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-q}
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -rf -s --timeout 300 --timeout-method thread -k "${PYTEST_K}" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/${TAG}_attn.json 2>&1 || { echo "ATTN BENCH FAILED"; tail -5 gpurun_out/${TAG}_attn.json; exit 1; }
cat gpurun_out/${TAG}_attn.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'], 'loss', d['loss'])"
