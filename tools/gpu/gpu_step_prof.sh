# selected GPU tests, short bench, kernel-trace breakdown of the step (TAG, PYTEST_K)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sp}
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -rf --timeout 300 --timeout-method thread -k "${PYTEST_K}" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/${TAG}_attn.json 2>&1 || { echo "ATTN BENCH FAILED"; tail -5 gpurun_out/${TAG}_attn.json; exit 1; }
cat gpurun_out/${TAG}_attn.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'], 'loss', d['loss'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "PROF FAILED"; exit 1; }
python tools/prof_summary.py $(ls gpurun_out/${TAG}_prof/*kernel_trace.csv | head -1) 5 40 > gpurun_out/${TAG}_breakdown.txt
head -30 gpurun_out/${TAG}_breakdown.txt
