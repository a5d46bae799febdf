set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/sp8_tests.log 2>&1 || { tail -20 gpurun_out/sp8_tests.log; exit 1; }
tail -1 gpurun_out/sp8_tests.log
timeout -k 10 300 python tools/gemm_fixed_cost.py > gpurun_out/sp8_fixed.jsonl 2>gpurun_out/sp8_fixed.err || exit 1
cat gpurun_out/sp8_fixed.jsonl
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sp8_bench.json 2> gpurun_out/sp8_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/sp8_bench.json')); print('pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'])"
