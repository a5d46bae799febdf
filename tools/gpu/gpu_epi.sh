set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "gemm" --timeout 300 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 || { grep -E "^FAILED|Error" gpurun_out/epi_tests.log | head -20; tail -5 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
GB_VARIANTS=31,0 timeout -k 10 500 python tools/gemm_bench.py > gpurun_out/epi_ab.jsonl 2> gpurun_out/epi_ab.err || exit 1
GB_RES=1 GB_VARIANTS=31,0 timeout -k 10 500 python tools/gemm_bench.py > gpurun_out/epi_ab_res.jsonl 2> gpurun_out/epi_ab_res.err || exit 1
timeout -k 10 200 python tools/gemm_phases.py > gpurun_out/phases3.jsonl 2> gpurun_out/phases3.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/epi_bench.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/epi_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
