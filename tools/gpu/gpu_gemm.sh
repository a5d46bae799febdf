set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k gemm > gpurun_out/gemm_tests.log 2>&1; echo "EXIT=$?" >> gpurun_out/gemm_tests.log
grep -q "EXIT=0" gpurun_out/gemm_tests.log || exit 1
timeout -k 10 400 python tools/gemm_bench.py > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err
