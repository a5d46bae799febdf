set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -rf -k "${TK:-skinny or gemm}" > gpurun_out/exp_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/exp_tests.log; exit 1; }
timeout -k 10 120 python tools/skinny_bench.py > gpurun_out/skinny.jsonl 2> gpurun_out/skinny.err || { echo SKINNY FAILED; tail gpurun_out/skinny.err; exit 1; }
GB_VARIANTS=${GBV:-0,1,6,7} timeout -k 10 500 python tools/gemm_bench.py > gpurun_out/gemm_bench_exp.jsonl 2> gpurun_out/gemm_bench_exp.err || { echo GEMM FAILED; tail gpurun_out/gemm_bench_exp.err; exit 1; }
echo done
