set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -rf -k "attention or skinny or lora_pack" > gpurun_out/attn_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/attn_tests.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_step.py -q -m gpu -p no:cacheprovider -rf >> gpurun_out/attn_tests.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/a_prof.json 2> gpurun_out/a_prof.err
echo done
GB_VARIANTS=0,1,5 timeout -k 10 400 python tools/gemm_bench.py > gpurun_out/gemm_bench5.jsonl 2> gpurun_out/gemm_bench5.err
echo gemm done
