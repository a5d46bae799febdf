set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "lora_da or lora_wgrad or f32acc or skinny" > gpurun_out/da_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/da_tests.log; exit 1; }
tail -1 gpurun_out/da_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "dropout or bench_config" > gpurun_out/da_step.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/da_step.log; exit 1; }
tail -1 gpurun_out/da_step.log
timeout -k 10 300 python -u tools/lora_da_bench.py > gpurun_out/da_bench_drop.jsonl 2> gpurun_out/da_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/da_bench.err; exit 1; }
grep per_layer gpurun_out/da_bench_drop.jsonl
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/da_benchpy.json 2> gpurun_out/da_benchpy.err || { echo "BENCH.PY FAILED"; tail -20 gpurun_out/da_benchpy.err; exit 1; }
cut -c1-220 gpurun_out/da_benchpy.json
