set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "lora_da or dropout or skinny or split" > gpurun_out/da_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/da_tests.log; exit 1; }
tail -1 gpurun_out/da_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "dropout or bench_config" > gpurun_out/da_step.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/da_step.log; exit 1; }
tail -1 gpurun_out/da_step.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/da_benchpy.json 2> gpurun_out/da_benchpy.err || { echo "BENCH.PY FAILED"; tail -20 gpurun_out/da_benchpy.err; exit 1; }
cut -c1-220 gpurun_out/da_benchpy.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/da_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/da_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/da_prof.log; exit 1; }
echo prof ok
