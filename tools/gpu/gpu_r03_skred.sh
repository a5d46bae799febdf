set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "skinny or swiglu or keep_bits or lora_da" > gpurun_out/skr_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/skr_tests.log; exit 1; }
tail -1 gpurun_out/skr_tests.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "dropout or bench_config or 7b_shapes" > gpurun_out/skr_step.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/skr_step.log; exit 1; }
tail -1 gpurun_out/skr_step.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/skr_b1.json 2> gpurun_out/skr_b1.err || { echo "BENCH FAILED"; tail -5 gpurun_out/skr_b1.err; exit 1; }
cut -c1-200 gpurun_out/skr_b1.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/skr_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/skr_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/skr_prof.log; exit 1; }
echo prof ok
