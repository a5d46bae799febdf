# split-K fixup loads in flight + MXFP8 copies from the attention stores: tests, benches, kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_step.py -q -m gpu -p no:cacheprovider -rf --timeout 400 --timeout-method thread -k "split or schedule or swiglu_bwd_fused or rope or gemm or mx8 or flash" > gpurun_out/fx_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/fx_tests.log | head -20; tail -3 gpurun_out/fx_tests.log; exit 1; }
tail -1 gpurun_out/fx_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fx_bench.json 2> gpurun_out/fx_bench.err || { echo "BENCH FAILED"; tail -5 gpurun_out/fx_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fx_bench.json')); print('bf16 pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'], 'loss', d['loss'])"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --linear-dtype mx8 > gpurun_out/fx_mx8.json 2> gpurun_out/fx_mx8.err || { echo "MX8 BENCH FAILED"; tail -5 gpurun_out/fx_mx8.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fx_mx8.json')); print('mx8 pairs/s', d['value'], 'ms', d['ms_per_step'], 'loss', d['loss'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fx_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fx_prof.json 2> gpurun_out/fx_prof.err || { echo "ROCPROF FAILED"; tail -3 gpurun_out/fx_prof.err; exit 1; }
python tools/prof_summary.py gpurun_out/fx_prof/prof_kernel_trace.csv > gpurun_out/fx_breakdown.txt && rm -f gpurun_out/fx_prof/prof_kernel_trace.csv
head -12 gpurun_out/fx_breakdown.txt
