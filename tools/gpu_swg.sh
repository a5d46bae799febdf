set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTHONPATH=. timeout -k 10 200 python -u tools/swg_diag.py > gpurun_out/swg_diag.log 2>&1 || { echo "DIAG FAILED"; grep -v Warn gpurun_out/swg_diag.log | tail -20; exit 1; }
grep -v Warn gpurun_out/swg_diag.log | tail -12
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider -k "swiglu" --timeout 120 --timeout-method thread > gpurun_out/swg_tests.log 2>&1 || { echo "KTESTS FAILED"; tail -30 gpurun_out/swg_tests.log; exit 1; }
tail -2 gpurun_out/swg_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/swg_step.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/swg_step.log; exit 1; }
tail -2 gpurun_out/swg_step.log
OSPO_FUSE_SWIGLU_BWD=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/swg_bench_off.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/swg_bench_on.json 2>/dev/null || exit 1
OSPO_FUSE_SWIGLU_BWD=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/swg_bench_off2.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/swg_bench_on2.json 2>/dev/null || exit 1
for f in off on off2 on2; do python -c "import json;d=json.load(open('gpurun_out/swg_bench_$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"; done
