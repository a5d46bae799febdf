set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_step.py tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -rf -s > gpurun_out/t2.log 2>&1 || { echo "TESTS FAILED rc=$?" >> gpurun_out/t2.log; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo "BENCH FAILED rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1_prof.json 2> gpurun_out/prof1.err
echo done
