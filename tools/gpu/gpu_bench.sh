set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-b}
timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { echo "BENCH FAILED rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo done
