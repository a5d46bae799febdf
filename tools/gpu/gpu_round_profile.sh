# Bench (with CPU baseline) + rocprofv3 kernel stats of the same command + PMC passes (traffic, MFMA busy)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-rp}
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "PROF FAILED"; exit 1; }
bash tools/gpu/gpu_pmc_bench.sh
