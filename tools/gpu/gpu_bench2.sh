# same-box A/B of the bench: dropout 0.05 (throughput config, the default) vs 0 (parity config)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_drop.json 2> gpurun_out/${TAG}_drop.err || { echo "BENCH FAILED"; tail gpurun_out/${TAG}_drop.err; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --lora-dropout 0 > gpurun_out/${TAG}_nodrop.json 2> gpurun_out/${TAG}_nodrop.err || { echo "BENCH FAILED"; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_drop2.json 2> gpurun_out/${TAG}_drop2.err || { echo "BENCH FAILED"; exit 1; }
echo done
