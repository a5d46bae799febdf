# the non-default bench lines: drop-in wrapper path (ids / inline VQ), T2I generation with decode
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-l}
timeout -k 10 300 python bench.py --workload wrapper --steps 10 --warmup 3 > gpurun_out/${TAG}_wrapper.json 2> gpurun_out/${TAG}_wrapper.err || { echo "WRAPPER FAILED"; tail -5 gpurun_out/${TAG}_wrapper.err; exit 1; }
cat gpurun_out/${TAG}_wrapper.json
timeout -k 10 300 python bench.py --workload wrapper --inline-vq --steps 10 --warmup 3 > gpurun_out/${TAG}_wrapper_vq.json 2> gpurun_out/${TAG}_wrapper_vq.err || { echo "WRAPPER VQ FAILED"; tail -5 gpurun_out/${TAG}_wrapper_vq.err; exit 1; }
cat gpurun_out/${TAG}_wrapper_vq.json
timeout -k 10 400 python bench.py --workload t2i --steps 2 --warmup 1 > gpurun_out/${TAG}_t2i.json 2> gpurun_out/${TAG}_t2i.err || { echo "T2I FAILED"; tail -5 gpurun_out/${TAG}_t2i.err; exit 1; }
cat gpurun_out/${TAG}_t2i.json
