# A/B of the side-stream dA placement (engine da_under_gemm), alternating on one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --da-under-gemm $v > gpurun_out/da_${v}_${r}.json 2> gpurun_out/da_${v}_${r}.err || { echo "BENCH FAILED $v $r"; tail -5 gpurun_out/da_${v}_${r}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/da_${v}_${r}.json')); print('da_under_gemm=$v round $r', 'pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'], 'loss', d['loss'])"
  done
done
