# cost of LoRA dropout in the step: --lora-dropout 0 vs 0.05, alternating on one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for p in 0.05 0; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --lora-dropout $p > gpurun_out/drop_${p}_${r}.json 2> gpurun_out/drop_${p}_${r}.err || { echo "BENCH FAILED $p $r"; tail -5 gpurun_out/drop_${p}_${r}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/drop_${p}_${r}.json')); print('dropout $p round $r', 'pairs/s', d['value'], 'ms', d['ms_per_step'], 'gemm us', d['roofline']['avg_launch_us'])"
  done
done
