# same-box A/B of bench.py flag sets, alternating, 2 rounds: ARGS_A / ARGS_B
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    eval "args=\$ARGS_$v"
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $args > gpurun_out/ab_${v}_$r.json 2>/dev/null || { echo "BENCH FAILED $v"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${v}_$r.json')); print('$v', '$args', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
