# other BASELINE configs on one GPU: 8 pairs/GPU (config 3's per-GPU batch), MXFP8 at r = 16 and r = 32 (config 5)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-c}
for cfg in "--pairs-per-gpu 8" "--linear-dtype mx8 --lora-r 32" "--linear-dtype mx8"; do
  name=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $cfg > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "BENCH FAILED $cfg"; tail -3 gpurun_out/${TAG}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['achieved'], d['roofline']['frac'])"
done
