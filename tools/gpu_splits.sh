set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for cfg in "8,4,4,8" "4,2,2,4" "16,8,8,16"; do
  OSPO_DADB_SPLITS=$cfg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/splits_${cfg}_r$r.json 2>gpurun_out/splits.err || { echo "BENCH FAILED $cfg"; tail -5 gpurun_out/splits.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/splits_${cfg}_r$r.json'));print('splits $cfg r$r',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])" | tee -a gpurun_out/splits.log
done; done
