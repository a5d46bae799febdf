set -o pipefail
mkdir -p gpurun_out
python -c "import torch;print('prio range', torch.cuda.Stream.priority_range())" > gpurun_out/prio.log 2>&1 || true
for r in 1 2; do
for cfg in "0 0" "-1 0" "0 -1"; do
  set -- $cfg
  OSPO_MAIN_PRIO=$1 OSPO_SIDE_PRIO=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prio_m$1_s$2_r$r.json 2>/dev/null || { echo "BENCH FAILED $cfg"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/prio_m$1_s$2_r$r.json'));print('main',$1,'side',$2,'r$r',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])" | tee -a gpurun_out/prio.log
done; done
