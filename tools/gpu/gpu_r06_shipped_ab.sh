# Round 6: the reference's shipped config (16 pairs, LoRA r = 32, bf16) with the rank-32 fused g / dB streams on
# (default) and off (--lora-variant gdb_unfused), alternating on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6ship}
for v in on off on off; do
  if [ $v = on ]; then LV=""; else LV="gdb_unfused"; fi
  timeout -k 10 400 python -u bench.py --pairs-per-gpu 16 --lora-r 32 --steps 5 --warmup 2 --no-cpu-baseline --no-wrapper --lora-variant "$LV" \
    > gpurun_out/${TAG}_${v}.json 2> gpurun_out/${TAG}_${v}.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/${TAG}_${v}.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_${v}.json').read().splitlines()[-1]); print('shipped r32 fusion=$v', d['value'], d['ms_per_step'], d.get('box_probe',{}).get('tflops'))" | tee -a gpurun_out/${TAG}_ab.txt
done
