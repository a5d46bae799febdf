# config 5 A/B: MXFP8 copies from the attention stores (new) vs the standalone quantizer (old), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in new old; do
    flag=""; [ $v = old ] && flag="--old"
    timeout -k 10 300 python tools/mx8_attn_ab.py $flag --linear-dtype mx8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/mxa_${v}_${r}.json 2> gpurun_out/mxa_${v}_${r}.err || { echo "BENCH FAILED $v $r"; tail -5 gpurun_out/mxa_${v}_${r}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/mxa_${v}_${r}.json')); print('$v round $r', 'pairs/s', d['value'], 'ms', d['ms_per_step'], 'loss', d['loss'])"
  done
done
