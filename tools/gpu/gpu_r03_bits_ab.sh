set -o pipefail
# same-box A/B of the round-3 LoRA path (dA stream + keep bits) against round 2's (dA tiles, re-hashed masks)
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_r3_$r.json 2> gpurun_out/ab_r3_$r.err || { echo "R3 FAILED"; tail -5 gpurun_out/ab_r3_$r.err; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --round2-lora > gpurun_out/ab_r2_$r.json 2> gpurun_out/ab_r2_$r.err || { echo "R2 FAILED"; tail -5 gpurun_out/ab_r2_$r.err; exit 1; }
  python -c "
import json
for t in ('r3', 'r2'):
    d = json.load(open('gpurun_out/ab_%s_$r.json' % t)); print(t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
