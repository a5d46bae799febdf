set -o pipefail
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/swg2_b_$r.json 2> gpurun_out/swg2_b_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/swg2_b_$r.err; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --round2-lora > gpurun_out/swg2_r2_$r.json 2> gpurun_out/swg2_r2_$r.err || { echo "R2 FAILED"; tail -5 gpurun_out/swg2_r2_$r.err; exit 1; }
  python -c "
import json
for t in ('b', 'r2'):
    d = json.load(open('gpurun_out/swg2_%s_$r.json' % t)); print(t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss_first_step'))"
done
