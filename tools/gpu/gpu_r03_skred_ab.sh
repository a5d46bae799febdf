# same-box A/B: split sum in the skinny launch (default) vs the separate reduce kernel (ablation env)
set -o pipefail
export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/skab_new_$r.json 2> gpurun_out/skab_new_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/skab_new_$r.err; exit 1; }
  OSPO_SK_REDUCE_LAUNCH=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/skab_old_$r.json 2> gpurun_out/skab_old_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/skab_old_$r.err; exit 1; }
  python -c "
import json
for t in ('new', 'old'):
    d = json.load(open('gpurun_out/skab_%s_$r.json' % t)); print(t, d['value'], d['ms_per_step'], d.get('loss_first_step'))"
done
