# A/B of per-layer vs per-group side-stream events; tools/_engine_prev_ab.py was `git show <prev>:ospo_amd/engine.py`
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_dp_overlap.py -q -x -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/ev_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ev_tests.log; exit 1; }
tail -1 gpurun_out/ev_tests.log
cp ospo_amd/engine.py /tmp/engine_new.py
for r in 1 2; do
  cp /tmp/engine_new.py ospo_amd/engine.py
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ev_new_$r.json 2> gpurun_out/ev_new_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/ev_new_$r.err; exit 1; }
  cp tools/_engine_prev_ab.py ospo_amd/engine.py
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ev_old_$r.json 2> gpurun_out/ev_old_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/ev_old_$r.err; exit 1; }
  python -c "
import json
for t in ('new', 'old'):
    d = json.load(open('gpurun_out/ev_%s_$r.json' % t)); print(t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss_first_step'))"
done
cp /tmp/engine_new.py ospo_amd/engine.py
