set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "swiglu" > gpurun_out/vab_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/vab_tests.log; exit 1; }
tail -1 gpurun_out/vab_tests.log
for r in 1 2; do
  for v in base swiglu_u da_stream; do
    if [ $v = base ]; then X=; else X="--lora-variant $v"; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $X > gpurun_out/vab_${v}_$r.json 2> gpurun_out/vab_${v}_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/vab_${v}_$r.err; exit 1; }
  done
  python -c "
import json
for t in ('base', 'swiglu_u', 'da_stream'):
    d = json.load(open('gpurun_out/vab_%s_$r.json' % t)); print(t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss_first_step'))"
done
