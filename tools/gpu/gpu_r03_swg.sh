set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "swiglu or skinny or lora_da or keep_bits" > gpurun_out/swg_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/swg_tests.log; exit 1; }
tail -1 gpurun_out/swg_tests.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "dropout or bench_config or 7b_shapes_2" > gpurun_out/swg_step.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/swg_step.log; exit 1; }
tail -1 gpurun_out/swg_step.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/swg2_b_$r.json 2> gpurun_out/swg2_b_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/swg2_b_$r.err; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --round2-lora > gpurun_out/swg2_r2_$r.json 2> gpurun_out/swg2_r2_$r.err || { echo "R2 FAILED"; tail -5 gpurun_out/swg2_r2_$r.err; exit 1; }
  python -c "
import json
for t in ('b', 'r2'):
    d = json.load(open('gpurun_out/swg2_%s_$r.json' % t)); print(t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss_first_step'))"
done
