set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -k "gdb or step or dp_overlap or skinny or wrapper" --timeout 300 --timeout-method thread > gpurun_out/gdb_tests.log 2>&1 || { grep -E "^FAILED|Error" gpurun_out/gdb_tests.log | head -20; tail -5 gpurun_out/gdb_tests.log; exit 1; }
tail -1 gpurun_out/gdb_tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gdb_on_$r.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/gdb_on_$r.json')); print('fused', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  ABL=nogdb timeout -k 10 300 python tools/ablate_side.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gdb_off_$r.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/gdb_off_$r.json')); print('unfused', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
