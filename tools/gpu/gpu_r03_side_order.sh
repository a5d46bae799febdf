# Where a layer's LoRA dA work joins the side stream: parity test, then step A/B (alternating, same box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_step.py -k "side_after_norm or dropout" > gpurun_out/side_order_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/side_order_tests.log; exit 1; }
tail -3 gpurun_out/side_order_tests.log
for r in 1 2 3; do
  for v in 0 1; do
    SIDE_AFTER_NORM=$v timeout -k 10 400 python -u tools/side_order_ab.py --no-cpu-baseline > gpurun_out/side_order_${v}_$r.json 2> gpurun_out/side_order_${v}_$r.err || { echo "AB BENCH FAILED"; tail -5 gpurun_out/side_order_${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss'))" gpurun_out/side_order_${v}_$r.json "after_norm=$v round $r"
  done
done
