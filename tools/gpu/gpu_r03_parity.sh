# Round 3: the new full-depth / bench-config / 8-pair parity tests, the two-rank gloo bench, then the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3p}
export OSPO_PARITY_LOG=gpurun_out/${TAG}_parity.jsonl
rm -f $OSPO_PARITY_LOG
( while sleep 45; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_dp_overlap.py -v -s -p no:cacheprovider --durations=0 \
  --timeout 400 --timeout-method thread -k "${PYTEST_K:-full_depth or bench_config or 8_pairs or two_ranks}" > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -30; tail -15 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -2
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json | cut -c1-600
