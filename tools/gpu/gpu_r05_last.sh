# Round 5 last check after the per-step counter resets: smoke, a step parity test, the generate tests, default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5v}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_generate.py -m gpu -x -v -p no:cacheprovider -rf --timeout 400 --timeout-method thread -k "bench_config_first_step or 8_pairs or trajectory or generate or decode" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.json
