# Round 5: the whole GPU suite (parity log) and smoke; NO_BENCH unset adds the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5s}
export OSPO_PARITY_LOG=gpurun_out/${TAG}_parity.jsonl
rm -f $OSPO_PARITY_LOG
timeout -k 10 1500 python -u -m pytest tests/ -m gpu -v -p no:cacheprovider -rf -s --durations=15 --timeout 600 \
  --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -30; tail -15 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
