# GPU suite with the parity log, then smoke (round 2)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r}
export OSPO_PARITY_LOG=gpurun_out/${TAG}_parity.jsonl
rm -f $OSPO_PARITY_LOG
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -rf -s --timeout 400 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" gpurun_out/${TAG}_tests.log | head -30; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -3 gpurun_out/${TAG}_smoke.log
