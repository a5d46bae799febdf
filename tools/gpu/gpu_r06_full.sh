# Round 6: the whole GPU suite (one process), then smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6full}
export OSPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_parity.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -30; tail -15 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
PROF_ARGS="--no-box-probe" TAG=${TAG}p bash tools/gpu/gpu_r05_prof.sh > gpurun_out/${TAG}_prof_out.txt 2>&1 || { echo "PROF FAILED"; tail gpurun_out/${TAG}_prof_out.txt; exit 1; }
head -30 gpurun_out/${TAG}p_breakdown.txt
