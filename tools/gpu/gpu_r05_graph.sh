# Round 5: eager training step vs the same step replayed from a hipGraph (launch-gap estimate)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/step_graph_ab.py > gpurun_out/r5graph.log 2>&1 || { echo "GRAPH AB FAILED"; tail -30 gpurun_out/r5graph.log; exit 1; }
cat gpurun_out/r5graph.log | tail -3
