# Round 6: fwd3 / fwd4 (software-pipelined) / fwd2 A/B at the step shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6fwd4}
timeout -k 10 300 python -u tools/attn_r6_ab.py > gpurun_out/${TAG}_ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
