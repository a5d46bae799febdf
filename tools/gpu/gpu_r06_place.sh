# Round 6: fwd3 DMA placement A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6place}
timeout -k 10 300 python -u tools/attn_r6_ab.py --place > gpurun_out/${TAG}.log 2>&1 || { echo "PLACE FAILED"; tail -20 gpurun_out/${TAG}.log; exit 1; }
cat gpurun_out/${TAG}.log
