# Round 6: fwd3 decomposition + stamps, then the A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6attn2}
timeout -k 10 300 python -u tools/attn_r6_ab.py --decompose > gpurun_out/${TAG}_dec.log 2>&1 || { echo "DEC FAILED"; tail -20 gpurun_out/${TAG}_dec.log; exit 1; }
cat gpurun_out/${TAG}_dec.log
timeout -k 10 300 python -u tools/attn_r6_ab.py > gpurun_out/${TAG}_ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
