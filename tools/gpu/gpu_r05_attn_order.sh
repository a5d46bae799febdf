# Round 5, verdict r4 item 2a: workgroup orders of the attention backward (ablation library), same process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5d}
timeout -k 10 300 python -u tools/attn_order_ab.py > gpurun_out/${TAG}_attn_order.log 2>&1 || { echo "ATTN ORDER FAILED"; tail -20 gpurun_out/${TAG}_attn_order.log; exit 1; }
cut -c1-200 gpurun_out/${TAG}_attn_order.log
