# Round 5, verdict r4 item 1: the w4 split-K tail model on config 3's per-GPU shapes (M = 9600)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5e}
SWEEP_M=9600 timeout -k 10 400 python -u tools/w4_split_sweep.py > gpurun_out/${TAG}_split9600.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/${TAG}_split9600.log; exit 1; }
cut -c1-300 gpurun_out/${TAG}_split9600.log
