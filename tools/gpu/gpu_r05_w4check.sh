# Round 5: the w4 GEMM (now with the epilogue staged inside the last K-tile) against the SP8 kernel, bit-equality on
# every epilogue / extension / dropout / split-K form (tools/w4_check.py, no timing), then the attention A/B tool
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5h}
timeout -k 10 300 python -u tools/w4_check.py --no-time > gpurun_out/${TAG}_w4_check.log 2>&1 || { echo "W4 CHECK FAILED"; tail -20 gpurun_out/${TAG}_w4_check.log; exit 1; }
tail -5 gpurun_out/${TAG}_w4_check.log | cut -c1-300
