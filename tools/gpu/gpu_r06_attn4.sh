# Round 6: attention kernel tests (default path = attn_fwd3 + attn_bwd_dkdv5), then the fwd/bwd A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6attn5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx8.py -k "flash or attention" -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -30; tail -25 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u tools/attn_r6_ab.py > gpurun_out/${TAG}_ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
