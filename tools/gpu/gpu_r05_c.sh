# Round 5 call C: step A/B of the kernel changes, the w4 bit-equality check, the GEMM / attention kernel tests and
# the two step tests whose loss bounds were restated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r5c2
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -v -p no:cacheprovider -rf -s --timeout 600 --timeout-method thread \
  -k "gemm or flash or attn or trajectory or bench_config or full_depth" > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -30; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash tools/gpu/gpu_r05_w4check.sh || exit 1
bash tools/gpu/gpu_r05_step_ab.sh || exit 1
