# Round 5: generate tests (the sampler rewrite: tokens bit-exact vs the oracle), then the final profiles / lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -m gpu -x -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/r5h_gen_tests.log 2>&1 || { echo "GEN TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r5h_gen_tests.log | head -20; tail -5 gpurun_out/r5h_gen_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5h_gen_tests.log | tail -1
TAG=r5f bash tools/gpu/gpu_r05_final.sh
