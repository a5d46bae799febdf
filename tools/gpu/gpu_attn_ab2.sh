# attention tests + dK/dV A/B (ABVAR) + stamps
set -o pipefail
mkdir -p gpurun_out/attn_ab
export TMPDIR=/tmp
ABVAR=${ABVAR:-OSPO_ATTN_DKDV_R2}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "flash" -m gpu > gpurun_out/attn_ab/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/attn_ab/tests.log | head; tail -3 gpurun_out/attn_ab/tests.log; exit 1; }
tail -1 gpurun_out/attn_ab/tests.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py 2>/dev/null || { echo "FAILED A"; exit 1; }
  env $ABVAR=1 timeout -k 10 120 python tools/attn_bench.py 2>/dev/null || { echo "FAILED B"; exit 1; }
done
timeout -k 10 120 python tools/attn_stamps.py || { echo "STAMPS FAILED"; exit 1; }
