# attention tests + variants (default, OSPO_ATTN_ORDER=1, OSPO_ATTN_ORDER=0, R2 dK/dV) + stamps
set -o pipefail
mkdir -p gpurun_out/attn_ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "flash" -m gpu > gpurun_out/attn_ab/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/attn_ab/tests.log | head; tail -3 gpurun_out/attn_ab/tests.log; exit 1; }
tail -1 gpurun_out/attn_ab/tests.log
for i in 1 2; do
  echo "default $(timeout -k 10 120 python tools/attn_bench.py 2>/dev/null)" || exit 1
  echo "order1 $(OSPO_ATTN_ORDER=1 timeout -k 10 120 python tools/attn_bench.py 2>/dev/null)" || exit 1
  echo "order0 $(OSPO_ATTN_ORDER=0 timeout -k 10 120 python tools/attn_bench.py 2>/dev/null)" || exit 1
  echo "r2 $(OSPO_ATTN_DKDV_R2=1 OSPO_ATTN_DQ_2SLOT=1 timeout -k 10 120 python tools/attn_bench.py 2>/dev/null)" || exit 1
done
timeout -k 10 120 python tools/attn_stamps.py || { echo "STAMPS FAILED"; exit 1; }
