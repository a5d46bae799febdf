# attention backward A/B: 8-wave vs 4-wave dK/dV workgroups (ablation build), + kernel stats, + attention tests
set -o pipefail
mkdir -p gpurun_out/attn_w
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "flash" -m gpu > gpurun_out/attn_w/tests.log 2>&1 || { echo "TESTS FAILED"; tail -20 gpurun_out/attn_w/tests.log; exit 1; }
tail -2 gpurun_out/attn_w/tests.log
for w in 8 4 8 4; do
  OSPO_ATTN_WAVES=$w timeout -k 10 120 python tools/attn_bench.py 2>/dev/null || { echo "FAILED w=$w"; exit 1; }
done
for w in 8 4; do
  OSPO_ATTN_WAVES=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_w/prof$w -o p -- python tools/attn_bench.py > gpurun_out/attn_w/prof$w.log 2>&1 || { echo "PROF FAILED $w"; exit 1; }
done
echo done
