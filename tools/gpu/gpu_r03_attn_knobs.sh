# attention ablation knobs: forward DMA spread (tests with it on, then timings), dQ kernel workgroup order
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so
OSPO_ATTN_FWD_SPREAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k "flash" > gpurun_out/aknob_tests.log 2>&1 || { echo "TESTS FAILED"; tail -20 gpurun_out/aknob_tests.log; exit 1; }
tail -1 gpurun_out/aknob_tests.log
for r in 1 2; do
  for v in base fwdspread dqorder1; do
    unset OSPO_ATTN_FWD_SPREAD OSPO_ATTN_ORDER_DQ
    [ $v = fwdspread ] && export OSPO_ATTN_FWD_SPREAD=1
    [ $v = dqorder1 ] && export OSPO_ATTN_ORDER_DQ=1
    echo "$v $r $(timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | tail -1)"
  done
done
