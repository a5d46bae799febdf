set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for V in 1 0; do
  for SET in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY" "FETCH_SIZE" ; do
    tag=$(echo $SET | cut -d' ' -f1)
    GO_VARIANT=$V timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/pmc/v${V}_${tag} -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc/err.log || echo "fail $V $tag" >> gpurun_out/pmc/err.log
  done
done
GO_BLAS=1 GO_ITERS=20 timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc/blas_TCC -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc/err.log || true
GO_BLAS=1 timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/blas_SQ -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc/err.log || true
echo done
